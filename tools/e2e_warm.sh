F=/tmp/synth427k.vcf
build/bin/vcfx_synth $F 427409 2504 && cat $F > /dev/null
VCFX_TIMING=1 timeout -k 10 120 python tools/e2e_warm.py $F 2>&1 | tee gpurun_out/e2e_warm.txt
rm -f $F
