# e2e wall-clock probe of the drop-in binaries on a page-cache-warm synthetic file (measurement
# tool): file path, `< file`, a pipe, and the phase breakdown (VCFX_TIMING=1)
set -e
mkdir -p gpurun_out
F=/tmp/synth427k.vcf
build/bin/vcfx_synth $F 427409 2504
cat $F > /dev/null
AF=build/src/VCFX_allele_freq_calc/VCFX_allele_freq_calc
RF=build/src/VCFX_record_filter/VCFX_record_filter
GQ=build/src/VCFX_genotype_query/VCFX_genotype_query
TIMEFORMAT="%R s wall  %U user  %S sys"
{
for i in 1 2 3; do echo -n "af_file: "; { time timeout -k 10 120 $AF -q -i $F > /dev/null; } 2>&1; done
VCFX_TIMING=1 timeout -k 10 120 $AF -q -i $F 2>&1 > /dev/null
for i in 1 2; do echo -n "af_stdin_redirect: "; { time timeout -k 10 120 $AF -q < $F > /dev/null; } 2>&1; done
for i in 1 2; do echo -n "af_stdin_pipe: "; { time (cat $F | timeout -k 10 120 $AF -q > /dev/null); } 2>&1; done
cat $F | VCFX_TIMING=1 timeout -k 10 120 $AF -q 2>&1 > /dev/null
echo -n "cat_to_devnull_pipe: "; { time (cat $F | cat > /dev/null); } 2>&1
echo -n "af_tiny: "; head -c 100000 $F > /tmp/tiny.vcf; { time timeout -k 10 120 $AF -q -i /tmp/tiny.vcf > /dev/null; } 2>&1
echo -n "rf_file_devnull: "; { time timeout -k 10 120 $RF --filter "QUAL>=30;FILTER==PASS" -i $F > /dev/null; } 2>&1
echo -n "rf_gq_pipe_devnull: "; { time (timeout -k 10 120 $RF --filter "QUAL>=30;FILTER==PASS" -i $F | timeout -k 10 120 $GQ -g "0|1" > /dev/null); } 2>&1
timeout -k 10 120 $RF --filter "QUAL>=30;FILTER==PASS" -i $F | VCFX_TIMING=1 timeout -k 10 120 $GQ -g "0|1" 2>&1 > /dev/null
echo -n "rf_file_to_file: "; { time timeout -k 10 120 $RF --filter "QUAL>=30;FILTER==PASS" -i $F > /tmp/rf_out.vcf; } 2>&1
} | tee gpurun_out/e2e_probe.txt
rm -f $F /tmp/rf_out.vcf /tmp/tiny.vcf
