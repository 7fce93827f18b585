# Phases of the AF drop-in on the bench shard's BGZF form (measurement tool): the file made once,
# then warm in-process runs (tools/e2e_warm.py) under each setting of VCFX_BGZF_BATCH_MIN given
# (0 = no batches: every member launched at the end) and two fresh processes, VCFX_TIMING=1.
#   bash tools/e2e_bgzf_phases.sh [OUT_DIR] [BATCH_MIN...]
set -e
cd $GRAFT_REPO_ROOT
out=${1:-gpurun_out/e2e_bgzf}
shift || true
mkdir -p $out
f=/tmp/vcfx_e2e_$$.vcf
python3 -c "
from vcfx_amd import synth
synth.generate_array(n_records=427409, n_samples=2504, seed=20251226).tofile('$f')"
build/bin/vcfx_bgzf $f $f.gz 16 1
rm -f $f
for b in ${@:-16384}; do
    if [ "$b" = 0 ]; then e="VCFX_BGZF_BATCH=0"; else e="VCFX_BGZF_BATCH_MIN=$b"; fi
    env $e VCFX_TIMING=1 timeout -k 10 120 python3 -u tools/e2e_warm.py $f.gz VCFX_allele_freq_calc -q > $out/warm_$b.txt 2>&1
    echo "batch_min $b: $(tail -1 $out/warm_$b.txt)"
done
for i in 1 2 3; do
    env ${FRESH_ENV:-VCFX_TIMING=1} VCFX_TIMING=1 timeout -k 10 120 build/src/VCFX_allele_freq_calc/VCFX_allele_freq_calc -q -i $f.gz > /dev/null 2> $out/fresh$i.txt
    echo "fresh $i: $(grep -h 'tool done' $out/fresh$i.txt)"
done
rm -f $f.gz
