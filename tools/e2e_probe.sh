#!/bin/bash
# End-to-end probe (measurement tool): AF on the 427,409 x 2,504 shard written to /tmp --
# the pipe ceiling (`cat F | drain`), a fresh process per run (file and pipe), and the
# in-process warm-context phase breakdown (VCFX_TIMING=1).  Output under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
F=/tmp/e2e_chr21.vcf
python -c "
from vcfx_amd import synth
synth.generate_array(427409, 2504, seed=20251226).tofile('$F')" || exit 1
ls -l $F
cat $F > /dev/null
AF=build/src/VCFX_allele_freq_calc/VCFX_allele_freq_calc
DRAIN=build/bin/vcfx_drain
TIMEFORMAT="%R s"
for i in 1 2 3; do
    echo -n "cat_pipe_cat "; time (cat $F | cat > /dev/null)
    [ -x $DRAIN ] && { echo -n "cat_pipe_drain "; time (cat $F | $DRAIN); }
done
for i in 1 2 3; do
    echo -n "fresh_file "; time (VCFX_TIMING=$((i == 1)) timeout -k 5 60 $AF -q -i $F > /dev/null) || exit 1
done
for i in 1 2 3; do
    echo -n "fresh_pipe "; time (cat $F | VCFX_TIMING=$((i == 1)) timeout -k 5 60 $AF -q > /dev/null) || exit 1
done
echo -n "fresh_file_mapped "; time (VCFX_FILE_STREAM=0 timeout -k 5 60 $AF -q -i $F > /dev/null) || exit 1
VCFX_TIMING=1 timeout -k 5 120 python tools/e2e_warm.py $F || exit 1
rm -f $F
