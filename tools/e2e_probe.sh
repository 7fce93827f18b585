#!/bin/bash
# End-to-end probe (measurement tool): AF on the 427,409 x 2,504 shard written to /tmp --
# the pipe ceiling (`cat F | drain`), a fresh process per run (file and pipe), and the
# in-process warm-context phase breakdown (VCFX_TIMING=1).  Output under gpurun_out/.
#   bash tools/e2e_probe.sh [all|pipe|warm|bgzf]     pipe: the ceiling and the pipe runs only; bgzf: the
#   BGZF copy (fresh process and warm context)
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
MODE=${1:-all}
if [ $MODE = bgzf ]; then  # the BGZF copy: fresh process and warm context, phase breakdowns
    G=/tmp/e2e_chr21.vcf.gz
    build/bin/vcfx_bgzf $F $G 16 1 || exit 1
    ls -l $G
    cat $G > /dev/null
    for i in 1 2 3; do
        echo -n "fresh_bgzf "; time (VCFX_TIMING=$((i == 1)) timeout -k 5 60 $AF -q -i $G > /dev/null) || exit 1
    done
    VCFX_TIMING=1 timeout -k 5 120 python tools/e2e_warm.py $G || exit 1
    rm -f $F $G
    exit 0
fi
if [ $MODE = warm ]; then  # warm-context file ring shapes: slot bytes, slots, reader threads
    for i in 1 2; do
        timeout -k 5 120 python tools/e2e_warm.py $F 2>/dev/null || exit 1
        timeout -k 5 120 python tools/e2e_warm.py --torch $F 2>/dev/null || exit 1
    done
    for cfg in "16777216 12 8" "16777216 20 8" "16777216 24 12" "8388608 32 16" "16777216 32 16" "33554432 16 8"; do
        set -- $cfg
        echo "ring slot=$1 slots=$2 threads=$3"
        VCFX_FILE_SLOT=$1 VCFX_FILE_SLOTS=$2 VCFX_FILE_THREADS=$3 VCFX_TIMING=1 timeout -k 5 120 python tools/e2e_warm.py $F 2>&1 | \
            grep -E "^--- run|start|streamed|released" | tail -6 || exit 1
    done
    rm -f $F
    exit 0
fi
for i in 1 2 3; do
    [ $MODE = pipe ] && break
    echo -n "fresh_file "; time (VCFX_TIMING=$((i == 1)) timeout -k 5 60 $AF -q -i $F > /dev/null) || exit 1
done
for cfg in "1048576 16" "2097152 8" "524288 32" "1048576 8"; do
    set -- $cfg
    echo -n "cat_pipe_drain_ring $1x$2 "; time (cat $F | $DRAIN $1 $2)
    echo -n "fresh_pipe ring $1x$2 "
    time (cat $F | VCFX_RING_SLOT=$1 VCFX_RING_SLOTS=$2 VCFX_TIMING=1 timeout -k 5 60 $AF -q 2>&1 > /dev/null | grep "streamed") || exit 1
done
for i in 1 2 3; do
    echo -n "fresh_pipe "; time (cat $F | VCFX_TIMING=$((i == 1)) timeout -k 5 60 $AF -q > /dev/null) || exit 1
    echo -n "cat_pipe_drain_ring 1048576x16 "; time (cat $F | $DRAIN 1048576 16)
done
[ $MODE = pipe ] && { rm -f $F; exit 0; }
echo -n "fresh_file_mapped "; time (VCFX_FILE_STREAM=0 timeout -k 5 60 $AF -q -i $F > /dev/null) || exit 1
VCFX_TIMING=1 timeout -k 5 120 python tools/e2e_warm.py $F || exit 1
# ring shapes (warm context, the last of three runs each)
for cfg in "16777216 12" "16777216 8" "8388608 16" "33554432 8" "16777216 20"; do
    set -- $cfg
    echo "ring slot=$1 slots=$2"
    VCFX_FILE_SLOT=$1 VCFX_FILE_SLOTS=$2 VCFX_TIMING=1 timeout -k 5 120 python tools/e2e_warm.py $F 2>&1 | \
        grep -E "^--- run 2|start|streamed|released" | tail -3 || exit 1
done
for cfg in "16777216 12" "8388608 8"; do
    set -- $cfg
    echo -n "fresh_file slot=$1 slots=$2 "; time (VCFX_FILE_SLOT=$1 VCFX_FILE_SLOTS=$2 timeout -k 5 60 $AF -q -i $F > /dev/null) || exit 1
done
rm -f $F
