#!/bin/bash
# per-invocation start-up: where the drop-in's first ~0.3 s go
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/latency.txt
: > $out
timeout -k 5 60 python - <<'PY' || exit 1
from vcfx_amd import synth
open("/tmp/small.vcf", "wb").write(synth.generate(100, 2504, 5))
PY
echo "== hip_open probe" >> $out
timeout -k 5 60 tools/microbench/hip_open >> $out 2>&1 || exit 1
for v in "" "HIP_ENABLE_DEFERRED_LOADING=0" "HIP_ENABLE_DEFERRED_LOADING=1"; do
    for i in 1 2 3; do
        echo "== af small $v run $i" >> $out
        s=$(date +%s%N)
        env $v VCFX_TIMING=1 timeout -k 5 60 build/src/VCFX_allele_freq_calc/VCFX_allele_freq_calc -q -i /tmp/small.vcf > /dev/null 2>> $out || exit 1
        e=$(date +%s%N)
        echo "wall $(( (e - s) / 1000000 )) ms" >> $out
    done
done
echo "== reference" >> $out
for i in 1 2 3; do s=$(date +%s%N); oracle/_ref/VCFX_allele_freq_calc -q -i /tmp/small.vcf > /dev/null; e=$(date +%s%N); echo "ref wall $(( (e - s) / 1000000 )) ms" >> $out; done
cat $out
echo "== runtime start-up without / with the engine's fat binary" >> $out
for b in plain vcfx plain vcfx; do timeout -k 5 60 tools/microbench/hip_init_$b >> $out 2>&1 || exit 1; done
cat $out | tail -20
