#!/bin/bash
# r03: LD ablations (results invalid by design): EXPT 1 no epilogue, 9 + k-slice 0 every step,
# 17 + rows 0..383 for every tile; the 256x256 kernel without epilogue (build_old1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp VCFX_BENCH_ABLATION=1
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('avg_launch_ms'), r.get('frac'), (d.get('output_check') or {}).get('match'))" 2>/dev/null
    tail -1 "gpurun_out/$name.log" | cut -c1-200
    return $rc
}
B="--workload ld --no-cpu-baseline --no-e2e --steps 3 --warmup 1"
for i in 1 2; do
for v in 1 9 17; do
    VCFXG_GPU_LIB=build_v$v/libvcfx_gpu.so step expt_${v}_$i 300 python -u bench.py $B || exit $?
done
VCFXG_GPU_LIB=build_old1/libvcfx_gpu.so step expt_old1_$i 300 python -u bench.py $B || exit $?
step full_$i 300 python -u bench.py $B || exit $?
done
echo "=== done"
