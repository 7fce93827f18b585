#!/bin/bash
# r03 (session 3): k_fq_finish at a minimum of 4 / 5 waves per SIMD (build_fin4 / build_fin5,
# a few spills) against the compiler's choice (3 waves/SIMD, 142 VGPRs) -- parity, A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), round(r.get('avg_launch_ms') or 0,4), (d.get('output_check') or {}).get('match'), {k: round(v,3) for k,v in d.get('kernels_ms').items()})" 2>/dev/null
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
for L in build_fin4 build_fin5; do
    VCFXG_GPU_LIB=$L/libvcfx_gpu.so step t_$L 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fq_walk.py tests/test_gpu_rf.py tests/test_gpu_gq.py tests/test_legacy_api.py || exit $?
done
B="--no-cpu-baseline --no-e2e --steps 20 --warmup 3"
for i in 1 2 3; do
    step pipe_$i 300 python -u bench.py --workload pipeline $B || exit $?
    VCFXG_GPU_LIB=build_fin4/libvcfx_gpu.so step pipe_fin4_$i 300 python -u bench.py --workload pipeline $B || exit $?
    VCFXG_GPU_LIB=build_fin5/libvcfx_gpu.so step pipe_fin5_$i 300 python -u bench.py --workload pipeline $B || exit $?
done
echo "=== done"
