#!/bin/bash
# r03: deferred profiling harvest + dominant-kernel-only events in the timed loop: the AF step
# against the r03 base build; GT-first fast step A/B (build_gf) on GT:AD:DP; engine tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
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
    tail -1 "gpurun_out/$name.log" | cut -c1-200
    return $rc
}

B="--no-cpu-baseline --no-e2e --steps 20 --warmup 3"
for i in 1 2; do
    step af_$i 300 python -u bench.py $B || exit $?
    VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step af_base_$i 300 python -u bench.py $B || exit $?
done
step ld 300 python -u bench.py --workload ld --no-cpu-baseline --no-e2e || exit $?
for i in 1 2; do
    step gtadp_$i 300 python -u bench.py --format gt:ad:dp --no-cpu-baseline --no-e2e --steps 5 --warmup 2 || exit $?
    VCFXG_GPU_LIB=build_gf/libvcfx_gpu.so step gtadp_gf_$i 300 python -u bench.py --format gt:ad:dp --no-cpu-baseline --no-e2e --steps 5 --warmup 2 || exit $?
done
echo "=== done"
