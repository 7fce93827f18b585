#!/bin/bash
# r03: dosage head walk (DoseHeadOp + checked formatting): parity, full-size digest, A/B bench
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
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), r.get('avg_launch_ms'), r.get('frac'), (d.get('output_check') or {}).get('match'), d.get('kernels_ms'))" 2>/dev/null
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}


B="--workload dose --no-cpu-baseline --no-e2e --steps 10 --warmup 2"
for i in 1 2; do
    step dose_new_$i 300 python -u bench.py $B || exit $?
    VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step dose_base_$i 300 python -u bench.py $B || exit $?
done
step dose_new_miss 300 python -u bench.py $B --missing-rate 0.001 || exit $?

echo "=== done"
