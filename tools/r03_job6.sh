#!/bin/bash
# r03: AF fixed-stride sweep on raw blocks (af_fixed): parity, then A/B against the previous
# sweep (build_base) and the build without the in-batch fallback (build_nofb)
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
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), r.get('avg_launch_ms'), r.get('frac'), (d.get('output_check') or {}).get('match'))" 2>/dev/null
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}

step af_tests 600 python -u -m pytest tests/test_gpu_af.py tests/test_gpu_af_fused.py tests/test_gpu_hwe.py tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread || exit $?
B="--no-cpu-baseline --no-e2e --steps 20 --warmup 3"
for i in 1 2; do
    step af_new_$i 300 python -u bench.py $B || exit $?
    step af_new_$i 300 python -u bench.py $B || exit $?
    VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step af_base_$i 300 python -u bench.py $B || exit $?

done
step afmiss_new 300 python -u bench.py $B --missing-rate 0.001 || exit $?
VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step afmiss_base 300 python -u bench.py $B --missing-rate 0.001 || exit $?
step scale_af 900 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 600 --timeout-method thread -k "af_" || exit $?
echo "=== done"
