#!/bin/bash
# r03: dosage head walk + checked formatting: parity, full-size digest, A/B against build_base
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
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), (d.get('output_check') or {}).get('match'), {k: round(v,3) for k,v in d.get('kernels_ms').items()})" 2>/dev/null
    tail -1 "gpurun_out/$name.log" | cut -c1-200
    return $rc
}
step dose_tests 600 python -u -m pytest tests/test_gpu_dose.py -x -q --timeout 300 --timeout-method thread || exit $?
step dose_cli 600 python -u -m pytest tests/test_gpu_cli.py -x -q --timeout 300 --timeout-method thread -k dosage || exit $?
step scale_dose 900 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 600 --timeout-method thread -k "dose" || exit $?
B="--workload dose --no-cpu-baseline --no-e2e --steps 10 --warmup 2"
for i in 1 2; do
    step dose_head_$i 300 python -u bench.py $B || exit $?
    VCFXG_DOSE_HEAD=0 step dose_sweep_$i 300 python -u bench.py $B || exit $?
    VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step dose_base_$i 300 python -u bench.py $B || exit $?
done
step dose_miss 300 python -u bench.py $B --missing-rate 0.001 || exit $?
VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step dose_miss_base 300 python -u bench.py $B --missing-rate 0.001 || exit $?
echo "=== done"
