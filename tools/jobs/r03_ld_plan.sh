#!/bin/bash
# r03 (session 3): LD streaming block lists reused across identical calls -- parity, A/B
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
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), round(r.get('avg_launch_ms') or 0,4), (d.get('output_check') or {}).get('match'))" 2>/dev/null
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
step t_ld 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ld.py tests/test_gpu_ph.py tests/test_gpu_ngpu.py tests/test_gpu_cli.py -k "ld or phaser or ngpu" || exit $?
step t_scale 800 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_scale.py -k "ld" || exit $?
B="--no-cpu-baseline --no-e2e"
for i in 1 2; do
    step ld_$i 300 python -u bench.py --workload ld $B || exit $?
    VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step ld_base_$i 300 python -u bench.py --workload ld $B || exit $?
done
step ldmiss 300 python -u bench.py --workload ld --missing-rate 0.001 --steps 3 --warmup 2 $B || exit $?
echo "=== done"
