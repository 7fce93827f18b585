#!/bin/bash
# r03 (session 3): the walker chunk from the mean record length (16 records for records over
# 16 KiB) -- parity on long-record inputs, GT:AD:DP bench
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
    tail -2 "gpurun_out/$name.log" | cut -c1-200
    return $rc
}
step t_walk 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_af.py tests/test_gpu_fq_walk.py tests/test_gpu_dose.py tests/test_gpu_md.py tests/test_gpu_ngpu.py || exit $?
step t_scale 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_scale.py -k "gtadp or general" || exit $?
G="--format gt:ad:dp --no-cpu-baseline --no-e2e --steps 5 --warmup 2"
step gtadp 300 python -u bench.py $G || exit $?
step af 300 python -u bench.py --no-cpu-baseline --no-e2e || exit $?
echo "=== done"
