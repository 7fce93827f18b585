#!/bin/bash
# r03 (session 3): walker chunk size with the backward boundary scans (VCFXG_WALK_CHUNK), AF and
# the pipeline, two runs each
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
    return $rc
}
B="--no-cpu-baseline --no-e2e --steps 20 --warmup 3"
for i in 1 2; do
    for C in 65536 98304 131072 196608 262144; do
        VCFXG_WALK_CHUNK=$C step af_c${C}_$i 300 python -u bench.py $B || exit $?
    done
done
for C in 98304 131072 196608; do
    VCFXG_WALK_CHUNK=$C step pipe_c${C} 300 python -u bench.py --workload pipeline $B || exit $?
done
echo "=== done"
