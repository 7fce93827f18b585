#!/bin/bash
# r03 (session 3): walker chunk size on the GT:AD:DP shard (30 KB records: each walker's two
# backward boundary scans cover about a record)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    grep '^{' "gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), round(r.get('avg_launch_ms') or 0,4), (d.get('output_check') or {}).get('match'))" 2>/dev/null
    return $rc
}
G="--format gt:ad:dp --no-cpu-baseline --no-e2e --steps 5 --warmup 2"
for C in 131072 262144 524288 1048576; do
    VCFXG_WALK_CHUNK=$C step gtadp_c$C 300 python -u bench.py $G || exit $?
done
echo "=== done"
