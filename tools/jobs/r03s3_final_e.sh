#!/bin/bash
# r03 session-3 round end, part E: the full GPU suite and smoke on the final tree (chunk rule)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
step pytest_gpu_e 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread || exit $?
step smoke_e 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
echo "=== done"
