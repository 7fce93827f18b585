#!/bin/bash
# One gpurun session: GPU tests, a bench run, and a rocprofv3 kernel-trace of the bench.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -q --maxfail=10; rc=$?; ok_or_testfail $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py || exit $?
    cat gpurun_out/bench.log | tail -1 > gpurun_out/bench.json
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit $?
fi
echo "=== done"
