#!/bin/bash
# r03: LD tiles 128x256 two per CU -- LD parity first, the full GPU suite, LD benches, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -4 "gpurun_out/$name.log" | cut -c1-600
    return $rc
}
B="--no-cpu-baseline --no-e2e"
step ld_tests 600 python -u -m pytest tests/test_gpu_ld.py -x -v --timeout 300 --timeout-method thread || exit $?
step bench_ld 600 python -u bench.py --workload ld $B || exit $?
step rocprof_ld 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ld -o run --output-format csv -- \
    python bench.py --workload ld --steps 2 --warmup 1 $B || exit $?
step bench_ldmiss 600 python -u bench.py --workload ld --missing-rate 0.001 --steps 3 --warmup 1 $B || exit $?
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread || exit $?
echo "=== done"
