#!/bin/bash
# r03 round-end evidence, part A: the full GPU suite, smoke, and one bench line per workload
# (the default AF line with its cpu_baseline and e2e legs)
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
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
step bench_af 600 python -u bench.py || exit $?
for w in pipeline ld nonref hwe dose ac md ph; do
    step bench_$w 600 python -u bench.py --workload $w --no-e2e || exit $?
done
step bench_gtadp 600 python -u bench.py --format gt:ad:dp --no-e2e --steps 5 --warmup 2 || exit $?
step bench_ldmiss 600 python -u bench.py --workload ld --missing-rate 0.001 --no-e2e --no-cpu-baseline --steps 3 --warmup 2 || exit $?
step rehearse_af 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-e2e || exit $?
for f in gpurun_out/bench_*.log gpurun_out/rehearse_af.log; do grep '^{' "$f" | tail -1 > "${f%.log}.json"; done
echo "=== done"
