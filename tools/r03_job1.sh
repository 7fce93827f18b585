#!/bin/bash
# r03 first GPU pass: new LD mask kernel parity, new full-size digests, benches, 2-rank rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -4 "gpurun_out/$name.log" | cut -c1-600
    return $rc
}
step ld_tests 600 python -u -m pytest tests/test_gpu_ld.py -x -v --timeout 300 --timeout-method thread || exit $?
step bench_ld_miss 600 python -u bench.py --workload ld --missing-rate 0.001 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
step bench_ld 600 python -u bench.py --workload ld --no-cpu-baseline || exit $?
step bench_af 600 python -u bench.py || exit $?
step bench_pipeline 600 python -u bench.py --workload pipeline || exit $?
step rehearse_af 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo --no-e2e || exit $?
step scale_new 1100 python -u -m pytest tests/test_gpu_scale.py -v --timeout 900 --timeout-method thread \
    -k "missing_shard or irregular or gtadp or general_shards or ld20k_bench" || exit $?
echo "=== done"
