#!/bin/bash
# r03: the in-process multi-GPU drop-in on one GPU, masked-LD bench again
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
step ngpu_tests 900 python -u -m pytest tests/test_gpu_ngpu.py -x -v --timeout 300 --timeout-method thread || exit $?
step dose_tests 600 python -u -m pytest tests/test_gpu_dose.py -x -v --timeout 300 --timeout-method thread || exit $?
step bench_dose 600 python -u bench.py --workload dose --no-e2e || exit $?
step af_tests 600 python -u -m pytest tests/test_gpu_af.py -x -v --timeout 300 --timeout-method thread || exit $?
step bench_af_gtadp 600 python -u bench.py --format gt:ad:dp --steps 5 --warmup 2 --no-e2e || exit $?
step bench_ld_miss2 600 python -u bench.py --workload ld --missing-rate 0.001 --steps 3 --warmup 1 --no-cpu-baseline || exit $?

# A/B: the AF walk sweep over raw blocks (gt_fast_bytes) vs gt_fast, same box, alternating
for i in 1 2; do
    step bench_af_A$i 300 python -u bench.py --steps 30 --no-cpu-baseline --no-e2e || exit $?
    VCFXG_GPU_LIB=build_v/libvcfx_gpu.so step bench_af_B$i 300 python -u bench.py --steps 30 --no-cpu-baseline --no-e2e || exit $?
done
echo "=== done"
