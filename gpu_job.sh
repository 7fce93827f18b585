#!/bin/bash
# One gpurun session: GPU tests, bench runs, rocprofv3 kernel-trace summaries and PMC traffic passes.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
#   bash gpu_job.sh [test|bench|prof|pmc|all] [workloads...]     (workloads: af pipeline ld nonref hwe)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-400
    return $rc
}
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
MODE=${1:-all}
shift
WLS=${*:-af pipeline ld nonref hwe}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step pytest_gpu 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread; rc=$?; ok_or_testfail $rc || exit $rc
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    for w in $WLS; do
        step bench_$w 600 python bench.py --workload $w || exit $?
        tail -1 gpurun_out/bench_$w.log > gpurun_out/bench_$w.json
    done
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    for w in $WLS; do
        step rocprof_$w 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- \
            python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
        grep '^{' gpurun_out/rocprof_$w.log > gpurun_out/rocprof_bench_$w.json  # the bench line of the traced run
    done
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
    for w in $WLS; do
        for c in FETCH_SIZE WRITE_SIZE; do
            step pmc_${w}_$c 600 rocprofv3 --pmc $c -d gpurun_out/pmc_${w}_$c -o run --output-format csv -- \
                python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
        done
        python tools/pmc_traffic.py $w $(find gpurun_out/pmc_${w}_FETCH_SIZE -name '*counter_collection.csv' | head -1) \
            $(find gpurun_out/pmc_${w}_WRITE_SIZE -name '*counter_collection.csv' | head -1) gpurun_out/pmc_traffic.json \
            > gpurun_out/pmc_$w.log 2>&1 || echo "pmc fold failed for $w"
    done
fi

if [ "$MODE" = rehearse ]; then
    # bench.py launches its own ranks for --gpus N (torch.distributed.run on 127.0.0.1); gloo:
    # both ranks share the one GPU of this box
    step rehearse_af 600 python bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo || exit $?
    grep '^{' gpurun_out/rehearse_af.log > gpurun_out/rehearse_af.json
    step rehearse_ld 600 python bench.py --gpus 2 --workload ld --records 20000 --window 20000 --steps 2 --warmup 1 \
        --dist-backend gloo --no-cpu-baseline --no-e2e || exit $?
fi
if [ "$MODE" = scale ]; then  # full-size reference digests (tests/test_gpu_scale.py), optionally -k filtered
    step pytest_scale 1100 python -u -m pytest tests/test_gpu_scale.py -v -x --timeout 900 --timeout-method thread \
        ${*:+-k "$*"} || exit $?
fi
echo "=== done"

if [ "$MODE" = mfma ]; then
    # LD MFMA utilisation: MFMA-busy cycles, wave activity and the GPU clock, one pass
    timeout -k 5 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
    step pmc_ld_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
        -d gpurun_out/pmc_ld_mfma -o run --output-format csv -- \
        python bench.py --workload ld --steps 2 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
fi
