#!/bin/bash
# The one GPU job script (gpurun sessions): tests, bench lines, rocprofv3 kernel-trace summaries,
# PMC passes and A/B runs.  Each GPU step has its own time limit; a fault / abort / timeout stops
# the script (chain invocations with &&).
#
#   bash gpu_job.sh test [pytest args...]        -m gpu tests (default: all of tests/)
#   bash gpu_job.sh scale [-k expr]              full-size reference digests (tests/test_gpu_scale.py)
#   bash gpu_job.sh smoke                        __graft_entry__.smoke()
#   bash gpu_job.sh bench NAME [bench args...]   one bench line -> gpurun_out/bench_NAME.json
#   bash gpu_job.sh ab NAME LIB N [bench args..] N alternating runs: this build vs VCFXG_GPU_LIB=LIB
#   bash gpu_job.sh prof NAME [bench args...]    rocprofv3 --kernel-trace --stats of a short bench run
#   bash gpu_job.sh pmc NAME [bench args...]     FETCH_SIZE / WRITE_SIZE passes (+ pmc_traffic.json fold)
#   bash gpu_job.sh sq NAME [bench args...]      one SQ pass (VALU / SALU / LDS / waits / busy cycles)
#   bash gpu_job.sh mfma NAME [bench args...]    one MFMA-utilisation pass
#   bash gpu_job.sh rehearse                     bench.py --gpus 2 over gloo (both ranks on this GPU)
#   bash gpu_job.sh run NAME SECS CMD...         any command as a timed step
#   bash gpu_job.sh final                        validation: whole -m gpu suite, smoke, AF bench line,
#                                                its kernel trace and PMC passes
#   bash gpu_job.sh workloads                    one bench line per workload (configs 3 and 5 and the
#                                                8(f) tools, LD with missing calls, GT:AD:DP AF)
#   bash gpu_job.sh bgzf [NAME]                  device BGZF inflate at full size (tools/bgzf_probe.py)
#
# bench args default to the AF workload (config 2); e.g. `bench ld --workload ld`.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    try:
        d=json.loads(l)
    except ValueError:
        continue
    r=d.get('roofline') or {}
    print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), round(r.get('avg_launch_ms') or 0,4),
          round(r.get('frac') or 0,3), (d.get('output_check') or {}).get('match'),
          {k: round(v,3) for k,v in (d.get('kernels_ms') or {}).items()})" 2>/dev/null
    tail -3 "gpurun_out/$name.log" | cut -c1-400
    return $rc
}
FAST="--no-cpu-baseline --no-e2e"
MODE=${1:-test}
shift
case "$MODE" in
test)
    [ $# -eq 0 ] && set -- tests
    step pytest_gpu 1100 python -u -m pytest "$@" -m gpu -q -x --timeout 300 --timeout-method thread ;;
scale)
    step pytest_scale 1100 python -u -m pytest tests/test_gpu_scale.py -v -x --timeout 900 --timeout-method thread "$@" ;;
smoke)
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
bench)
    n=$1; shift
    step bench_$n 600 python -u bench.py "$@" || exit $?
    grep '^{' gpurun_out/bench_$n.log | tail -1 > gpurun_out/bench_$n.json ;;
ab)
    n=$1 lib=$2 k=$3; shift 3
    for i in $(seq 1 "$k"); do
        step ab_${n}_new_$i 300 python -u bench.py $FAST "$@" || exit $?
        VCFXG_GPU_LIB=$lib step ab_${n}_old_$i 300 python -u bench.py $FAST "$@" || exit $?
    done ;;
prof)
    n=$1; shift
    step rocprof_$n 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- \
        python bench.py --steps 5 --warmup 1 $FAST "$@" || exit $?
    grep '^{' gpurun_out/rocprof_$n.log > gpurun_out/rocprof_bench_$n.json ;;
pmc)
    n=$1; shift
    for c in FETCH_SIZE WRITE_SIZE; do
        step pmc_${n}_$c 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${n}_$c -o run --output-format csv -- \
            python bench.py --steps 2 --warmup 1 $FAST "$@" || exit $?
    done
    python tools/pmc_traffic.py $n $(find gpurun_out/pmc_${n}_FETCH_SIZE -name '*counter_collection.csv' | head -1) \
        $(find gpurun_out/pmc_${n}_WRITE_SIZE -name '*counter_collection.csv' | head -1) gpurun_out/pmc_traffic.json \
        > gpurun_out/pmc_$n.log 2>&1 || echo "pmc fold failed for $n" ;;
sq)
    n=$1; shift
    step pmc_${n}_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY \
        SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES -d gpurun_out/pmc_${n}_sq -o run --output-format csv -- \
        python bench.py --steps 2 --warmup 1 $FAST "$@" || exit $? ;;
mfma)
    n=$1; shift
    step pmc_${n}_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_${n}_mfma -o run --output-format csv -- \
        python bench.py --steps 2 --warmup 1 $FAST "$@" || exit $? ;;
rehearse)
    step rehearse_af 600 python bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo || exit $?
    grep '^{' gpurun_out/rehearse_af.log > gpurun_out/rehearse_af.json ;;
run)
    n=$1 secs=$2; shift 2
    step "$n" "$secs" "$@" ;;
final)
    bash "$0" test || exit $?
    cp gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_full.log
    bash "$0" smoke || exit $?
    bash "$0" bench af || exit $?
    bash "$0" prof af || exit $?
    bash "$0" pmc af || exit $? ;;
workloads)
    for w in pipeline nonref hwe dose ac md ph ld; do
        bash "$0" bench $w --workload $w --no-e2e || exit $?
    done
    bash "$0" bench ldmiss --workload ld --missing-rate 0.001 --no-e2e || exit $?
    bash "$0" bench gtadp --format gt:ad:dp --no-e2e || exit $? ;;
bgzf)
    n=${1:-probe}
    step bgzf_$n 400 python -u tools/bgzf_probe.py --out gpurun_out/bgzf_$n.json || exit $? ;;
*)
    echo "unknown mode $MODE"; exit 2 ;;
esac
