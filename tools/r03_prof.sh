#!/bin/bash
# r03 profiles: rocprofv3 kernel-trace summaries of the benches, PMC passes (each its own run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
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
B="--no-cpu-baseline --no-e2e"
for spec in "af:--steps 5 --warmup 1" "pipeline:--workload pipeline --steps 5 --warmup 1" \
            "ld:--workload ld --steps 2 --warmup 1" "ldmiss:--workload ld --missing-rate 0.001 --steps 2 --warmup 1" \
            "dose:--workload dose --steps 5 --warmup 1" "gtadp:--format gt:ad:dp --steps 3 --warmup 1"; do
    w=${spec%%:*}; args=${spec#*:}
    step rocprof_$w 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- \
        python bench.py $args $B || exit $?
    grep '^{' gpurun_out/rocprof_$w.log > gpurun_out/rocprof_bench_$w.json
done
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
step pmc_af_sq 300 rocprofv3 --pmc $SQ -d gpurun_out/pmc_af_sq -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 $B || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_af_sq -name '*counter_collection.csv' | head -1) 'k_af_walk' gpurun_out/pmc_af_walk_sq.json
step pmc_gtadp_sq 300 rocprofv3 --pmc $SQ -d gpurun_out/pmc_gtadp_sq -o run --output-format csv -- \
    python bench.py --format gt:ad:dp --steps 1 --warmup 1 $B || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_gtadp_sq -name '*counter_collection.csv' | head -1) 'k_af_walk' gpurun_out/pmc_gtadp_walk_sq.json
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
step pmc_ldmiss_mfma 300 rocprofv3 --pmc $MF -d gpurun_out/pmc_ldmiss_mfma -o run --output-format csv -- \
    python bench.py --workload ld --missing-rate 0.001 --steps 1 --warmup 1 $B || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_ldmiss_mfma -name '*counter_collection.csv' | head -1) 'k_ld_mask' gpurun_out/pmc_ld_mask_mfma.json
for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_ldmiss_$c 300 rocprofv3 --pmc $c -d gpurun_out/pmc_ldmiss_$c -o run --output-format csv -- \
        python bench.py --workload ld --missing-rate 0.001 --steps 1 --warmup 1 $B || exit $?
done
echo "=== done"
