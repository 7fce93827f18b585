#!/bin/bash
# r03: LD 128x256 two-per-CU tiles vs the 256x256 kernel (build_old), ablations (EXPT 1: no
# epilogue, 9: + k-slice 0 every step, 17: + rows 0..383 for every tile), MFMA-busy and fetch PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('avg_launch_ms'), r.get('frac'), (d.get('output_check') or {}).get('match'))" 2>/dev/null
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
B="--workload ld --no-cpu-baseline --no-e2e --steps 3 --warmup 1"
for i in 1 2; do
    step ab_new_$i 300 python -u bench.py $B || exit $?
    VCFXG_GPU_LIB=build_old/libvcfx_gpu.so step ab_old_$i 300 python -u bench.py $B || exit $?
done
for v in 1 9 17; do
    VCFXG_GPU_LIB=build_v$v/libvcfx_gpu.so step expt_$v 300 python -u bench.py $B
    rc=$?; [ $rc -le 1 ] || exit $rc
done
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
step pmc_ld_mfma 300 rocprofv3 --pmc $MF -d gpurun_out/pmc_ld_mfma -o run --output-format csv -- \
    python bench.py --workload ld --steps 1 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_ld_mfma -name '*counter_collection.csv' | head -1) 'k_ld_fast' gpurun_out/pmc_ld_fast_mfma.json
cat gpurun_out/pmc_ld_fast_mfma.json
LD="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
step pmc_ld_lds 300 rocprofv3 --pmc $LD -d gpurun_out/pmc_ld_lds -o run --output-format csv -- \
    python bench.py --workload ld --steps 1 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_ld_lds -name '*counter_collection.csv' | head -1) 'k_ld_fast' gpurun_out/pmc_ld_fast_lds.json
cat gpurun_out/pmc_ld_fast_lds.json
step pmc_ld_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_ld_fetch -o run --output-format csv -- \
    python bench.py --workload ld --steps 1 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
echo "=== done"
