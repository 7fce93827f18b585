#!/bin/bash
# r03: dose_fmt SQ counters, checked formatting vs the r03 base build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
B="--workload dose --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
VCFXG_DOSE_HEAD=0 timeout -k 10 300 rocprofv3 --pmc $SQ -d gpurun_out/pmc_dose_new -o run --output-format csv -- python bench.py $B > gpurun_out/pmc_dose_new.log 2>&1 || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_dose_new -name '*counter_collection.csv' | head -1) 'k_dose_fmt' gpurun_out/pmc_dose_fmt_new.json
VCFXG_GPU_LIB=build_base/libvcfx_gpu.so timeout -k 10 300 rocprofv3 --pmc $SQ -d gpurun_out/pmc_dose_base -o run --output-format csv -- python bench.py $B > gpurun_out/pmc_dose_base.log 2>&1 || exit $?
python tools/pmc_sq.py $(find gpurun_out/pmc_dose_base -name '*counter_collection.csv' | head -1) 'k_dose_fmt' gpurun_out/pmc_dose_fmt_base.json
cat gpurun_out/pmc_dose_fmt_new.json gpurun_out/pmc_dose_fmt_base.json
