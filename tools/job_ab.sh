#!/bin/bash
# r04 job: dense LD count epilogue reading each row group's terms once (A/B against the previous build)
bash gpu_job.sh test tests/test_gpu_ld.py || exit $?
for i in 1 2; do
    unset VCFXG_GPU_LIB
    bash gpu_job.sh run ld_new_$i 300 python -u bench.py --workload ld --no-cpu-baseline --no-e2e --steps 3 || exit $?
    VCFXG_GPU_LIB=build_ldold/libvcfx_gpu.so bash gpu_job.sh run ld_old_$i 300 python -u bench.py --workload ld --no-cpu-baseline --no-e2e --steps 3 || exit $?
done
