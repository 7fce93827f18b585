#!/bin/bash
# r04 job: HWE clean-step genotype classes in gt_fast (HweOp::clean), 5 wave-steps (build/) and
# 4 (build_hu4), against the previous build (build_hweprev); the gt_fast users' tests first
bash gpu_job.sh test tests/test_gpu_hwe.py tests/test_gpu_dose.py tests/test_gpu_gq.py tests/test_gpu_nr.py tests/test_gpu_pipe.py || exit $?
bash gpu_job.sh ab hwe build_hweprev/libvcfx_gpu.so 2 --steps 20 --workload hwe || exit $?
bash gpu_job.sh ab hu4 build_hu4/libvcfx_gpu.so 2 --steps 20 --workload hwe || exit $?
bash gpu_job.sh ab af build_hweprev/libvcfx_gpu.so 1 --steps 20 || exit $?
