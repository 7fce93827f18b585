#!/bin/bash
# r04 job: clean-step forms for the NR, MD and DOSE sweeps (NrOp / MdOp / DoseWalkOp::clean),
# their tests, then A/B against the previous build (build_cprev)
bash gpu_job.sh test tests/test_gpu_nr.py tests/test_gpu_md.py tests/test_gpu_dose.py tests/test_gpu_hwe.py || exit $?
bash gpu_job.sh ab md build_cprev/libvcfx_gpu.so 2 --steps 20 --workload md || exit $?
bash gpu_job.sh ab nr build_cprev/libvcfx_gpu.so 2 --steps 20 --workload nonref || exit $?
bash gpu_job.sh ab dose build_cprev/libvcfx_gpu.so 1 --steps 20 --workload dose || exit $?
