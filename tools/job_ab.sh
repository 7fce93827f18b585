#!/bin/bash
# r04 job: GT-first sweep sharing the OR of a lane's words between the ASCII check and the
# newline shortcut: the AF tests, then GT:AD:DP A/B against the previous build (build_gfprev2)
bash gpu_job.sh test tests/test_gpu_af.py tests/test_gpu_af_fused.py || exit $?
bash gpu_job.sh ab gtadp build_gfprev2/libvcfx_gpu.so 2 --steps 20 --format gt:ad:dp || exit $?
