#!/bin/bash
# r04 job: GT-first sweep batch depth (5 / 3 wave-steps against the default 4) on GT:AD:DP, and
# the AF early first batch at 5 wave-steps again ('old' rows = the variant)
bash gpu_job.sh ab gu5 build_gu5/libvcfx_gpu.so 2 --steps 20 --format gt:ad:dp || exit $?
bash gpu_job.sh ab gu3 build_gu3/libvcfx_gpu.so 1 --steps 20 --format gt:ad:dp || exit $?
bash gpu_job.sh ab eu5 build_eu5/libvcfx_gpu.so 3 --steps 20 || exit $?
