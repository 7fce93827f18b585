#!/bin/bash
# r04: SQ passes of the pipeline, HWE and GT:AD:DP walks on the final code (for the next round's
# bound analysis)
bash gpu_job.sh sq pipe --workload pipeline || exit $?
bash gpu_job.sh sq hwe --workload hwe || exit $?
bash gpu_job.sh sq gtadp --format gt:ad:dp || exit $?
