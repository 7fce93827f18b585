#!/bin/bash
# r04 validation 3 (after the scalar head analysis): the whole -m gpu suite, smoke, the headline
# bench line (all legs), its kernel trace and PMC passes; the PMC fetch with 512 KiB chunks (does
# the walk's over-fetch scale with the walker count?)
bash gpu_job.sh test || exit $?
bash gpu_job.sh smoke || exit $?
bash gpu_job.sh bench af || exit $?
bash gpu_job.sh prof af || exit $?
bash gpu_job.sh pmc af || exit $?
VCFXG_WALK_CHUNK=524288 bash gpu_job.sh pmc afc512 || exit $?
