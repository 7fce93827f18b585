#!/bin/bash
# r04 validation: the whole -m gpu suite, smoke, the headline bench line (all legs), its
# kernel trace and PMC passes
bash gpu_job.sh test || exit $?
bash gpu_job.sh smoke || exit $?
bash gpu_job.sh bench af || exit $?
bash gpu_job.sh prof af || exit $?
bash gpu_job.sh pmc af || exit $?
