#!/bin/bash
# r04 final (after the HWE clean steps): the whole -m gpu suite, smoke, the AF and HWE bench lines
bash gpu_job.sh test || exit $?
bash gpu_job.sh smoke || exit $?
bash gpu_job.sh bench af || exit $?
bash gpu_job.sh bench hwe --workload hwe --no-e2e || exit $?
