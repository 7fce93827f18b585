#!/bin/bash
# r04 validation 2: a bench line per workload (reference CPU baseline included), the warm file ring
for w in pipeline nonref hwe dose ac md ph ld; do
    bash gpu_job.sh bench $w --workload $w --no-e2e || exit $?
done
bash gpu_job.sh bench ldmiss --workload ld --missing-rate 0.001 --no-e2e || exit $?
bash gpu_job.sh bench gtadp --format gt:ad:dp --no-e2e || exit $?
bash gpu_job.sh run e2e_warm 400 bash tools/e2e_probe.sh warm || exit $?
