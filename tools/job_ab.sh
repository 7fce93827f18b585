#!/bin/bash
# r04 job: AC rows' prefix by aligned dword LDS writes
bash gpu_job.sh test tests/test_gpu_ac.py || exit $?
bash gpu_job.sh scale -k "ac_" || exit $?
for i in 1 2; do
bash gpu_job.sh run ac_$i 300 python -u bench.py --workload ac --no-cpu-baseline --no-e2e --steps 5 || exit $?
done
