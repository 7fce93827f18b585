#!/bin/bash
# r04 job: PH pair sums by byte dot products
bash gpu_job.sh test tests/test_gpu_ph.py || exit $?
bash gpu_job.sh scale -k "ph" || exit $?
for i in 1 2; do
    bash gpu_job.sh run ph_$i 300 python -u bench.py --workload ph --no-cpu-baseline --no-e2e --steps 20 || exit $?
done
