#!/bin/bash
# r04 job: sparse-missing LD with the per-block prefilter (parity + bench), pipe head release
bash gpu_job.sh test tests/test_gpu_ld.py tests/test_gpu_stream.py tests/test_gpu_pipe.py || exit $?
bash gpu_job.sh run ldmiss 300 python -u bench.py --workload ld --missing-rate 0.001 --no-cpu-baseline --no-e2e --steps 3 || exit $?
bash gpu_job.sh run ldmiss4 300 python -u bench.py --workload ld --missing-rate 0.004 --no-cpu-baseline --no-e2e --steps 3 --no-output-check || exit $?
bash gpu_job.sh run ld 300 python -u bench.py --workload ld --no-cpu-baseline --no-e2e --steps 3 || exit $?
bash gpu_job.sh run e2e_pipe 300 bash tools/e2e_probe.sh pipe || exit $?
