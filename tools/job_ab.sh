#!/bin/bash
# r04 job: pipe path (head prefaulter), stdin/pipe tests + probe
bash gpu_job.sh test tests/test_gpu_stream.py tests/test_gpu_pipe.py || exit $?
bash gpu_job.sh run e2e_pipe 300 bash tools/e2e_probe.sh pipe || exit $?
