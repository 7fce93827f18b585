#!/bin/bash
# VCFX_allele_counter: parity (unit, golden CLI cases, full-size digests), bench, rocprofv3 stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_ac.py \
    "tests/test_gpu_cli.py::test_golden_cases[VCFX_allele_counter]" tests/test_gpu_scale.py -k "ac_ or allele_counter or test_gpu_ac" \
    > gpurun_out/ac_tests.log 2>&1 || { tail -30 gpurun_out/ac_tests.log; exit 1; }
tail -1 gpurun_out/ac_tests.log
bash gpu_job.sh bench ac && bash gpu_job.sh prof ac
