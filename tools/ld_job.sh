#!/bin/bash
# VCFX_ld_calculator: parity (unit + golden CLI cases + full-size digests), bench, rocprofv3 stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ld.py \
    "tests/test_gpu_cli.py::test_golden_cases[VCFX_ld_calculator]" "tests/test_gpu_scale.py::test_ld_matches_reference" \
    > gpurun_out/ld_tests.log 2>&1 || { tail -30 gpurun_out/ld_tests.log; exit 1; }
tail -1 gpurun_out/ld_tests.log
bash gpu_job.sh bench ld && bash gpu_job.sh prof ld
