#!/bin/bash
# round-end rehearsal: every GPU test, smoke(), the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/final_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-600
