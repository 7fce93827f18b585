#!/bin/bash
# VCFX_haplotype_phaser: parity (unit, golden CLI cases, full-size digests), then the bench with
# the record sweep's 8 and 4 KiB-step batches, then the rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ph.py \
    "tests/test_gpu_cli.py::test_golden_cases[VCFX_haplotype_phaser]" tests/test_gpu_scale.py -k "ph" \
    > gpurun_out/ph_tests.log 2>&1 || { tail -30 gpurun_out/ph_tests.log; exit 1; }
tail -1 gpurun_out/ph_tests.log
for u in 4 8; do
  VCFXG_PH_UNROLL=$u timeout -k 10 300 python bench.py --workload ph --no-e2e > gpurun_out/ph_bench_u$u.log 2>&1 || exit $?
  echo "unroll=$u $(tail -1 gpurun_out/ph_bench_u$u.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d.get('output_check',{}).get('match'))")"
done
bash gpu_job.sh prof ph
