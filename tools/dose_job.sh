#!/bin/bash
# VCFX_dosage_calculator: parity (unit, golden CLI cases, full-size digest) and the dose_len
# kernel time under rocprofv3 for the default build and (if present) build_w5/ (5 waves/SIMD)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dose.py \
    "tests/test_gpu_cli.py::test_golden_cases[VCFX_dosage_calculator]" tests/test_gpu_scale.py -k "dose" \
    > gpurun_out/dose_tests.log 2>&1 || { tail -30 gpurun_out/dose_tests.log; exit 1; }
tail -1 gpurun_out/dose_tests.log
prof() {  # prof TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dose_$tag -o run --output-format csv -- \
      python bench.py --workload dose --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/dose_$tag.log 2>&1 || return $?
  grep '^{' gpurun_out/dose_$tag.log > gpurun_out/dose_$tag.json
  echo "$tag $(python -c "import json; d=json.load(open('gpurun_out/dose_$tag.json')); print(d['value'], d['ms_per_step'], d.get('output_check',{}).get('match'))")"
  python - "gpurun_out/dose_$tag" <<'PY'
import csv, glob, sys
for r in csv.reader(open(glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0])):
    if 'dose' in r[0]: print('   ', r[0][:40], r[1], r[3])
PY
}
prof split VCFXG_UNUSED=0 || exit $?
if [ -f build_w5/libvcfx_gpu.so ]; then prof w5 VCFXG_GPU_LIB=$PWD/build_w5/libvcfx_gpu.so || exit $?; fi
