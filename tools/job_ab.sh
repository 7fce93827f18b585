#!/bin/bash
# r04 job: AF walk VALU (SQ pass) and per-record ablations (row staging, frequency text)
bash gpu_job.sh sq afw || exit $?
for i in 1 2; do
  unset VCFXG_GPU_LIB
  bash gpu_job.sh run af_def_$i 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
  for v in build_afe1 build_afe2; do
    VCFXG_GPU_LIB=$v/libvcfx_gpu.so bash gpu_job.sh run af_${v#build_}_$i 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 --no-output-check || exit $?
  done
done
