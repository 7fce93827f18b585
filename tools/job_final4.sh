#!/bin/bash
# r04 final: the whole -m gpu suite, smoke and the headline bench line on the final code; then
# the early-first-batch walk variants (VCFXG_AF_EARLY) against it, with the AF tests on each
bash gpu_job.sh test || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_full.log
bash gpu_job.sh smoke || exit $?
bash gpu_job.sh bench af || exit $?
bash gpu_job.sh prof af || exit $?
for v in eu5 ew4 eu4; do
  VCFXG_GPU_LIB=build_$v/libvcfx_gpu.so bash gpu_job.sh test tests/test_gpu_af.py || exit $?
  mv gpurun_out/pytest_gpu.log gpurun_out/pytest_gpu_$v.log
  bash gpu_job.sh ab $v build_$v/libvcfx_gpu.so 2 --steps 20 || exit $?
done
