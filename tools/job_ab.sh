#!/bin/bash
# r04 job: AF walk after the scalar head analysis: the AF tests, A/B against the previous build
# (build_afold), load-pipelining variants (unroll 8, rolling loads, carried loads), and the
# GT:AD:DP walk with / without buffer loads in gt_first_af
bash gpu_job.sh test tests/test_gpu_af.py tests/test_gpu_af_fused.py || exit $?
bash gpu_job.sh ab af build_afold/libvcfx_gpu.so 2 --steps 20 || exit $?
for v in u8 roll xrec rollu8; do
  bash gpu_job.sh ab $v build_af$v/libvcfx_gpu.so 1 --steps 20 || exit $?
done
bash gpu_job.sh ab gtadp build_afold/libvcfx_gpu.so 2 --steps 20 --format gt:ad:dp || exit $?
bash gpu_job.sh ab gfglob build_gfglob/libvcfx_gpu.so 1 --steps 20 --format gt:ad:dp || exit $?
