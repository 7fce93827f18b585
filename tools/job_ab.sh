#!/bin/bash
# r04 job: AF walk head analysis in scalar code (4 B per lane, first_tabs), DPP sums, buffer
# loads in af_fixed / gt_fast / gt_first_af (build/); the analysis alone (build_afscal); the
# previous build (build_afold).  Whole -m gpu suite first.
bash gpu_job.sh test || exit $?
bash gpu_job.sh ab af build_afold/libvcfx_gpu.so 2 --steps 20 || exit $?
bash gpu_job.sh ab afs build_afscal/libvcfx_gpu.so 1 --steps 20 || exit $?
bash gpu_job.sh ab afw6 build_afw6/libvcfx_gpu.so 1 --steps 20 || exit $?
bash gpu_job.sh ab gtadp build_afold/libvcfx_gpu.so 1 --steps 20 --format gt:ad:dp || exit $?
bash gpu_job.sh ab hwe build_afold/libvcfx_gpu.so 1 --steps 20 --workload hwe || exit $?
bash gpu_job.sh ab pipe build_afold/libvcfx_gpu.so 1 --steps 20 --workload pipeline || exit $?
VCFXG_WALK_CHUNK=262144 bash gpu_job.sh run af_chunk256 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
VCFXG_WALK_CHUNK=196608 bash gpu_job.sh run af_chunk192 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
bash gpu_job.sh sq afw10 || exit $?
