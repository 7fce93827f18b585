#!/bin/bash
# r04 A/B job: AF walk variants (carried first loads across records, rolling loads, baseline)
bash gpu_job.sh test tests/test_gpu_af.py tests/test_gpu_af_fused.py tests/test_gpu_ld.py || exit $?
for i in 1 2; do
  for v in "" build_x3 build_r6 build_r5 build_base; do
    n=${v:-xrec6}
    if [ -n "$v" ]; then export VCFXG_GPU_LIB=$v/libvcfx_gpu.so; else unset VCFXG_GPU_LIB; fi
    bash gpu_job.sh run af_${n}_$i 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
  done
done
unset VCFXG_GPU_LIB
bash gpu_job.sh bench ldmiss --workload ld --missing-rate 0.001 --no-cpu-baseline --no-e2e || exit $?
bash gpu_job.sh scale -k "vcfx_pipe or ld_tail" || exit $?
bash gpu_job.sh run e2e_probe 400 bash tools/e2e_probe.sh || exit $?
