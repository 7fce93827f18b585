bash gpu_job.sh test tests/test_gpu_ld.py tests/test_gpu_af.py tests/test_gpu_af_fused.py || exit $?
bash gpu_job.sh bench ldmiss --workload ld --missing-rate 0.001 --no-cpu-baseline --no-e2e || exit $?
for i in 1 2; do
  bash gpu_job.sh run af_roll6_$i 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
  VCFXG_GPU_LIB=build_u5/libvcfx_gpu.so bash gpu_job.sh run af_roll5_$i 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
  VCFXG_GPU_LIB=build_base/libvcfx_gpu.so bash gpu_job.sh run af_base_$i 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
done
bash gpu_job.sh scale -k "vcfx_pipe or ld_tail" || exit $?
bash gpu_job.sh run e2e_probe 400 bash tools/e2e_probe.sh || exit $?
