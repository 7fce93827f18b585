#!/bin/bash
# r04 job: LD sparse-missing kernel (parity + gather batching / diagnostic variants), the pipe
# path's head catch-up and ring shape, AF walk defaults
bash gpu_job.sh test tests/test_gpu_ld.py tests/test_gpu_stream.py tests/test_gpu_pipe.py || exit $?
for v in "" build_ldu4 build_lde32 build_lde64 build_lde96; do
    n=${v:-cur}
    if [ -n "$v" ]; then export VCFXG_GPU_LIB=$v/libvcfx_gpu.so; else unset VCFXG_GPU_LIB; fi
    bash gpu_job.sh run ldmiss_$n 300 python -u bench.py --workload ld --missing-rate 0.001 --no-cpu-baseline --no-e2e --steps 3
    rc=$?; [ $rc -ne 0 ] && [ -z "$v" -o "$v" = build_ldu4 ] && exit $rc
    [ $rc -gt 1 ] && exit $rc
done
unset VCFXG_GPU_LIB
bash gpu_job.sh run af_def 300 python -u bench.py --no-cpu-baseline --no-e2e --steps 20 || exit $?
bash gpu_job.sh run e2e_pipe 300 bash tools/e2e_probe.sh pipe || exit $?
