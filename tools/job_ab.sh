#!/bin/bash
# r04 job: LD sparse-missing kernel (gather batching / ablations), pipe-path exit cost
for v in build_ldu4 build_ldu2 build_ldu8 build_lde32 build_lde64 build_lde96; do
    export VCFXG_GPU_LIB=$v/libvcfx_gpu.so
    x=""; case $v in *e32|*e64|*e96) x=--no-output-check;; esac
    bash gpu_job.sh run ldmiss_${v#build_} 300 python -u bench.py --workload ld --missing-rate 0.001 --no-cpu-baseline --no-e2e --steps 3 $x || exit $?
done
unset VCFXG_GPU_LIB
TIMEFORMAT="%R s"
for m in 0 1 2 3 4; do
    echo "teardown mode $m"; time (timeout -k 5 60 build/bin/teardown 1800000000 $m) || exit $?
done > gpurun_out/teardown.log 2>&1
cat gpurun_out/teardown.log
