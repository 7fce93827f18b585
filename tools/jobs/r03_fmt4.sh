#!/bin/bash
# r03 (session 3): k_af_format_w with four clean walkers per wave (16 B rotated copies) --
# parity, A/B against build_base (a wave per walker, byte copies)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline',{}); print('VAL', d.get('value'), d.get('ms_per_step'), r.get('kernel'), round(r.get('avg_launch_ms') or 0,4), (d.get('output_check') or {}).get('match'), {k: round(v,3) for k,v in d.get('kernels_ms').items()})" 2>/dev/null
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
step t_af 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_af.py tests/test_gpu_ngpu.py tests/test_gpu_stream.py tests/test_gpu_gzip.py tests/test_gpu_cli.py -k "allele_freq or af or freq or ngpu or stream or gzip" || exit $?
step t_scale 800 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_scale.py -k "af_ or gtadp or general or irregular" || exit $?
B="--no-cpu-baseline --no-e2e --steps 20 --warmup 3"
for i in 1 2 3; do
    step af_$i 300 python -u bench.py $B || exit $?
    VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step af_base_$i 300 python -u bench.py $B || exit $?
done
step af_irr 300 python -u bench.py --irregular-rate 0.05 $B || exit $?
VCFXG_GPU_LIB=build_base/libvcfx_gpu.so step af_irr_base 300 python -u bench.py --irregular-rate 0.05 $B || exit $?
echo "=== done"
