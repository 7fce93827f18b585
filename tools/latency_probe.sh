set -e
mkdir -p gpurun_out
python - <<'PY'
from vcfx_amd import synth
buf = synth.generate(100, 2504, 5)
open("/tmp/small.vcf", "wb").write(buf)
PY
for i in 1 2 3; do VCFX_TIMING=1 timeout -k 5 60 build/src/VCFX_allele_freq_calc/VCFX_allele_freq_calc -q -i /tmp/small.vcf > /dev/null 2>> gpurun_out/lat.txt; echo --- >> gpurun_out/lat.txt; done
for i in 1 2 3; do /usr/bin/time -f "%e s wall %U user %S sys" timeout -k 5 60 build/src/VCFX_allele_freq_calc/VCFX_allele_freq_calc -q -i /tmp/small.vcf > /dev/null 2>> gpurun_out/lat.txt; done
timeout -k 5 60 python - >> gpurun_out/lat.txt 2>&1 <<'PY'
import ctypes, time
t0 = time.perf_counter()
lib = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
t1 = time.perf_counter()
n = ctypes.c_int()
lib.hipGetDeviceCount(ctypes.byref(n))
t2 = time.perf_counter()
lib.hipSetDevice(0)
p = ctypes.c_void_p()
lib.hipMalloc(ctypes.byref(p), 1 << 20)
t3 = time.perf_counter()
print("dlopen %.3f  hipGetDeviceCount %.3f  first malloc %.3f" % (t1 - t0, t2 - t1, t3 - t2))
PY
cat gpurun_out/lat.txt
