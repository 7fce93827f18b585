#!/usr/bin/env python3
"""Developer timing of the AF kernels (two-pass and fused) for an experiment build
(VCFXG_GPU_LIB=build_exp/<v>/libvcfx_gpu.so)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vcfx_amd import engine, synth  # noqa: E402

recs = int(sys.argv[1]) if len(sys.argv) > 1 else 427409
arr = synth.generate_array(recs, 2504, seed=20251226)
ds = engine.data_start_of(arr[:1 << 20].tobytes())
e = engine.Engine(0)
e.load(arr)
res = {}
for name, fn in (("two-pass", lambda: (e.index(ds), e.allele_freq())), ("fused", lambda: e.allele_freq_region(ds))):
    for _ in range(2):
        fn()
    e.set_profiling(True)
    e.reset_kernel_stats()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    dt = (time.perf_counter() - t0) / 5
    ks = {}
    for k in ("line_count", "line_emit", "af_scan", "af_records", "af_fused", "af_chunks"):
        tot, n = e.kernel_stats(k)
        if n:
            ks[k] = round(tot / n, 3)
    e.set_profiling(False)
    res[name] = (round(dt * 1e3, 3), ks)
print(os.environ.get("VCFXG_GPU_LIB"), res)
