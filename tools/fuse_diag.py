#!/usr/bin/env python3
"""Developer diagnostics of the fused AF kernel (VCFXG_FUSE_DEBUG bits: 1 = index part only,
2 = print self-counted predecessor chunks)."""
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
for _ in range(2):
    e.allele_freq_region(ds)
e.set_profiling(True)
e.reset_kernel_stats()
t0 = time.perf_counter()
for _ in range(5):
    s = e.allele_freq_region(ds)
dt = (time.perf_counter() - t0) / 5
tot, n = e.kernel_stats("af_fused")
print("dbg=%s records=%d lines=%d step=%.3f ms af_fused=%.3f ms" % (os.environ.get("VCFXG_FUSE_DEBUG"), recs,
                                                                  s.n_lines, dt * 1e3, tot / n))
