"""Diagnostics: per-mode kernel times of the filter / query walk on the bench shard
(record_filter alone, genotype_query alone, the fused pipeline)."""
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from vcfx_amd import engine, synth  # noqa: E402

arr = synth.generate_array(427409, 2504, seed=20251226)
ds = engine.data_start_of(arr[:1 << 20].tobytes())
eng = engine.Engine(0)
eng.load(arr)
crits = [(engine.QUAL, engine.GE, 1, 30.0, "", ""), (engine.FILTER, engine.EQ, 0, 0.0, "", "PASS")]
runs = {"rf": lambda: eng.record_filter_region(ds, crits),
        "gq": lambda: eng.genotype_query_region(ds, "0|1"),
        "gq_strict": lambda: eng.genotype_query_region(ds, "0|1", strict=True),
        "both": lambda: eng.filter_query_region(ds, crits, "0|1")}
for name, f in runs.items():
    for _ in range(2):
        f()
    eng.set_profiling(True)
    eng.reset_kernel_stats()
    for _ in range(5):
        s = f()
    eng.set_profiling(False)
    out = {k: round(eng.kernel_stats(k)[0] / max(1, eng.kernel_stats(k)[1]), 3) for k in ("fq_walk", "fq_rest")}
    print(name, out, "rows", s.rows, "lines", s.n_lines, "general", s.general_records, flush=True)
