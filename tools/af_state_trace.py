#!/usr/bin/env python3
"""The AF walk's two states: the region call timed call by call over a long
run in one process, to see whether a process switches between the ~0.77 and ~0.85 ms states and
when.  Prints one JSON line: per block of `--block` calls the mean and min call time (host wall
clock around vcfxg_allele_freq_region, which synchronises), and the walk's own HIP-event mean.

usage: af_state_trace.py [--calls 3000] [--block 100]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=3000)
    ap.add_argument("--block", type=int, default=100)
    a = ap.parse_args()
    from vcfx_amd import engine, synth
    arr = synth.generate_array(n_records=427409, n_samples=2504, seed=20251226)
    ds = engine.data_start_of(arr[:1 << 20].tobytes())
    e = engine.Engine(0)
    t_start = time.perf_counter()
    out = {"blocks": []}
    try:
        e.load(arr)
        for b in range(a.calls // a.block):
            ts = []
            for _ in range(a.block):
                t0 = time.perf_counter()
                e.allele_freq_region(ds)
                ts.append(time.perf_counter() - t0)
            out["blocks"].append({"t_s": round(time.perf_counter() - t_start, 2),
                                  "mean_ms": round(1e3 * sum(ts) / len(ts), 4), "min_ms": round(1e3 * min(ts), 4)})
            print("block %d t=%.1fs mean %.4f ms min %.4f ms" % (b, out["blocks"][-1]["t_s"], out["blocks"][-1]["mean_ms"],
                                                                 out["blocks"][-1]["min_ms"]), flush=True)
    finally:
        e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
