"""The AF walk's box states (measurement tool): the same process loads the
config-2 shard into a fresh device input buffer `--trials` times (a fresh context each time, with a
spacer allocation of a varying size kept alive between trials so the buffer lands at other
physical / virtual placements) and times `af_walk` over `--steps` calls each (HIP events on the
engine stream).  Prints one JSON line per trial: the walk's mean / min ms, the buffer's device
address and its alignment (the clock: tools/af_state_clock.sh); a bimodal walk time that follows the
placement (not the order) points at the allocation.

    python tools/af_state_probe.py [--trials 8] [--steps 20] [--out JSON]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from vcfx_amd import engine, synth
    import torch
    arr = synth.generate_array(n_records=427409, n_samples=2504, seed=20251226)
    ds = engine.data_start_of(arr[:1 << 20].tobytes())
    res = []
    spacers = []
    for t in range(a.trials):
        # a spacer of (t * 1.3 GB) % 6 GB + 64 MB held by torch's allocator, then a fresh context
        sz = ((t * 1300) % 6000 + 64) << 20
        spacers.append(torch.empty(sz, dtype=torch.uint8, device="cuda"))
        eng = engine.Engine(0)
        eng.load(arr)
        ptr = eng.L.vcfxg_input_device_ptr(eng.h) or 0
        eng.set_profiling(True)
        eng.set_profiling_only("af_walk")
        for _ in range(3):
            eng.allele_freq_region(ds, engine.MODE_FILE)
        eng.reset_kernel_stats()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.allele_freq_region(ds, engine.MODE_FILE)
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        tot, n = eng.kernel_stats("af_walk")
        eng.close()
        r = {"trial": t, "spacer_mb": sz >> 20, "walk_ms_mean": round(tot / max(n, 1), 4), "step_ms": round(wall, 4),
             "input_ptr": hex(ptr), "ptr_mod_2M": ptr % (2 << 20), "ptr_mod_1G": ptr % (1 << 30)}
        print(json.dumps(r), flush=True)
        res.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
