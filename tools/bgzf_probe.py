"""Device BGZF inflate at BASELINE scale (measurement tool): the 427,409 x 2,504 shard as BGZF
(build/bin/vcfx_bgzf, level 1 as bench.py's e2e leg, or --level), inflated on the device by
vcfxg_ingest_bgzf in a warm context, K times; per-kernel HIP-event times (bgzf_h2d, bgzf_inflate,
bgzf_crc32) and the inflated bytes' GB/s; the output checked against the plain bytes once (sha256).

    python tools/bgzf_probe.py [--records N] [--level L] [--reps K] [--out JSON]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=427409)
    ap.add_argument("--samples", type=int, default=2504)
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    from vcfx_amd import engine, synth
    arr = synth.generate_array(n_records=a.records, n_samples=a.samples, seed=20251226)
    d = tempfile.mkdtemp(prefix="vcfx_bgzfprobe_")
    plain, bgz = os.path.join(d, "s.vcf"), os.path.join(d, "s.vcf.gz")
    try:
        arr.tofile(plain)
        t0 = time.perf_counter()
        subprocess.check_call([os.path.join(REPO, "build", "bin", "vcfx_bgzf"), plain, bgz, "16", str(a.level)])
        comp = np.fromfile(bgz, np.uint8)
        mem = engine.bgzf_members(comp)
        print("members %d, compressed %.1f MB, inflated %.3f GB (bgzf write %.1f s)" % (
            len(mem), comp.size / 1e6, arr.size / 1e9, time.perf_counter() - t0), flush=True)
        eng = engine.Engine(0)
        eng.set_profiling(True)
        walls, ks = [], {"bgzf_h2d": [], "bgzf_inflate": [], "bgzf_crc32": []}
        for r in range(a.reps + 1):
            eng.reset_kernel_stats()
            t0 = time.perf_counter()
            res = eng.load_bgzf(comp, mem)
            w = time.perf_counter() - t0
            assert res is None, res
            if r == 0:  # (the first call allocates)
                got = eng.input_bytes(0, arr.size)
                assert hashlib.sha256(got).digest() == hashlib.sha256(arr.tobytes()).digest(), "inflated bytes differ"
                del got
                continue
            walls.append(w)
            handed = eng.bgzf_handed_over()
            for k in ks:
                ks[k].append(eng.kernel_stats(k)[0])
            print("rep %d: wall %.2f ms, %s, handed over %d" % (r, 1e3 * w, {k: round(v[-1], 3) for k, v in ks.items()},
                                                                handed), flush=True)
        eng.close()
        best = {k: min(v) for k, v in ks.items()}
        out = {"records": a.records, "samples": a.samples, "level": a.level, "members": len(mem),
               "compressed_bytes": int(comp.size), "inflated_bytes": int(arr.size),
               "wall_ms_best": round(1e3 * min(walls), 3), "kernel_ms_best": {k: round(v, 3) for k, v in best.items()},
               "inflate_GBps_output": round(arr.size / (best["bgzf_inflate"] * 1e-3) / 1e9, 1),
               "crc_GBps": round(arr.size / (best["bgzf_crc32"] * 1e-3) / 1e9, 1),
               "records_per_s_device_inflate": round(a.records / (best["bgzf_inflate"] + best["bgzf_crc32"]) * 1e3),
               "members_handed_to_wave_decoder": handed,
               "lane_decoder": os.environ.get("VCFX_INFLATE_LANES", "1") != "0",
               "output_sha256_matches_plain": True}
        print(json.dumps(out))
        if a.out:
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        for x in os.listdir(d):
            os.unlink(os.path.join(d, x))
        os.rmdir(d)


if __name__ == "__main__":
    main()
