"""Store-only HBM ceiling on one MI355X (measurement tool for write-bound kernels such as k_ac_fmt).

Times torch's fill_ over an N-byte buffer (a store-only stream: 16 B vector stores, nothing read)
and a copy_ of N / 10 bytes into N bytes' worth of destinations (the k_ac_fmt shape: about ten
output bytes per input byte), by HIP events on the current stream, best and median of R reps.

    python tools/write_ceiling.py [--gb 42.6] [--reps 10]
"""
import argparse
import json
import statistics

import torch


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ms.append(s.elapsed_time(e))
    return min(ms), statistics.median(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=42.6)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n = int(a.gb * 1e9) // 64 * 64
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    best, med = timed(lambda: dst.fill_(7), a.reps)
    out = {"bytes": n, "fill_ms_best": round(best, 3), "fill_ms_median": round(med, 3),
           "fill_gbps_best": round(n / best / 1e6, 1)}
    src = torch.empty(n // 10, dtype=torch.uint8, device="cuda").fill_(3)
    views = [dst[k * (n // 10):(k + 1) * (n // 10)] for k in range(10)]

    def fan():
        for v in views:
            v.copy_(src)
    best, med = timed(fan, a.reps)
    out.update({"fanout_copy_ms_best": round(best, 3), "fanout_copy_ms_median": round(med, 3),
                "fanout_write_gbps_best": round(10 * (n // 10) / best / 1e6, 1)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
