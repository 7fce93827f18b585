#!/usr/bin/env python3
"""bench.py -- VCFX_allele_freq_calc hot path on MI355X (BASELINE.json configs[1]; N>1 =
configs[3], record-sharded, weak scaling).

A step = one pass of the hot path over one batch of synthetic input that is already
resident in HBM: record index (K1) + per-record allele counts (K2) + device-formatted
output rows (K5).  Each rank processes its own 427,409-record x 2,504-sample shard
(≈4.3 GB, chr21-like layout; seed = 20251226 + rank).  value = records processed by all
ranks / max-over-ranks wall time of the timed steps.

Prints ONE JSON line on rank 0 (see the contract in the task / DESIGN.md §Measurement).
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "variant-records/sec (and GB/s vs HBM roofline), 427K var × 2504 samp"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=427409)
    ap.add_argument("--samples", type=int, default=2504)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(arr, offs, n_records, budget_s):
    """The C restatement oracle (oracle/, kind "port"), 1 thread, file (mmap) path of
    VCFX_allele_freq_calc over a bounded prefix sample of this rank's synthetic input."""
    from tests._golden import Oracle
    sample_records = min(n_records, 20000)
    sample = arr[:int(offs[sample_records])].tobytes()  # header + first sample_records records
    o = Oracle()
    with tempfile.NamedTemporaryFile(suffix=".vcf", dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as f:
        f.write(sample)
        f.flush()
        reps, t_total = 0, 0.0
        while t_total < budget_s or reps == 0:
            t0 = time.perf_counter()
            out, err, rc = o.run(["VCFX_allele_freq_calc", "-q", "-i", f.name])
            t_total += time.perf_counter() - t0
            reps += 1
            assert rc == 0
    return {"value": sample_records * reps / t_total, "unit": "records/s", "cores": 1, "kind": "port",
            "sample": "first %d records (%.1f MB) of the rank-0 shard, VCFX_allele_freq_calc -q -i (file path), "
                      "%d reps, %.1f s" % (sample_records, len(sample) / 1e6, reps, t_total)}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from vcfx_amd import engine, synth

    arr, offs = synth.generate_array(a.records, a.samples, seed=20251226 + rank, rec_offsets=True)
    head = arr[:1 << 20].tobytes()
    ds = engine.data_start_of(head)
    eng = engine.Engine(local)
    eng.load(arr)
    region_bytes = arr.size - ds

    def step():
        eng.index(ds)
        return eng.allele_freq(engine.MODE_FILE)

    s = None
    for _ in range(a.warmup):
        s = step()
    assert s is None or s.rows == a.records, "unexpected row count %s" % (s and s.rows)

    def barrier():
        if dist is not None:
            dist.barrier()

    eng.set_profiling(True)
    eng.reset_kernel_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = step()
    barrier()
    dt = time.perf_counter() - t0
    eng.set_profiling(False)
    assert s.rows == a.records and s.general_records == 0

    kernels = {}
    for k in ("line_count", "line_emit", "af_records", "af_rows", "af_format"):
        tot, n = eng.kernel_stats(k)
        if n:
            kernels[k] = tot / n
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    records_total = a.records * world
    value = records_total * a.steps / dt

    if rank == 0:
        # dominant kernel + its algorithmic bytes per launch
        L = s.n_lines
        algo = {
            "af_records": region_bytes + L * (8 + 13),   # record bytes + line_end read + per-line results
            "line_count": region_bytes,
            "line_emit": region_bytes + 8 * L,
            "af_format": s.text_bytes + L * (8 + 8 + 13) + s.rows * 40,
            "af_rows": L * (5 + 8 + 8 + 8),
        }
        dom = max(kernels, key=kernels.get)
        ach = algo[dom] / (kernels[dom] * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "records/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: vcfx_synth seed 20251226+rank, chr21-like layout (FORMAT=GT, phased a|b, INFO=.)",
            "config": {"workload": "VCFX_allele_freq_calc -i (file path) on a device-resident %d x %d VCF shard "
                                   "per GPU: index + allele counts + formatted rows" % (a.records, a.samples),
                       "records_per_gpu": a.records, "samples": a.samples, "bytes_per_gpu": int(arr.size),
                       "parallelism": "record-sharded x%d (no data-path collective)" % world},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": None,
                         "algorithmic_bytes_per_launch": int(algo[dom]),
                         "avg_launch_ms": kernels[dom]},
            "kernels_ms": kernels,
            "pipeline_input_gbps": region_bytes * world * a.steps / dt / 1e9,
        }
        if not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(arr, offs, a.records, a.cpu_seconds)
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
