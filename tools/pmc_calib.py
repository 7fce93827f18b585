#!/usr/bin/env python3
"""PMC calibration for the walk's HBM traffic: on the AF bench shard
(427,409 x 2,504, 4.31 GB of records), one plain streaming read (k_count_byte: every byte read
once, 16 B per lane, no re-reads) and the AF region walk, three launches each, in one process.
Run under `rocprofv3 --pmc FETCH_SIZE` (and, separately, WRITE_SIZE); then

    python tools/pmc_calib.py --fold FETCH_CSV

prints each kernel's FETCH_SIZE bytes per launch (doubled per the gfx950 note, as
tools/pmc_traffic.py does) against the bytes it has to read: the streaming kernel's ratio is the
measurement's own floor for a read-once kernel, the walk's ratio above it is its real over-fetch."""
import csv
import json
import re
import sys


def run():
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from vcfx_amd import engine, synth
    arr = synth.generate_array(n_records=427409, n_samples=2504, seed=20251226)
    ds = engine.data_start_of(arr[:1 << 20].tobytes())
    e = engine.Engine(0)
    try:
        e.load(arr)
        for _ in range(3):
            e.count_byte(ds, 13)
        for _ in range(3):
            e.allele_freq_region(ds)
        print(json.dumps({"bytes": int(arr.size), "data_start": int(ds), "region_bytes": int(arr.size - ds)}))
    finally:
        e.close()


def fold(path):
    acc = {}
    for row in csv.DictReader(open(path, newline="")):
        if row.get("Counter_Name") != "FETCH_SIZE":
            continue
        k = ("count_byte" if re.search(r"k_count_byte", row["Kernel_Name"])
             else "af_walk" if re.search(r"k_af_walk<vcfxg::AfOp", row["Kernel_Name"]) else None)
        if k:
            acc.setdefault(k, []).append(float(row["Counter_Value"]) * 1024 * 2)
    region = 4313340782  # the records' bytes (bench.py algorithmic bytes of the AF walk)
    out = {k: {"launches": len(v), "fetch_bytes_per_launch": sum(v) / len(v),
               "ratio_to_region": sum(v) / len(v) / region} for k, v in acc.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--fold":
        fold(sys.argv[2])
    else:
        run()
