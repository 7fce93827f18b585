#!/usr/bin/env python3
"""Fold rocprofv3 --pmc counter CSVs into profiles/pmc_traffic.json (HBM bytes per launch).

usage: pmc_traffic.py WORKLOAD FETCH_CSV WRITE_CSV [OUT_JSON]

The kernels found are merged into OUT_JSON[WORKLOAD] (a second input of the same workload,
e.g. LD on data with missing calls, adds the masked-LD kernels beside the first run's).

FETCH_CSV / WRITE_CSV are the *_counter_collection.csv files of two SEPARATE runs
(`rocprofv3 --pmc FETCH_SIZE ...` and `rocprofv3 --pmc WRITE_SIZE ...`; the two counters do
not fit one pass on gfx950).  FETCH_SIZE / WRITE_SIZE are reported in KB (x1024 bytes);
per MI355X_MICROARCH.md §HBM, FETCH_SIZE reports half of the bytes of a wide coalesced
streaming read on gfx950, so it is doubled here.  Per kernel: mean over its dispatches.
"""
import csv
import json
import os
import re
import sys

# engine profiling names (vcfxg_kernel_stats) -> device kernel symbol(s); a name that times
# several launches (af_records = head pass + sweep + full-path kernel) sums their traffic
KERNELS = {
    "line_count": r"vcfxg::k_idx_sweep<false>\(",
    "line_emit": r"vcfxg::k_idx_sweep<true>\(",
    "line_compact": r"vcfxg::k_nl_compact\(",
    "af_records": r"vcfxg::k_(line_meta|af_sweep|af_complex)\(",
    "af_walk": r"vcfxg::k_af_walk<vcfxg::AfOp(, false)?>\(",
    "hwe_walk": r"vcfxg::k_af_walk<vcfxg::HweOp(, false)?>\(",
    "dose_walk": r"vcfxg::k_af_walk<vcfxg::Dose(Walk|Head)Op(, false)?>\(",
    "dose_fmt": r"vcfxg::k_dose_fmt<",
    "walk_compact": r"vcfxg::k_walk_compact\(",
    "af_complex": r"vcfxg::k_af_(complex|cx)\(",
    "af_rows": r"vcfxg::k_(walker_scan|af_rowlen|af_summary)\(",
    "af_format": r"vcfxg::k_af_format(_w)?\(",
    "hwe_lines": r"vcfxg::k_hwe_lines\(",
    "hwe_rows": r"vcfxg::k_hwe_rowlen\(",
    "hwe_format": r"vcfxg::k_hwe_format\(",
    "rf_records": r"vcfxg::k_rf_records\(",
    "fq_walk": r"vcfxg::k_fq_walk<",
    "fq_rest": r"vcfxg::k_(fq_compact<|fq_finish<|gq_complex\(|nr_complex\()",
    "nr_records": r"vcfxg::k_nr_records\(",
    "gq_records": r"vcfxg::k_(line_meta|gq_sweep|gq_complex)\(",
    "ld_parse": r"vcfxg::k_ld_parse\(",
    "ld_count": r"vcfxg::k_ld_fast<1, ?false>\(",
    "ld_count_sparse": r"vcfxg::k_ld_fast<1, ?true>\(",
    "ld_emit": r"vcfxg::k_ld_fast<2, ?(false|true)>\(",
    "ld_count_gen": r"vcfxg::k_ld_block<1>\(",
    "ld_emit_gen": r"vcfxg::k_ld_block<2>\(",
    "ld_matrix": r"vcfxg::k_ld_matrix\(",
    "ld_pack_vq": r"vcfxg::k_ld_pack_vq\(",
    "ld_count_mask": r"vcfxg::k_ld_mask<1>\(",
    "ld_emit_mask": r"vcfxg::k_ld_mask<2>\(",
}


# the engine names bench.py times per workload (a symbol shared by two names, e.g.
# k_af_complex, would otherwise leave a spurious entry under a workload that never times it)
TIMED = {
    "af": ("line_count", "line_emit", "line_compact", "af_records", "af_walk", "walk_compact", "af_complex",
           "af_rows", "af_format"),
    "hwe": ("hwe_walk", "walk_compact", "hwe_lines", "hwe_rows", "hwe_format", "line_count", "line_emit",
            "line_compact"),
    "pipeline": ("fq_walk", "fq_rest", "line_count", "line_emit", "line_compact", "rf_records", "gq_records"),
    "nonref": ("fq_walk", "fq_rest", "line_count", "line_emit", "line_compact", "nr_records"),
    "dose": ("dose_walk", "walk_compact", "dose_fmt"),
    "ld": ("line_count", "line_emit", "line_compact", "ld_parse", "ld_count", "ld_emit", "ld_count_gen",
           "ld_emit_gen", "ld_matrix", "ld_pack_vq", "ld_count_mask", "ld_emit_mask", "ld_count_sparse"),
}


# names that share a symbol with another name: kept only when their own primary kernel ran
PRIMARY = {"af_records": "vcfxg::k_af_sweep", "gq_records": "vcfxg::k_gq_sweep", "fq_rest": "vcfxg::k_fq_compact<"}


# names whose kernels launch several times per step (one per pipelined piece): the per-step
# divisor is the count of this once-per-step symbol instead
ANCHOR = {}


def per_kernel(path, counter):
    """mean per timed step: sum over the matching dispatches / number of dispatches of the
    most frequent matching symbol (one launch of each per step), or of the ANCHOR symbol"""
    acc, calls = {}, {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            for k, pat in KERNELS.items():
                if re.search(pat, name):
                    acc[k] = acc.get(k, 0.0) + float(row["Counter_Value"])
                    sym = name.split("(")[0]
                    calls.setdefault(k, {})[sym] = calls.setdefault(k, {}).get(sym, 0) + 1
    acc = {k: v for k, v in acc.items() if k not in PRIMARY or any(PRIMARY[k] in s for s in calls[k])}
    return {k: v / (calls[k].get(ANCHOR[k], 0) if k in ANCHOR and calls[k].get(ANCHOR[k]) else max(calls[k].values()))
            for k, v in acc.items()}


def main():
    workload, fcsv, wcsv = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fetch = per_kernel(fcsv, "FETCH_SIZE")
    write = per_kernel(wcsv, "WRITE_SIZE")
    try:
        with open(out) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    res = dict(d.get(workload, {}))
    for k in sorted(set(fetch) | set(write)):
        if workload in TIMED and k not in TIMED[workload]:
            continue
        fb = fetch.get(k, 0.0) * 1024 * 2   # KB -> bytes, gfx950 streaming-read correction (x2)
        wb = write.get(k, 0.0) * 1024
        res[k] = {"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb,
                  "fetch_size_kb_raw": fetch.get(k), "write_size_kb_raw": write.get(k)}
    d[workload] = res
    d["_note"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE doubled "
                  "(gfx950 wide streaming reads, MI355X_MICROARCH.md HBM section); mean per dispatch")
    with open(out, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print(json.dumps({k: res[k] for k in sorted(set(fetch) | set(write)) if k in res}, indent=1))


if __name__ == "__main__":
    main()
