"""Fold a rocprofv3 --pmc counter CSV into per-kernel sums and wave-state fractions
(measurement tool).  Counters are summed over every dispatch whose kernel name matches.

  python tools/pmc_sq.py COUNTER_CSV KERNEL_REGEX OUT_JSON

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave; wait_frac =
SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked in s_waitcnt / barriers), issue_stall_frac =
SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, active_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES;
GRBM_GUI_ACTIVE / 8 / duration = the clock (MI355X_MICROARCH.md, DVFS give-back)."""
import collections
import csv
import json
import re
import sys


def main():
    path, kre, out = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3]
    tot = collections.defaultdict(float)
    disp = {}
    for r in csv.DictReader(open(path)):
        if not kre.search(r["Kernel_Name"]):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    n = len(disp)
    res = {"kernel_regex": sys.argv[2], "dispatches": n, "mean_duration_ms": sum(disp.values()) / max(n, 1) / 1e6,
           "per_dispatch": {k: v / max(n, 1) for k, v in tot.items()}}
    w = tot.get("SQ_WAVE_CYCLES", 0.0)
    if w:
        for k, name in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                        ("SQ_ACTIVE_INST_ANY", "active_frac"), ("SQ_ACTIVE_INST_VALU", "valu_active_frac")):
            if k in tot:
                res[name] = tot[k] / w
    if "GRBM_GUI_ACTIVE" in tot and n:
        res["clock_ghz"] = tot["GRBM_GUI_ACTIVE"] / 8.0 / sum(disp.values())
    if "SQ_VALU_MFMA_BUSY_CYCLES" in tot and "GRBM_GUI_ACTIVE" in tot:
        res["mfma_util"] = tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["GRBM_GUI_ACTIVE"] / 8.0 * 1024)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
