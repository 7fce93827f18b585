"""The AF walk's two states against the clock (measurement tool).

Each process of tools/af_state_clock.sh ran tools/af_state_probe.py (one trial, the config-2 walk
`--steps` times) under `rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES`.  Per process and
per `af_walk` dispatch: the duration (the counter CSV's timestamps), GRBM_GUI_ACTIVE (GPU-busy
cycles summed over the 8 XCDs: / 8 / duration = the clock the walk ran at, MI355X_MICROARCH.md),
SQ_BUSY_CYCLES and the cycles the walk took at that clock.  A walk whose duration follows the
clock at a constant cycle count is a DVFS state; a walk that takes more cycles at the same clock
is not.

    python tools/af_state_clock.py OUT_JSON DIR...   (DIR: one process's rocprofv3 -d directory)
"""
import csv
import glob
import json
import os
import statistics
import sys


def one(d):
    csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not csvs:
        return None
    disp = {}
    for r in csv.DictReader(open(csvs[0])):
        if "af_walk" not in r["Kernel_Name"]:
            continue
        e = disp.setdefault(r["Dispatch_Id"], {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = [v for _, v in sorted(disp.items(), key=lambda kv: int(kv[0]))][3:]  # (the probe's 3 warm calls)
    if not rows:
        return None
    ms = [v["ns"] / 1e6 for v in rows]
    ghz = [v["GRBM_GUI_ACTIVE"] / 8.0 / v["ns"] for v in rows if "GRBM_GUI_ACTIVE" in v]
    cyc = [v["GRBM_GUI_ACTIVE"] / 8.0 for v in rows if "GRBM_GUI_ACTIVE" in v]
    busy = [v.get("SQ_BUSY_CYCLES", 0.0) for v in rows]
    out = {"process": os.path.basename(d.rstrip("/")), "dispatches": len(rows),
           "walk_ms_median": round(statistics.median(ms), 4), "walk_ms_min": round(min(ms), 4),
           "walk_ms_max": round(max(ms), 4)}
    if ghz:
        out["clock_ghz_median"] = round(statistics.median(ghz), 4)
        out["clock_ghz_min"] = round(min(ghz), 4)
        out["clock_ghz_max"] = round(max(ghz), 4)
        out["walk_kcycles_median"] = round(statistics.median(cyc) / 1e3, 1)
    out["sq_busy_cycles_median"] = statistics.median(busy)
    log = d.rstrip("/") + ".log"
    if os.path.exists(log):  # the probe's own HIP-event figure (profiled process)
        for line in open(log):
            if line.startswith("{") and "walk_ms_mean" in line:
                out["probe_walk_ms_mean"] = json.loads(line)["walk_ms_mean"]
    return out


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    procs = [p for p in (one(d) for d in dirs) if p]
    res = {"method": "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES, one process per row; "
                     "clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration",
           "processes": procs}
    if len(procs) >= 2:
        ms = [p["walk_ms_median"] for p in procs]
        kc = [p.get("walk_kcycles_median", 0) for p in procs]
        gh = [p.get("clock_ghz_median", 0) for p in procs]
        res["spread"] = {"walk_ms": [min(ms), max(ms)], "clock_ghz": [min(gh), max(gh)],
                         "walk_kcycles": [min(kc), max(kc)]}
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
