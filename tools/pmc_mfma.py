"""Fold a rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (+ wave-state
counters) into MFMA utilisation per kernel launch (measurement tool).

  util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * SIMDs)
  clock = GRBM_GUI_ACTIVE / 8 / kernel duration
GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back); MFMA busy
cycles are summed over every SIMD (32 per v_mfma_scale_f32_32x32x64_f8f6f4).  ROCm 7.2's
derived MfmaUtil uses the gfx94x formula (max GRBM over one XCD) and reads 8x low here.

  python tools/pmc_mfma.py COUNTER_CSV KERNEL_REGEX OUT_JSON [SIMDS=1024]
"""
import collections
import csv
import json
import re
import sys


def main():
    path, kre, out = sys.argv[1], re.compile(sys.argv[2]), sys.argv[3]
    simds = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    per = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        if not kre.search(r["Kernel_Name"]):
            continue
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"].split("(")[0])
    launches = []
    for d, c in per.items():
        dur_ns, name = meta[d]
        gui = c["GRBM_GUI_ACTIVE"] / 8.0
        launches.append({"dispatch": int(d), "kernel": name, "duration_ms": dur_ns / 1e6,
                         "mfma_busy_cycles": c["SQ_VALU_MFMA_BUSY_CYCLES"], "gui_active_per_xcd": gui,
                         "clock_ghz": gui / dur_ns, "mfma_util": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * simds),
                         "wave_wait_frac": c.get("SQ_WAIT_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0)),
                         "wave_issue_stall_frac": c.get("SQ_WAIT_INST_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0)),
                         "wave_active_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0))})
    launches.sort(key=lambda x: x["dispatch"])
    n = len(launches)
    summ = {k: sum(x[k] for x in launches) / n for k in ("mfma_util", "clock_ghz", "duration_ms", "wave_wait_frac",
                                                          "wave_issue_stall_frac", "wave_active_frac")} if n else {}
    json.dump({"simds": simds, "launches": launches, "mean": summ}, open(out, "w"), indent=1)
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
