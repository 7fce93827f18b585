# The dense LD count kernel under counters (measurement tool): the config-5
# bench (W = 100 K, 2,504 samples, 100 K variants) with a kernel trace and two SQ counter passes,
# folded by tools/pmc_sq.py for `k_ld_fast<1, false>` (MFMA busy, LDS instructions and bank
# conflicts, issue stalls, the clock).
#   bash tools/prof_ld.sh [OUT_DIR] [extra bench args...]
set -e
cd $GRAFT_REPO_ROOT
out=${1:-gpurun_out/pld}
shift || true
mkdir -p $out
export TMPDIR=/tmp
args="--workload ld --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-output-check $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 -u bench.py $args > $out/kt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $out/p1 -o p1 -- python3 -u bench.py $args > $out/p1.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d $out/p2 -o p2 -- python3 -u bench.py $args > $out/p2.log 2>&1
for p in p1 p2; do
    python3 tools/pmc_sq.py $(ls $out/$p/*counter_collection.csv) 'k_ld_fast<1, false>' $out/$p.json > /dev/null
done
python3 - $out <<'PY'
import json, sys
out = sys.argv[1]
a, b = json.load(open(out + "/p1.json")), json.load(open(out + "/p2.json"))
pd = dict(a["per_dispatch"]); pd.update(b["per_dispatch"])
res = {"kernel": "k_ld_fast<1, false>", "dispatches": a["dispatches"], "mean_duration_ms_pmc": a["mean_duration_ms"],
       "per_dispatch": pd}
clk = pd["GRBM_GUI_ACTIVE"] / 8.0 / (b["mean_duration_ms"] * 1e6)
res["clock_ghz"] = clk
cyc_cu = pd["GRBM_GUI_ACTIVE"] / 8.0  # cycles per dispatch (each CU)
res["mfma_busy_frac"] = pd["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc_cu * 256 * 4)
res["lds_instr_per_cu_cycle"] = pd["SQ_INSTS_LDS"] / (cyc_cu * 256)
res["lds_bank_conflict_per_lds_instr"] = pd["SQ_LDS_BANK_CONFLICT"] / max(pd["SQ_INSTS_LDS"], 1)
res["issue_stall_frac"] = pd["SQ_WAIT_INST_ANY"] / pd["SQ_WAVE_CYCLES"]
res["wait_frac"] = pd["SQ_WAIT_ANY"] / pd["SQ_WAVE_CYCLES"]
res["active_lds_frac"] = pd["SQ_ACTIVE_INST_LDS"] / pd["SQ_WAVE_CYCLES"]
json.dump(res, open(out + "/ld_fast_sq.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
