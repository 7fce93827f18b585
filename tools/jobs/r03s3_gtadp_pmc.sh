#!/bin/bash
# r03 session 3: PMC of the GT-first walk on per-byte flags (GT:AD:DP shard): HBM fetch / write
# (separate passes) and the SQ wave / VALU counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    return $rc
}
B="--format gt:ad:dp --steps 1 --warmup 1 --no-cpu-baseline --no-e2e"
for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_gtadp_$c 300 rocprofv3 --pmc $c -d gpurun_out/pmc_gtadp_$c -o run --output-format csv -- python bench.py $B || exit $?
done
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
step pmc_gtadp_sq 300 rocprofv3 --pmc $SQ -d gpurun_out/pmc_gtadp_sq2 -o run --output-format csv -- python bench.py $B || exit $?
python3 tools/pmc_sq.py $(find gpurun_out/pmc_gtadp_sq2 -name '*counter_collection.csv' | head -1) 'k_af_walk' gpurun_out/pmc_gtadp_walk_sq_flags.json
python3 - <<'PY'
import csv, glob, json
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob("gpurun_out/pmc_gtadp_%s/**/*counter_collection.csv" % c, recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_af_walk<vcfxg::AfOp, true>" in r["Kernel_Name"] and r["Counter_Name"] == c]
    out[c] = {"dispatches": len(vals), "kb_mean": sum(vals) / max(1, len(vals))}
fb = out["FETCH_SIZE"]["kb_mean"] * 1024 * 2  # gfx950 wide streaming reads: x2 (MI355X_MICROARCH.md)
wb = out["WRITE_SIZE"]["kb_mean"] * 1024
out["fetch_bytes_per_launch"], out["write_bytes_per_launch"] = fb, wb
out["kernel"] = "k_af_walk<AfOp, true> (GT-first walk, per-byte flags)"
json.dump(out, open("gpurun_out/pmc_gtadp_traffic.json", "w"), indent=1)
print(json.dumps(out))
PY
cat gpurun_out/pmc_gtadp_walk_sq_flags.json
echo "=== done"
