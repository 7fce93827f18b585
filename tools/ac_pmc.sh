#!/bin/bash
# k_ac_fmt counters: wave-state split, LDS issue / bank conflicts, HBM write and fetch bytes
# (separate passes; SQ <= 8, TCC <= 4 counters per pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run TAG COUNTERS...
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/acpmc_$tag -o run --output-format csv -- \
      python bench.py --workload ac --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/acpmc_$tag.log 2>&1 || return $?
  echo "pass $tag done"
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS || exit $?
run wr WRITE_SIZE || exit $?
run rd FETCH_SIZE || exit $?
python - <<'PY'
import csv, glob, collections
for tag in ("sq", "wr", "rd"):
    f = glob.glob("gpurun_out/acpmc_%s/**/*counter_collection.csv" % tag, recursive=True)
    if not f:
        print(tag, "no csv"); continue
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "k_ac_fmt" not in r.get("Kernel_Name", ""): continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    for k in acc:
        print(tag, k, acc[k], "records", n[k])
PY
