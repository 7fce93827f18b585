# k_ac_fmt under counters (measurement tool): the store-only ceiling
# (tools/write_ceiling.py, with AC_CEILING=1), then the AC bench (427 K x 2,504, text rows) with a kernel trace, two SQ
# passes and the two TCC traffic passes, folded by tools/pmc_sq.py for `k_ac_rows` and `k_ac_fmt`.
#   bash tools/prof_ac.sh [OUT_DIR] [extra bench args...]
set -e
cd $GRAFT_REPO_ROOT
out=${1:-gpurun_out/pac}
shift || true
mkdir -p $out
export TMPDIR=/tmp
[ -n "$AC_CEILING" ] && timeout -k 10 120 python3 -u tools/write_ceiling.py > $out/ceiling.json && cat $out/ceiling.json
args="--workload ac --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-output-check $@"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 -u bench.py $args > $out/kt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $out/p1 -o p1 -- python3 -u bench.py $args > $out/p1.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE --output-format csv -d $out/p2 -o p2 -- python3 -u bench.py $args > $out/p2.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/p3 -o p3 -- python3 -u bench.py $args > $out/p3.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/p4 -o p4 -- python3 -u bench.py $args > $out/p4.log 2>&1
for k in k_ac_rows k_ac_fmt; do for p in p1 p2 p3 p4; do
    python3 tools/pmc_sq.py $(ls $out/$p/*counter_collection.csv) $k $out/$p.$k.json
done; done
grep -h "ac_rows\|ac_fmt\|ac_len" $out/kt/*kernel_stats.csv | cut -c1-200
grep -h '"metric"' $out/kt.log | cut -c1-400
