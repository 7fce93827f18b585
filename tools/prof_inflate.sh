# BGZF inflate kernels on the bench shard: kernel trace + two SQ counter passes (rocprofv3 sqlite)
set -e
cd $GRAFT_REPO_ROOT
out=${1:-gpurun_out/pinf}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o kt -- python3 -u tools/bgzf_probe.py --reps 1 > $out/kt.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $out/p1 -o p1 -- python3 -u tools/bgzf_probe.py --reps 1 > $out/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $out/p2 -o p2 -- python3 -u tools/bgzf_probe.py --reps 1 > $out/p2.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC -d $out/p3 -o p3 -- python3 -u tools/bgzf_probe.py --reps 1 > $out/p3.log 2>&1
python3 tools/rocpd_summary.py $(ls $out/*/*/*.db $out/*/*.db 2>/dev/null) --kernel inflate > $out/summary.txt
