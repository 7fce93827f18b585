# The AF walk's states against the clock: K fresh processes, each the config-2 walk under one
# rocprofv3 counter pass (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES, SQ_WAVES), then K without the profiler;
# tools/af_state_clock.py folds the passes into one JSON.
#   bash tools/af_state_clock.sh [K] [OUT_DIR]
set -e
cd $GRAFT_REPO_ROOT
K=${1:-6}
out=${2:-gpurun_out/afclk}
mkdir -p $out
export TMPDIR=/tmp
for i in $(seq 1 $K); do
    timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $out/p$i -o p \
        -- python3 -u tools/af_state_probe.py --trials 1 --steps 30 > $out/p$i.log 2>&1
    echo "pmc process $i: $(grep -m1 walk_ms_mean $out/p$i.log | cut -c1-120)"
done
for i in $(seq 1 $K); do
    timeout -k 10 240 python3 -u tools/af_state_probe.py --trials 1 --steps 30 > $out/plain$i.log 2>&1
    echo "plain process $i: $(grep -m1 walk_ms_mean $out/plain$i.log | cut -c1-120)"
done
python3 tools/af_state_clock.py $out/af_state_clock.json $(for i in $(seq 1 $K); do echo $out/p$i; done) > /dev/null
