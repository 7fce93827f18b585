#!/bin/bash
# r03 session-3 round end, part C: kernel-trace summaries of the AF and pipeline benches on
# the final code (staged rows copied four walkers per wave, memoised criteria bounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
B="--no-cpu-baseline --no-e2e"
for spec in "af:--steps 5 --warmup 2" "pipeline:--workload pipeline --steps 5 --warmup 2"; do
    w=${spec%%:*}; args=${spec#*:}
    step rocprof2_$w 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2_$w -o run --output-format csv -- \
        python bench.py $args $B || exit $?
    grep '^{' gpurun_out/rocprof2_$w.log > gpurun_out/rocprof2_bench_$w.json
done
echo "=== done"
