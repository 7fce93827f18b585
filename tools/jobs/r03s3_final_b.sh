#!/bin/bash
# r03 round-end evidence, part B: rocprofv3 kernel-trace summaries of the benches and the
# FETCH_SIZE / WRITE_SIZE passes (each its own run) folded into profiles/pmc_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-300
    return $rc
}
B="--no-cpu-baseline --no-e2e"
for spec in "af:--steps 5 --warmup 2" "pipeline:--workload pipeline --steps 5 --warmup 2" \
            "ld:--workload ld --steps 2 --warmup 2" "dose:--workload dose --steps 5 --warmup 2" \
            "gtadp:--format gt:ad:dp --steps 3 --warmup 2"; do
    w=${spec%%:*}; args=${spec#*:}
    step rocprof_$w 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- \
        python bench.py $args $B || exit $?
    grep '^{' gpurun_out/rocprof_$w.log > gpurun_out/rocprof_bench_$w.json
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
for spec in "af:" "pipeline:--workload pipeline" "dose:--workload dose"; do
    w=${spec%%:*}; args=${spec#*:}
    for c in FETCH_SIZE WRITE_SIZE; do
        step pmc_${w}_$c 300 rocprofv3 --pmc $c -d gpurun_out/pmc_${w}_$c -o run --output-format csv -- \
            python bench.py $args --steps 2 --warmup 2 $B || exit $?
    done
    python tools/pmc_traffic.py $w $(find gpurun_out/pmc_${w}_FETCH_SIZE -name '*counter_collection.csv' | head -1) \
        $(find gpurun_out/pmc_${w}_WRITE_SIZE -name '*counter_collection.csv' | head -1) gpurun_out/pmc_traffic.json \
        > gpurun_out/pmc_$w.log 2>&1 || echo "pmc fold failed for $w"
done
echo "=== done"
