cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for s in 4 2 8 16 3 6; do
  echo "== super $s"
  VCFXG_LD_SUPER=$s timeout -k 10 240 python bench.py --workload ld --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ld_super_$s.log 2>&1 || exit $?
  tail -1 gpurun_out/ld_super_$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
