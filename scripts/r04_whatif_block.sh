cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for b in 64 128 256; do
  OPENR_SPF_ROUNDS_BLOCK=$b timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp > gpurun_out/wb_$b.log 2>&1 || exit 1
  echo "block $b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wb_$b.log)"
  OPENR_SPF_ROUNDS_BLOCK=$b OPENR_SPF_PROF=1 timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp --steps 2 --warmup 1 > gpurun_out/wp_$b.log 2>&1 || exit 1
  grep "whatif resolve" gpurun_out/wp_$b.log | tail -1
done
