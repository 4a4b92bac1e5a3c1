# Round-3 A/B evidence: multi-wave rounds kernel (what-if base SPF and overflow re-solves)
# and the two-lane KSP2 chunk pipeline; parity tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "rounds_kernel_block or wan or whatif or ksp" > gpurun_out/rounds_tests.log 2>&1 || { tail -30 gpurun_out/rounds_tests.log; exit 1; }
tail -2 gpurun_out/rounds_tests.log
for b in 64 auto; do
  if [ $b = auto ]; then unset OPENR_SPF_ROUNDS_BLOCK; else export OPENR_SPF_ROUNDS_BLOCK=$b; fi
  timeout -k 10 300 python -u bench.py --workload whatif --steps 5 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/b_whatif_$b.log 2>&1 || { tail -20 gpurun_out/b_whatif_$b.log; exit 1; }
  grep '^{' gpurun_out/b_whatif_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('whatif', '$b', d['ms_per_step'], d['roofline'].get('kernel_ms_mean'))"
done
unset OPENR_SPF_ROUNDS_BLOCK
for l in 1 2; do
  OPENR_SPF_KSP_LANES=$l timeout -k 10 300 python -u bench.py --workload ksp2 --topology fabric --ksp-sources 512 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_ksp_$l.log 2>&1 || { tail -20 gpurun_out/b_ksp_$l.log; exit 1; }
  grep '^{' gpurun_out/b_ksp_$l.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ksp lanes', '$l', d['ms_per_step'], d['value'])"
done
OPENR_SPF_PROF=1 timeout -k 10 200 python -u bench.py --workload whatif --steps 2 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/b_whatif_prof.log 2>&1 || exit 1
grep whatif_group gpurun_out/b_whatif_prof.log | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_whatif -o run --output-format csv -- python3 bench.py --workload whatif --steps 5 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/prof_whatif.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ksp -o run --output-format csv -- python3 bench.py --workload ksp2 --topology fabric --ksp-sources 512 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ksp.log 2>&1 || exit 1
for d in prof_whatif prof_ksp; do
find gpurun_out/$d -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 -c "
import csv
r=list(csv.DictReader(open('{}')))
print('$d total_ms', sum(float(x['TotalDurationNs']) for x in r)/1e6)
for x in r[:6]: print(x['Name'][:60], x['Calls'], x['AverageNs'], x['Percentage'])"
done
