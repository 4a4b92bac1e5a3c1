# Full GPU suite + smoke + the default G100 bench line + the WAN what-if line.
set -o pipefail
mkdir -p gpurun_out
SKIP_BENCH=1 bash scripts/gpu_check.sh || exit $?
timeout -k 10 200 python -u bench.py --workload whatif --steps 5 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/b_whatif_def.log 2>&1 || exit 1
grep '^{' gpurun_out/b_whatif_def.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('whatif', round(d['ms_per_step'],3), round(d['roofline'].get('kernel_ms_mean'),3))"
