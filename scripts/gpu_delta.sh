# Lean pass with delta rows (elld) vs 16-byte ellv rows: parity tests, then G100 A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_update.py -m gpu -k "lean or grid or config3 or wave or patch or refresh" > gpurun_out/delta_tests.log 2>&1 || { tail -30 gpurun_out/delta_tests.log; exit 1; }
tail -2 gpurun_out/delta_tests.log
for r in 1 2; do for dl in 1 0; do
  OPENR_SPF_LEAN_DELTA=$dl timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gather > gpurun_out/b_delta_$dl.log 2>&1 || { tail -20 gpurun_out/b_delta_$dl.log; exit 1; }
  grep '^{' gpurun_out/b_delta_$dl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('g100 delta=$dl', round(d['ms_per_step'],4), round(d['roofline'].get('kernel_ms_mean'),4))"
done; done
