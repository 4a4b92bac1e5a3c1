# Lean pass register target A/B (waves per SIMD 5 vs 8) + lean parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "lean or config3 or grid" > gpurun_out/wpe_tests.log 2>&1 || { tail -30 gpurun_out/wpe_tests.log; exit 1; }
tail -1 gpurun_out/wpe_tests.log
for r in 1 2; do for w in 5 8; do
  OPENR_SPF_LEAN_WPE=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gather > gpurun_out/b_wpe_$w.log 2>&1 || { tail -20 gpurun_out/b_wpe_$w.log; exit 1; }
  grep '^{' gpurun_out/b_wpe_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('g100 wpe=$w', round(d['ms_per_step'],4), round(d['roofline'].get('kernel_ms_mean'),4))"
done; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "whatif_wan_sample" > gpurun_out/wpe_wtests.log 2>&1 || { tail -30 gpurun_out/wpe_wtests.log; exit 1; }
for w in 1 5 7 1 5; do
  OPENR_SPF_WHATIF_WPE=$w timeout -k 10 200 python -u bench.py --workload whatif --steps 5 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/b_wwpe_$w.log 2>&1 || { tail -20 gpurun_out/b_wwpe_$w.log; exit 1; }
  grep '^{' gpurun_out/b_wwpe_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('whatif wpe=$w', round(d['ms_per_step'],3), round(d['roofline'].get('kernel_ms_mean'),3))"
done
