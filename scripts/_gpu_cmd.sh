set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/parity.log 2>&1 || { tail -30 gpurun_out/parity.log; exit 1; }
tail -2 gpurun_out/parity.log
for t in grid100 fabric; do for r in 1 2; do
timeout -k 10 200 python -u bench.py --topology $t --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_$t.log 2>&1 || { tail -20 gpurun_out/b_$t.log; exit 1; }
grep '^{' gpurun_out/b_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['ms_per_step'], d['roofline']['kernel_ms_mean'], d['roofline']['frac'])"
done; done
