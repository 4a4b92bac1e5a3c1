set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_update.py -m gpu > gpurun_out/update_tests.log 2>&1 || { tail -40 gpurun_out/update_tests.log; exit 1; }
tail -3 gpurun_out/update_tests.log
for t in grid100 fabric; do
  timeout -k 10 200 python -u bench.py --workload update --topology $t --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/update_$t.log 2>&1 || { tail -20 gpurun_out/update_$t.log; exit 1; }
  grep '^{' gpurun_out/update_$t.log | cut -c1-900
done
