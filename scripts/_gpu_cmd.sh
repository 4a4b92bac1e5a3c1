set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k whatif > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload whatif --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/whatif.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/whatif.log | tail -1 | cut -c1-300; exit $rc
