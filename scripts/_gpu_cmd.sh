set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload whatif --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/whatif.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/whatif.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/sweep.py --topology wan --variants "G=1;NT=0" --rounds 3 > gpurun_out/sweepw.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweepw.log; exit $rc
