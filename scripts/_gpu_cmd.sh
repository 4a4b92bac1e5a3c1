set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ksp or kth" > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/ksp_probe.py > gpurun_out/ksp_probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ksp_probe.log; exit $rc
