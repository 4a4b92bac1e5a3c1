set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lean or deep or overflow or grid" > gpurun_out/lean_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lean_tests.log; exit $rc
