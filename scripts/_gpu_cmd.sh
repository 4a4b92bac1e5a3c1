set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k fabric_faults > gpurun_out/faults.log 2>&1 || { tail -30 gpurun_out/faults.log; exit 1; }
tail -2 gpurun_out/faults.log
SKIP_BENCH=1 bash scripts/gpu_check.sh
