# Scratch GPU experiment script: rewritten for each A/B measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/full_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/full_tests.log | head; tail -30 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python -u scripts/sweep.py --topology grid100 --variants "ORD=0;ORD=1" --rounds 10 > gpurun_out/ord_sweep.log 2>&1 || { tail -20 gpurun_out/ord_sweep.log; exit 1; }
grep -E "variant" gpurun_out/ord_sweep.log | cut -c1-120 | tail -2
