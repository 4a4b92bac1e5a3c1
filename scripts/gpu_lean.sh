set -o pipefail
mkdir -p gpurun_out
OPENR_SPF_CODE_BU=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_update.py > gpurun_out/bu_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/bu_tests.log | head; tail -40 gpurun_out/bu_tests.log; exit 1; }
tail -2 gpurun_out/bu_tests.log
timeout -k 10 300 python -u scripts/sweep.py --topology fabric --variants "BU=0;BU=1" --rounds 8 > gpurun_out/bu_sweep.log 2>&1 || { tail -20 gpurun_out/bu_sweep.log; exit 1; }
grep -E "variant" gpurun_out/bu_sweep.log | cut -c1-120 | tail -2
