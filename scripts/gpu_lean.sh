set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grid or lvl or config or G100 or smoke" > gpurun_out/lean_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lean_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/sweep.py --topology grid100 --variants "LEAN=1;LEAN=0" --rounds 8 > gpurun_out/lean_sweep.log 2>&1; rc=$?; cat gpurun_out/lean_sweep.log | tail -4; [ $rc -eq 0 ] || exit $rc
OPENR_SPF_BFS_LEAN=1 timeout -k 10 200 python -u scripts/batch_latency.py > gpurun_out/lean_batch1.log 2>&1 || exit 1
OPENR_SPF_BFS_LEAN=0 timeout -k 10 200 python -u scripts/batch_latency.py > gpurun_out/lean_batch0.log 2>&1 || exit 1
tail -4 gpurun_out/lean_batch1.log gpurun_out/lean_batch0.log
