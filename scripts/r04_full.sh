#!/bin/bash
# Round 4: the full GPU suite, then the what-if and KSP2 bench lines.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head -20; exit $rc;; esac
for t in decision_test linkstate_test; do
  timeout -k 10 300 tests/cpp/build/$t gpu > gpurun_out/$t.log 2>&1; rc=$?; echo "$t rc=$rc"; tail -1 gpurun_out/$t.log
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 300 python3 -u bench.py --workload whatif > gpurun_out/whatif.log 2>&1; rc=$?; echo "whatif rc=$rc"
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*' gpurun_out/whatif.log | head -3
case $rc in 0) ;; *) tail -20 gpurun_out/whatif.log; exit $rc;; esac
timeout -k 10 400 python3 -u bench.py --workload ksp2 > gpurun_out/ksp2.log 2>&1; rc=$?; echo "ksp2 rc=$rc"
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*' gpurun_out/ksp2.log | head -3
exit $rc
