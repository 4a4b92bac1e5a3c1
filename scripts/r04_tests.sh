#!/bin/bash
# Round 4: the full GPU suite and the C++ GPU tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) grep -E "FAIL|Error" gpurun_out/gpu_tests.log | head -20; exit $rc;; esac
for t in decision_test linkstate_test; do
  timeout -k 10 300 tests/cpp/build/$t gpu > gpurun_out/$t.log 2>&1; rc=$?; echo "$t rc=$rc"; tail -1 gpurun_out/$t.log
  case $rc in 0) ;; *) exit $rc;; esac
done
