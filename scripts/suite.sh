#!/bin/bash
# The full GPU suite, the C++ GPU tests, then every DecisionBenchmark case
# (bench.py --workload decision). Output under gpurun_out/$ROUND/suite/ (ROUND=r06 by default).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROUND="${ROUND:-r06}"
O="$R/gpurun_out/$ROUND/suite"
mkdir -p "$O" && cd "$R"
if [ "${PYTESTS:-1}" = 1 ]; then
  timeout -k 10 1000 python3 -u -m pytest -v -m gpu -x --timeout 300 --timeout-method thread tests/ > "$O/gpu_tests.log" 2>&1; rc=$?
  echo "gpu tests rc=$rc"; tail -1 "$O/gpu_tests.log"
  case $rc in 0) ;; *) grep -E "FAIL|Error" "$O/gpu_tests.log" | head -20; exit $rc;; esac
fi
for t in decision_test linkstate_test; do
  timeout -k 10 300 tests/cpp/build/$t gpu > "$O/$t.log" 2>&1; rc=$?; echo "$t rc=$rc"; tail -1 "$O/$t.log"
  case $rc in 0) ;; *) grep FAIL "$O/$t.log" | head; exit $rc;; esac
done
if [ "${DECISION:-1}" = 1 ]; then
  timeout -k 10 1100 python3 -u bench.py --workload decision --steps 10 --warmup 2 > "$O/decision.log" 2>&1; rc=$?
  echo "decision rc=$rc"; grep '^{' "$O/decision.log" > "$O/decision.jsonl"
  grep -o '"workload": "BM[^"]*"\|"ms_per_update": [0-9.]*\|"check": "[^"]*"' "$O/decision.log" | paste - - - 
  exit $rc
fi
