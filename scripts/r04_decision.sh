#!/bin/bash
# DecisionBenchmark lines (bench.py --workload decision, every default case) after the
# C++ decision / linkstate GPU suites.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for t in decision_test linkstate_test; do
  timeout -k 10 300 tests/cpp/build/$t gpu > gpurun_out/$t.log 2>&1; rc=$?; echo "$t rc=$rc"; tail -1 gpurun_out/$t.log
  case $rc in 0) ;; *) grep FAIL gpurun_out/$t.log | head; exit $rc;; esac
done
timeout -k 10 900 python3 -u bench.py --workload decision --steps 10 --warmup 2 > gpurun_out/decision.log 2>&1; rc=$?
echo "decision rc=$rc"; grep '^{' gpurun_out/decision.log > gpurun_out/decision.jsonl
grep -o '"workload": "BM[^"]*"\|"ms_per_update": [0-9.]*\|"check": "[^"]*"' gpurun_out/decision.log
exit $rc
