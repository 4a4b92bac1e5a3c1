#!/bin/bash
# Round-4 host route-build check on the GPU: the C++ drop-in suites, DecisionBenchmark
# cases and the all-node route build (G100) after the route-build fast path.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for t in decision_test linkstate_test; do
  timeout -k 10 300 tests/cpp/build/$t gpu > gpurun_out/$t.log 2>&1; rc=$?; echo "$t rc=$rc"
  grep -E "FAIL|failures" gpurun_out/$t.log | tail -6
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 600 python3 -u bench.py --workload decision --steps 10 --warmup 2 \
  --decision-cases grid:10000:sp,fabric:5000:sp,grid:1024:ksp2 > gpurun_out/decision.log 2>&1; rc=$?
echo "decision rc=$rc"; grep -o '"config": {[^}]*}\|"ms_per_update": [0-9.]*\|"ms_update_adjdb": [0-9.]*\|"ms_build_route_db": [0-9.]*\|"check": "[^"]*"' gpurun_out/decision.log
case $rc in 0) ;; *) tail -c 2000 gpurun_out/decision.log; exit $rc;; esac
timeout -k 10 300 python3 -u bench.py --workload routes --topology grid100 --steps 2 > gpurun_out/routes.log 2>&1; rc=$?
echo "routes rc=$rc"; tail -c 1500 gpurun_out/routes.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python3 -u bench.py --workload routes --topology grid100 --steps 2 --lfa > gpurun_out/routes_lfa.log 2>&1; rc=$?
echo "routes lfa rc=$rc"; tail -c 1500 gpurun_out/routes_lfa.log
exit $rc
