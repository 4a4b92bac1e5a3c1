#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for t in decision_test linkstate_test; do
  timeout -k 10 300 tests/cpp/build/$t gpu > gpurun_out/$t.log 2>&1; rc=$?; echo "$t rc=$rc"; grep -E "FAIL|failures" gpurun_out/$t.log | tail -4
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 300 python3 -u scripts/rss_probe.py > gpurun_out/rss.log 2>&1; rc=$?; echo "rss rc=$rc"; grep -v amdgpu.ids gpurun_out/rss.log
case $rc in 0) ;; *) exit $rc;; esac
for lfa in "" "--lfa"; do
  timeout -k 10 300 python3 -u bench.py --workload routes --topology grid100 --steps 2 $lfa > gpurun_out/routes$lfa.log 2>&1; rc=$?
  echo "routes $lfa rc=$rc"; grep -o '"ms_per_step": [0-9.]*\|"checksum": "[0-9a-f]*"\|"peak_rss_mb": [0-9.]*' gpurun_out/routes$lfa.log
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 600 python3 -u bench.py --workload decision --steps 10 --warmup 2 \
  --decision-cases grid:10000:sp,fabric:5000:sp,grid:1024:ksp2,grid:10000:ksp2 > gpurun_out/decision.log 2>&1; rc=$?
echo "decision rc=$rc"; grep -o '"ms_per_update": [0-9.]*\|"check": "[^"]*"' gpurun_out/decision.log
exit $rc
