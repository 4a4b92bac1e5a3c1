#!/bin/bash
# What-if: parity of every mode (incl. the seeded re-solves), then the WAN step
# (and, with PROF=1, the re-solves' per-phase profile).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -k "whatif or config4" tests/ > gpurun_out/whatif_tests.log 2>&1; rc=$?
echo "whatif tests rc=$rc"; tail -2 gpurun_out/whatif_tests.log
case $rc in 0) ;; *) grep -E "FAIL|Error|assert" gpurun_out/whatif_tests.log | head -20; exit $rc;; esac
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp > gpurun_out/whatif_b.log 2>&1 || { tail -5 gpurun_out/whatif_b.log; exit 1; }
  echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/whatif_b.log) $(grep -o '"kernel_ms_mean": [0-9.]*' gpurun_out/whatif_b.log | head -1)"
done
if [ "${PROF:-0}" = 1 ]; then
  OPENR_SPF_PROF=1 timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp --steps 3 --warmup 1 > gpurun_out/wprof.log 2>&1 || { tail -5 gpurun_out/wprof.log; exit 1; }
  grep -A1 "whatif resolve" gpurun_out/wprof.log | tail -2
fi
