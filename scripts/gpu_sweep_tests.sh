#!/bin/bash
# GPU box: kernel-variant sweep (scripts/sweep.py) then a pytest selection; stops on a fault.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 300 python -u scripts/sweep.py --topology ${TOPO:-grid100} --rounds ${ROUNDS:-7} --variants "$SWEEP" > gpurun_out/sweep.log 2>&1
  rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep.log | grep -v amdgpu.ids | tail -12
  case $rc in 0) ;; *) exit $rc;; esac
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/tests.log
  exit $rc
fi
