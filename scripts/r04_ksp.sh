#!/bin/bash
# KSP2: parity tests (every tier / chunk / tag mode), then the fabric sample step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -k "ksp or config5" tests/ > gpurun_out/ksp_tests.log 2>&1; rc=$?
echo "ksp tests rc=$rc"; tail -2 gpurun_out/ksp_tests.log
case $rc in 0) ;; *) grep -E "FAIL|Error|assert" gpurun_out/ksp_tests.log | head -20; exit $rc;; esac
bash scripts/r04_ksp_prof.sh
