#!/bin/bash
# GPU-box check: smoke -> parity tests -> short bench. Stops on a GPU fault/timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_on_fault() { case $1 in 124|137|134|139) echo "GPU step faulted/timed out (rc=$1); stopping"; exit $1;; esac; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_on_fault $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -3; stop_on_fault $rc
if grep -qiE "illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure" gpurun_out/gpu_tests.log; then
  echo "GPU fault reported inside the tests; stopping"; exit 3
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; stop_on_fault $rc
fi
exit 0
