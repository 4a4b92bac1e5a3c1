#!/bin/bash
# GPU box: the config-named parity tests + multi-rank tests, then a default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py tests/test_gpu_multirank.py} -m gpu -v -x \
  --timeout 300 --timeout-method thread > gpurun_out/new_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/new_tests.log | tail -20
case $rc in 124|137|134|139) exit $rc;; esac
[ -n "${SKIP_BENCH:-}" ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_new.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -1 gpurun_out/bench_new.log
exit $rc
