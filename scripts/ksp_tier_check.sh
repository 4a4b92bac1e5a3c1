#!/bin/bash
# KSP2 capacity tiers: parity tests, then the sampled fabric bench with and without the
# small tier (OPENR_SPF_KSP_TIER=0 = full capacities only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/ksp_tier
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "ksp2" -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ksp_tier/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/ksp_tier/tests.log; exit 1; }
tail -1 gpurun_out/ksp_tier/tests.log
for t in 1; do
  OPENR_SPF_KSP_TIER=$t timeout -k 10 300 python -u bench.py --workload ksp2 --ksp-sources ${KSP_SOURCES:-256} --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/ksp_tier/bench_tier$t.log 2>&1 || exit 1
  echo "tier=$t $(grep '^{' gpurun_out/ksp_tier/bench_tier$t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
