#!/bin/bash
# What-if first-pass slot cap A/B after the seeded, fused re-solve (WAN step).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for c in 128 64 80 96 112 128; do
  OPENR_SPF_WHATIF_CAP=$c timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp > gpurun_out/wcap.log 2>&1 || { tail -5 gpurun_out/wcap.log; exit 1; }
  echo "cap=$c $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wcap.log) $(grep -o '"kernel_ms_mean": [0-9.]*' gpurun_out/wcap.log | head -1)"
done
