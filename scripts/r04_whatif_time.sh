#!/bin/bash
# What-if WAN step only (two bench runs), for A/B of a build.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp > gpurun_out/whatif_b.log 2>&1 || { tail -5 gpurun_out/whatif_b.log; exit 1; }
  echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/whatif_b.log) $(grep -o '"kernel_ms_mean": [0-9.]*' gpurun_out/whatif_b.log | head -1)"
done
