#!/bin/bash
# KSP2 small-tier capacity sweep on the sampled fabric bench (tuning aid).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out/ksp_sweep
for v in "default" "OPENR_SPF_KSP_SMALL_ARENA=384" "OPENR_SPF_KSP_SMALL_ARENA=256" "OPENR_SPF_KSP_SMALL_ARENA=320" "OPENR_SPF_KSP_SMALL_ARENA=448" \
         "OPENR_SPF_KSP_SMALL_ARENA=256 OPENR_SPF_KSP_SMALL_FRAMES=8" "OPENR_SPF_KSP_TIER=0" "default"; do
  envs=""; [ "$v" != "default" ] && envs="$v"
  env $envs timeout -k 10 300 python -u bench.py --workload ksp2 --ksp-sources ${KSP_SOURCES:-256} --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/ksp_sweep/b.log 2>&1 || exit 1
  echo "$v: $(grep '^{' gpurun_out/ksp_sweep/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],1), round(d["value"]))')"
done
