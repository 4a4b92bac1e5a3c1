#!/bin/bash
# KSP2 small-tier arena sweep on the all-pairs fabric step (after the packed arena and the
# profiling-only stats slot). Output: gpurun_out/r05/ksparena/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05/ksparena"; mkdir -p "$O" && cd "$R"
for A in ${ARENAS:-default 192 128}; do
  if [ "$A" = default ]; then unset OPENR_SPF_KSP_SMALL_ARENA; else export OPENR_SPF_KSP_SMALL_ARENA=$A; fi
  timeout -k 10 300 python3 -u bench.py --workload ksp2 --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench_a$A.log" 2>&1 || exit $?
  echo "arena=$A $(grep -o '"ms_per_step": [0-9.]*' "$O/bench_a$A.log")"
done
