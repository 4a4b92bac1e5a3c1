#!/bin/bash
# One GPU call's worth of round evidence for a topology: the bench line (with the CPU
# baseline), the rocprofv3 kernel-trace summary of the same command, and the PMC HBM
# traffic passes. Everything lands in gpurun_out/<tag>/ (copy to profiles/<round>/).
#   TAG=r01 TOPO=grid100 bash scripts/round_profile.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-prof}"
TOPO="${TOPO:-grid100}"
OUT="$R/gpurun_out/$TAG/$TOPO"
mkdir -p "$OUT"
stop() { case $1 in 0) ;; *) echo "step failed rc=$1; stopping"; exit $1;; esac; }
# 1) PMC traffic first, so the bench line below can carry it: every engine kernel of a
#    step (PMC_AGG=1: an all-sources call is several launches — classes, re-runs, merges)
PMC_AGG=1 PMC_TAG="$TAG/$TOPO/pmc" BENCH_ARGS="--topology $TOPO" bash "$R/scripts/pmc_traffic.sh"; stop $?
cp "$R/gpurun_out/pmc_$TAG/$TOPO/pmc/pmc_traffic.json" "$OUT/pmc_traffic.json"
# 2) bench line (default steps/warmup, CPU baseline included)
cd "$R" && timeout -k 10 300 python3 -u bench.py --topology "$TOPO" --traffic-json "$OUT/pmc_traffic.json" \
  > "$OUT/bench.log" 2>&1; stop $?
grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"; cat "$OUT/bench.json"
# 3) kernel-trace summary of the same bench command (without the CPU leg)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --topology "$TOPO" --no-cpu-baseline --traffic-json "$OUT/pmc_traffic.json" \
  > "$OUT/trace_bench.log" 2>&1; stop $?
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && head -4 "$OUT/kernel_stats.csv" | cut -c1-220
exit 0
