#!/bin/bash
# Bench evidence of a round (ROUND=r06 by default): for each workload the bench line (CPU baseline included; the
# bench reads the tracked profiles/$ROUND PMC summaries) and the rocprofv3 kernel-trace summary
# of the same command without the CPU leg. Output: gpurun_out/$ROUND/ev/<name>/.
#   ROUND=r06 bash scripts/evidence.sh grid100 fabric grid10 whatif update ksp2 routes decision
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROUND="${ROUND:-r06}"
stop() { case $1 in 0) ;; *) echo "step failed rc=$1; stopping"; exit $1;; esac; }
export TMPDIR=/tmp
for W in "$@"; do
  OUT="$R/gpurun_out/$ROUND/ev/$W"
  mkdir -p "$OUT"
  case $W in
    grid100) ARGS="" ;;
    fabric)  ARGS="--topology fabric" ;;
    grid10)  ARGS="--topology grid10" ;;
    whatif)  ARGS="--workload whatif --steps 20 --warmup 3" ;;
    update)  ARGS="--workload update --topology fabric --steps 20 --warmup 2" ;;
    ksp2)    ARGS="--workload ksp2 --steps 2 --warmup 1" ;;
    routes)  ARGS="--workload routes --steps 3 --warmup 1" ;;
    decision) ARGS="--workload decision --steps 10 --warmup 2" ;;
    *) echo "unknown workload $W"; exit 2 ;;
  esac
  cd "$R" && timeout -k 10 1000 python3 -u bench.py $ARGS > "$OUT/bench.log" 2>&1; stop $?
  grep '^{' "$OUT/bench.log" > "$OUT/bench.jsonl"; echo "$W: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench.jsonl" | tr '\n' ' ')"
  case $W in decision|routes) continue ;; esac  # host-dominated lines: no kernel trace
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/trace_bench.log" 2>&1; stop $?
  f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && head -3 "$OUT/kernel_stats.csv" | cut -c1-160
done
