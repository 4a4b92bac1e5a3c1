#!/bin/bash
# Evidence for the non-default bench workloads (BASELINE configs 4 and 5, and the
# incremental-update loop): one bench line each plus the rocprofv3 kernel-trace summary
# of the same command. Output: gpurun_out/<TAG>/<workload>/.
#   TAG=r01c bash scripts/workload_profile.sh [ksp2|whatif|update ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-prof}"
WORKLOADS="${*:-ksp2 whatif update}"
ROUND="${ROUND:-r03}"
stop() { case $1 in 0) ;; *) echo "step failed rc=$1; stopping"; exit $1;; esac; }
export TMPDIR=/tmp
for W in $WORKLOADS; do
  OUT="$R/gpurun_out/$TAG/$W"
  mkdir -p "$OUT"
  case $W in
    ksp2)   ARGS="--workload ksp2 --steps 2 --warmup 1" ;;       # all 24.9 M fabric pairs per step
    whatif) ARGS="--workload whatif --steps 5 --warmup 1" ;;     # all 3 M WAN (link, source) units
    update) ARGS="--workload update --topology fabric --steps 20 --warmup 2" ;;
    adjdb)  ARGS="--workload adjdb --steps 5 --warmup 1" ;;                    # G100 full adj: sync
    routes) ARGS="--workload routes --steps 3 --warmup 1" ;;                   # every G100 node's route DB
    routes_lfa) ARGS="--workload routes --lfa --steps 3 --warmup 1" ;;
    adjdb_fabric) ARGS="--workload adjdb --topology fabric --steps 5 --warmup 1" ;;
    *) echo "unknown workload $W"; exit 2 ;;
  esac
  # PMC HBM traffic first (what-if: its repair kernel; KSP2: every engine kernel of a step,
  # on a 64-source sample), installed where bench.py reads it (profiles/$ROUND/)
  PMC=""
  case $W in
    whatif) PMC="PMC_KERNEL=whatif_group|--workload whatif --no-ucmp" ;;
    ksp2)   PMC="PMC_AGG=1|--workload ksp2 --ksp-sources 64" ;;
  esac
  if [ -n "$PMC" ] && [ -z "${NO_PMC:-}" ]; then
    env ${PMC%%|*} PMC_TAG="$TAG/$W/pmc" BENCH_ARGS="${PMC#*|}" bash "$R/scripts/pmc_traffic.sh"; stop $?
    mkdir -p "$R/profiles/$ROUND" && cp "$R/gpurun_out/pmc_$TAG/$W/pmc/pmc_traffic.json" "$R/profiles/$ROUND/pmc_traffic_$W.json"
    cp "$R/gpurun_out/pmc_$TAG/$W/pmc/pmc_traffic.json" "$OUT/pmc_traffic.json"
  fi
  cd "$R" && timeout -k 10 400 python3 -u bench.py $ARGS > "$OUT/bench.log" 2>&1; stop $?
  grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"; cat "$OUT/bench.json"
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS --no-cpu-baseline > "$OUT/trace_bench.log" 2>&1; stop $?
  f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" "$OUT/kernel_stats.csv" && head -6 "$OUT/kernel_stats.csv" | cut -c1-200
  rm -rf "$OUT/trace"
done
exit 0
