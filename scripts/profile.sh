#!/bin/bash
# rocprofv3 kernel-trace summary (+ optional PMC passes) of the bench command.
#   PROF_TAG=r01 PMC=1 BENCH_ARGS="--topology grid100" bash scripts/profile.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${PROF_TAG:-prof}"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
BARGS="${BENCH_ARGS:---steps 10 --warmup 2} --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" $BARGS > "$OUT/trace_bench.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 "$OUT/trace_bench.log"
case $rc in 0) ;; *) exit $rc;; esac
if [ -n "${PMC:-}" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$OUT/pmc_$ctr" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_TOPO:-} > "$OUT/pmc_$ctr.log" 2>&1
    rc=$?; echo "pmc $ctr rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
fi
find "$OUT" -name "*stats*.csv" -o -name "*counter_collection*.csv" | head -20
exit 0
