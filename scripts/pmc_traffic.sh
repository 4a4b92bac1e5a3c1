#!/bin/bash
# HBM traffic of the bench's dominant kernel from rocprofv3 PMC counters, one pass per
# counter (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: they cannot share a pass).
#   PMC_TAG=r01 BENCH_ARGS="--topology grid100" bash scripts/pmc_traffic.sh
# Writes gpurun_out/pmc_<tag>/pmc_traffic.json (copy it to profiles/<round>/).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_${PMC_TAG:-x}"
mkdir -p "$OUT"
BARGS="${BENCH_ARGS:-} --steps 3 --warmup 1 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$OUT/$ctr" -o run --output-format csv -- \
    python3 "$R/bench.py" $BARGS > "$OUT/$ctr.log" 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/$ctr.log"; exit $rc;; esac
done
python3 "$R/scripts/pmc_summary.py" "$OUT" $BARGS > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
