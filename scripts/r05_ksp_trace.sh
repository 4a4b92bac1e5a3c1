#!/bin/bash
# Kernel-trace summary of the KSP2 all-pairs fabric step (current tree). Output: gpurun_out/r05/ksptrace/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r05/ksptrace"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload ksp2 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace_bench.log" 2>&1 || exit $?
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "$OUT/kernel_stats.csv"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r['Name'][:100], r['Calls'], round(int(r['TotalDurationNs'])/1e6, 1), r['Percentage'])
PY
