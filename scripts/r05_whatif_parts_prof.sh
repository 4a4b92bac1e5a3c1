#!/bin/bash
# Kernel and copy trace of the what-if step in P source parts. Output: gpurun_out/r05/wp<P>/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
P=${PARTS:-2}; O="$R/gpurun_out/r05/wp$P"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
OPENR_SPF_WHATIF_PARTS=$P timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$O/trace" -o run \
  --output-format csv -- python3 "$R/bench.py" --workload whatif --no-cpu-baseline --no-ucmp > "$O/bench.log" 2>&1 || exit $?
for f in $(find "$O/trace" -name "*_stats.csv"); do
  echo "== $f"
  python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(r["Name"][:80], r["Calls"], r["AverageNs"][:9], r["TotalDurationNs"])
PY
done
