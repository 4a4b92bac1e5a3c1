#!/bin/bash
# What-if in source parts (OPENR_SPF_WHATIF_PARTS): parity of every what-if mode, then the
# WAN step at P = 1, 2, 3, 4. Output: gpurun_out/r05/whatif_srcparts/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05/whatif_srcparts"; mkdir -p "$O" && cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -k "whatif or config4" tests/ \
  > "$O/tests.log" 2>&1; rc=$?
echo "whatif tests rc=$rc"; tail -1 "$O/tests.log"
[ $rc = 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; exit $rc; }
for P in ${PARTS:-1 2 3 4}; do
  OPENR_SPF_WHATIF_PARTS=$P timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp \
    > "$O/bench_p$P.log" 2>&1 || { tail -5 "$O/bench_p$P.log"; exit 1; }
  echo "P=$P $(grep -o '"ms_per_step": [0-9.]*' "$O/bench_p$P.log")"
done
