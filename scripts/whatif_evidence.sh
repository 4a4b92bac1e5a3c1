#!/bin/bash
# What-if evidence (ROUND=r06 by default): parity of every mode, the WAN step twice, then the repair kernel's PMC
# traffic (FETCH_SIZE / WRITE_SIZE passes) and a rocprofv3 kernel-trace summary.
# Output under gpurun_out/${ROUND:-r06}/whatif/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${ROUND:-r06}/whatif"
mkdir -p "$O" && cd "$R"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -k "whatif or config4" tests/ > "$O/tests.log" 2>&1; rc=$?
  echo "whatif tests rc=$rc"; tail -2 "$O/tests.log"
  [ $rc = 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; exit $rc; }
fi
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --workload whatif --no-cpu-baseline --no-ucmp > "$O/bench_$i.log" 2>&1 || { tail -5 "$O/bench_$i.log"; exit 1; }
  echo "$(grep -o '"ms_per_step": [0-9.]*' "$O/bench_$i.log") $(grep -o '"kernel_ms_mean": [0-9.]*' "$O/bench_$i.log" | head -1)"
done
if [ "${PMC:-1}" = 1 ]; then
  PMC_TAG=${ROUND:-r06}_whatif PMC_KERNEL=whatif_group BENCH_ARGS="--workload whatif --no-ucmp" bash scripts/pmc_traffic.sh > "$O/pmc.log" 2>&1 || { tail -5 "$O/pmc.log"; exit 1; }
  cp "$R/gpurun_out/pmc_${ROUND:-r06}_whatif/pmc_traffic.json" "$O/pmc_traffic.json" && cat "$O/pmc_traffic.json"
fi
if [ "${ROCPROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload whatif --no-cpu-baseline --no-ucmp > "$O/rocprof.log" 2>&1 || { tail -5 "$O/rocprof.log"; exit 1; }
  f=$(find "$O/rocprof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$O/kernel_stats.csv" && head -6 "$O/kernel_stats.csv"
fi
