# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: tile-active multi-source BFS with LDS neighbour lists — parity of the
# all-sources passes, then G100 batch latency of the tile / dense / lean passes and a trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3b
mkdir -p $OUT
cd $R
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_reach.py tests/test_gpu_configs.py -k "reach or config3" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 $PYT tests/test_gpu_update.py tests/test_cpp_host.py > $OUT/tests2.log 2>&1 || { tail -40 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
timeout -k 10 120 tests/cpp/build/linkstate_test gpu > $OUT/ls.log 2>&1; grep -E "weighted|FAIL|failures" $OUT/ls.log
timeout -k 10 200 python3 bench.py --workload update --topology fabric --steps 20 --warmup 2 --no-cpu-baseline > $OUT/update.json 2> $OUT/update.err || { tail $OUT/update.err; exit 1; }
cut -c1-300 $OUT/update.json; grep -o '"speedup_vs_full_resolve": [0-9.]*\|"mean_rows_resolved": [0-9.]*' $OUT/update.json
for cfg in "OPENR_SPF_MSBFS_TILE=1" "OPENR_SPF_MSBFS_TILE=0" "OPENR_SPF_BFS_MSBFS=0" "OPENR_SPF_BFS_MSBFS=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 scripts/batch_latency.py --sizes 640,1250,2500,10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
  grep sources $OUT/lat.log | cut -c1-110
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 10000 --reps 10 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" | head -5
