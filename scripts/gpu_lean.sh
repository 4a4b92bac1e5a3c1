# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: round-3 new paths — tile-active multi-source BFS, dense LinkState
# memo with in-place patches, compact gather, tagged KSP2 rows — parity first, then G100
# batch latency of the passes, a kernel trace, and the default and KSP2 bench lines)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3a
mkdir -p $OUT
cd $R
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_reach.py tests/test_gpu_configs.py -k "reach or config3" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 $PYT tests/test_cpp_host.py tests/test_gpu_multirank.py tests/test_gpu_parity.py -k "cpp or multirank or engine_ranks or context or ksp2" > $OUT/tests2.log 2>&1 || { tail -60 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
timeout -k 10 120 tests/cpp/build/linkstate_test gpu > $OUT/ls.log 2>&1; grep -E "weighted|FAIL|failures" $OUT/ls.log
for cfg in "OPENR_SPF_MSBFS_TILE=1" "OPENR_SPF_MSBFS_TILE=0" "OPENR_SPF_BFS_MSBFS=0" "OPENR_SPF_REACH_DIST=2"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 scripts/batch_latency.py --sizes 1250,2500,10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
  grep sources $OUT/lat.log
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
timeout -k 10 300 python3 bench.py --workload ksp2 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/ksp2.json 2> $OUT/ksp2.err || { tail $OUT/ksp2.err; exit 1; }
cut -c1-400 $OUT/ksp2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 10000 --reps 10 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')): print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
