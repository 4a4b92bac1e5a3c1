# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: all-sources level-pass parity tests (multi-source BFS and reach
# pass), then kernel times of the all-sources G100 launch per pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/msbfs
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reach.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for cfg in "" "OPENR_SPF_REACH_DIST=2" "OPENR_SPF_BFS_MSBFS=0"; do
  env $cfg timeout -k 10 120 python3 scripts/batch_latency.py --sizes 10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
  echo "$cfg: $(grep sources $OUT/lat.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 10000 --reps 10 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')): print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
