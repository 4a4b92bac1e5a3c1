# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: patch staging without a stream sync — update parity, C++ host tests,
# update bench; the wave-reach pass spread over every CU, with the level-store ablation)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r3g
mkdir -p $OUT
cd $R
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_update.py tests/test_cpp_host.py tests/test_gpu_reach.py -k "update or cpp or wreach" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
timeout -k 10 200 python3 bench.py --workload update --topology fabric --steps 40 --warmup 3 > $OUT/update$i.json 2> $OUT/update.err || { tail $OUT/update.err; exit 1; }
grep -o '"ms_per_step[^,]*\|"speedup[^,]*\|"full_resolve_ms[^,]*' $OUT/update$i.json | tr '\n' ' '; echo
done
for cfg in "OPENR_SPF_BFS_WREACH=1" "OPENR_SPF_BFS_WREACH=1 OPENR_SPF_WREACH_ABLATE=1" "OPENR_SPF_BFS_WREACH=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 scripts/batch_latency.py --sizes 1250,2500,5000,10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
  grep sources $OUT/lat.log | cut -c1-110
done
cd /tmp && export TMPDIR=/tmp
OPENR_SPF_BFS_WREACH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 1250,10000 --reps 10 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
python3 - <<'PY'
import csv, os
p = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r3g/kernel_stats.csv"
for r in list(csv.DictReader(open(p)))[:10]:
    print(r["Name"][:70], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
PY
