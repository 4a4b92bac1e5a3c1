# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: multi-source BFS pass timing + SQ counters at the full G100 batch)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/msprof
mkdir -p $OUT
cd $R
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_reach.py -k "msbfs" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python3 scripts/batch_latency.py --sizes 10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
grep sources $OUT/lat.log
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 10000 --reps 2 > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "msbfs" not in r.get("Kernel_Name", ""): continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
with open(out + "/sq_counters.txt", "w") as fo:
    for k in sorted(tot):
        line = f"{k:28s} {tot[k]/max(1,n[k]):.4g} per-dispatch-row (rows {n[k]})"
        print(line); fo.write(line + "\n")
PY
