# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: kernel trace + SQ counters of the wave pass on a G100 shard of
# 1 250 sources, the per-GPU step of an 8-GPU strong-scaling run)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/shard1250
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 1250 --reps 20 > $OUT/trace.log 2>&1 || exit 1
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
grep sources $OUT/trace.log | cut -c1-160
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $R/scripts/batch_latency.py --sizes 1250 --reps 3 > $OUT/p$i.log 2>&1 || exit 1
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bfs_wave" not in r.get("Kernel_Name", ""): continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
with open(out + "/sq_counters.txt", "w") as fo:
    for k in sorted(tot):
        line = f"{k:28s} {tot[k]/max(1,n[k]):.4g} per-dispatch-row (rows {n[k]})"
        print(line); fo.write(line + "\n")
PY
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" | head -3
