#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) for one kernel of a command.
#   BENCH_ARGS="--topology grid100" [KFILTER=kernel-name-substring] [SQ_TAG=name] bash scripts/sq_counters.sh
#   SQ_CMD="scripts/batch_latency.py --sizes 1250 --reps 3" KFILTER=bfs_wave SQ_TAG=shard bash scripts/sq_counters.sh
# (SQ_CMD: a python script + args run instead of bench.py)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/sq${SQ_TAG:+_$SQ_TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ -n "${SQ_CMD:-}" ]; then CMD="$R/$SQ_CMD"; else CMD="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"; fi
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- \
    python3 $CMD > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" "${KFILTER:-bfs_}" <<'PY' | tee "$OUT/summary.txt"
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] not in r.get("Kernel_Name", ""): continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(f"{k:28s} {tot[k]/max(1,n[k]):.4g} per-dispatch-row (rows {n[k]})")
PY
