set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for ns in 0 1; do
OPENR_SPF_NBR_NOSTORE=$ns timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/nbrprof3_$ns -o run --output-format csv -- python3 $R/bench.py --topology fabric --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/nbrprof3.log 2>&1 || exit 1
f=$(find $R/gpurun_out/nbrprof3_$ns -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" $f | grep nbr_nh
done
