# Kernel-trace breakdown of the WAN what-if step (default knobs and one variant).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in def l0; do
  if [ $v = l0 ]; then export OPENR_SPF_WHATIF_LIST=0 OPENR_SPF_ROUNDS_BLOCK=256; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$v -o run --output-format csv -- python3 bench.py --workload whatif --steps 5 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/tr_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/tr_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
print('$v', 'total kernel ms per step', sum(float(x['TotalDurationNs']) for x in r)/1e6/6)
for x in r[:9]: print('  ', x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1), 'us')"
done
