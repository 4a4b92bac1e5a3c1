# Scratch GPU experiment script: rewritten for each A/B measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/full_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/full_tests.log | head; tail -30 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/g100prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/g100prof.log 2>&1 || exit 1
grep '^{' $R/gpurun_out/g100prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_mean'])"
f=$(find $R/gpurun_out/g100prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])): print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" $f > $R/gpurun_out/g100prof.txt; head -4 $R/gpurun_out/g100prof.txt
