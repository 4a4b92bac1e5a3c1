set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_update.py > gpurun_out/code_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/code_tests.log | head; tail -40 gpurun_out/code_tests.log; exit 1; }
tail -2 gpurun_out/code_tests.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fabprof -o run --output-format csv -- python3 $R/bench.py --topology fabric --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/fabprof.log 2>&1 || exit 1
grep '^{' $R/gpurun_out/fabprof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])"
f=$(find $R/gpurun_out/fabprof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])): print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" $f > $R/gpurun_out/fabprof.txt; head -5 $R/gpurun_out/fabprof.txt
