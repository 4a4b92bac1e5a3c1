set -o pipefail
O=gpurun_out/r06/g7; mkdir -p $O
timeout -k 10 300 python3 -u bench.py --workload ksp2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ksp2.log 2>&1 || { tail $O/ksp2.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/ksp2.log; grep -o '"check": {[^}]*}' $O/ksp2.log
timeout -k 10 200 python3 -u bench.py --topology fabric --no-cpu-baseline > $O/fab.log 2>&1 || { tail $O/fab.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/fab.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "ksp or fabric or config5 or config2 or reach or random" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
