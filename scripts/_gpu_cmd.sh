set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/ -m gpu -k "ksp or KSP or fabric_faults" > gpurun_out/ksp_tests.log 2>&1 || { tail -30 gpurun_out/ksp_tests.log; exit 1; }
tail -2 gpurun_out/ksp_tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload ksp2 --topology fabric --ksp-sources 256 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_ksp.log 2>&1 || { tail -20 gpurun_out/b_ksp.log; exit 1; }
grep '^{' gpurun_out/b_ksp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ksp', d['ms_per_step'], d['value'])"
done
