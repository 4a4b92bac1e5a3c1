# What-if repair A/B on one box: parity tests, then the WAN step under repair knobs
# (dirty-slot cap and waves per workgroup change the LDS per wave, i.e. occupancy).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "whatif_wan_sample" > gpurun_out/whatif_tests.log 2>&1 || { tail -30 gpurun_out/whatif_tests.log; exit 1; }
tail -2 gpurun_out/whatif_tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --workload whatif --steps 5 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/b_whatif_$name.log 2>&1 || { tail -20 gpurun_out/b_whatif_$name.log; exit 1; }
  grep '^{' gpurun_out/b_whatif_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('whatif', '$name', round(d['ms_per_step'],3), round(d['roofline'].get('kernel_ms_mean'),3))"
}
run base OPENR_SPF_NOOP=1
run w5 OPENR_SPF_WHATIF_WAVES=5
run w6 OPENR_SPF_WHATIF_WAVES=6
run c144 OPENR_SPF_WHATIF_CAP=144
run c128w5c144 OPENR_SPF_WHATIF_CAP=144 OPENR_SPF_WHATIF_WAVES=5
run base2 OPENR_SPF_NOOP=1
OPENR_SPF_WHATIF_PROF=1 timeout -k 10 200 python -u bench.py --workload whatif --steps 2 --warmup 1 --no-cpu-baseline --no-ucmp > gpurun_out/b_whatif_prof.log 2>&1 || exit 1
grep "^whatif_group" gpurun_out/b_whatif_prof.log | tail -2
