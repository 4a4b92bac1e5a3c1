set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "ksp or kth or distance_only" > gpurun_out/ksp_tests.log 2>&1 || { tail -30 gpurun_out/ksp_tests.log; exit 1; }
tail -2 gpurun_out/ksp_tests.log
for p in 64; do
  echo "== probe $p"
  OPENR_SPF_KSP_STATS=1 OPENR_SPF_KSP_PROBE=$p timeout -k 10 200 python -u bench.py --workload ksp2 --ksp-sources 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ksp_st_$p.log 2>&1 || exit $?
  grep -E "ksp_stats|^\{" gpurun_out/ksp_st_$p.log | tail -3 | cut -c1-300
done
