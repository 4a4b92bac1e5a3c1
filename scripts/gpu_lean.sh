# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: KSP tracer ranking from rank-sorted in-edge records — KSP / update /
# route parity, the KSP2 counters on a 256-source sample, the full KSP2 bench line)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r3m
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_exact.py tests/test_gpu_multirank.py tests/test_gpu_update.py tests/test_cpp_host.py -k "ksp or kth or Ksp or update or cpp or config5 or multirank" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OPENR_SPF_KSP_STATS=1 timeout -k 10 300 python3 bench.py --workload ksp2 --ksp-sources 256 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/ksp.json 2> $OUT/ksp.err || { tail $OUT/ksp.err; exit 1; }
grep ksp_stats $OUT/ksp.err | tail -4
grep -o '"ms_per_step[^,]*' $OUT/ksp.json
timeout -k 10 300 python3 bench.py --workload ksp2 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/ksp_full.json 2> $OUT/ksp_full.err || { tail $OUT/ksp_full.err; exit 1; }
grep -o '"ms_per_step[^,]*\|"value[^,]*' $OUT/ksp_full.json
