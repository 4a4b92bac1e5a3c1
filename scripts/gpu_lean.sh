# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: LDS copies of the traced second-SPF rows — KSP parity with the copy
# forced on, then the full KSP2 bench with OPENR_SPF_KSP_D16 = 0 / 2 / 1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r3n
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
OPENR_SPF_KSP_D16=2 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multirank.py -k "ksp or kth or Ksp or config5" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for d in 0 2 1; do
OPENR_SPF_KSP_D16=$d timeout -k 10 300 python3 bench.py --workload ksp2 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/ksp_$d.json 2> $OUT/ksp_$d.err || { tail $OUT/ksp_$d.err; exit 1; }
echo "d16=$d $(grep -o '"ms_per_step[^,]*' $OUT/ksp_$d.json)"
done
