# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: the 2-bit-code lean pass — parity on its own cases and on the full
# G100 batch, then G100 latency with it on and off)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r3k
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "lean2" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 $PYT tests/test_gpu_configs.py -k "lean2" > $OUT/tests2.log 2>&1 || { tail -40 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
for cfg in "OPENR_SPF_BFS_LEAN2=1" "OPENR_SPF_BFS_LEAN2=0" "OPENR_SPF_BFS_LEAN2=1 OPENR_SPF_BFS_WAVE=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 scripts/batch_latency.py --sizes 1250,2500,5000,10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
  grep sources $OUT/lat.log | cut -c1-110
done
