# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: fabric all-sources with its source classes on side streams)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r3o
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
OPENR_SPF_CLASS_STREAMS=2 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_configs.py -k "fabric or class or sliced or hub" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 0 2 0 2; do
OPENR_SPF_CLASS_STREAMS=$c timeout -k 10 300 python3 bench.py --topology fabric --steps 20 --warmup 3 --no-cpu-baseline > $OUT/fab_$c.json 2> $OUT/fab_$c.err || { tail $OUT/fab_$c.err; exit 1; }
echo "streams=$c $(grep -o '"ms_per_step[^,]*\|"kernel_ms_mean[^,]*' $OUT/fab_$c.json | tr '\n' ' ')"
done
