# Scratch GPU experiment script: rewritten for each measurement and run as
#   gpurun -- bash scripts/gpu_lean.sh
# (its last contents: the 1 024-thread code-family shape for tiny batches and the two-chunk
# wave pass — parity, the update loop with the wide shape on / off, G100 shard latency
# with the unroll on / off)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/r3j
mkdir -p $OUT
PYT="python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_update.py tests/test_gpu_parity.py tests/test_cpp_host.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OPENR_SPF_WAVE_UNROLL=2 timeout -k 10 300 $PYT tests/test_gpu_configs.py tests/test_gpu_reach.py -k "wave or shard or lean or partial" > $OUT/tests2.log 2>&1 || { tail -40 $OUT/tests2.log; exit 1; }
tail -1 $OUT/tests2.log
for cfg in "OPENR_SPF_BFS_WIDE=1" "OPENR_SPF_BFS_WIDE=0"; do
env $cfg timeout -k 10 200 python3 bench.py --workload update --topology fabric --steps 40 --warmup 4 --no-cpu-baseline > $OUT/update.json 2> $OUT/update.err || { tail $OUT/update.err; exit 1; }
echo "$cfg $(grep -o '"ms_per_step[^,]*\|"speedup[^,]*\|"full_resolve_ms[^,]*' $OUT/update.json | tr '\n' ' ')"
done
for cfg in "OPENR_SPF_WAVE_UNROLL=1" "OPENR_SPF_WAVE_UNROLL=2" "OPENR_SPF_WAVE_UNROLL=2 OPENR_SPF_BFS_WAVE=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 scripts/batch_latency.py --sizes 640,1250,2500,5000,10000 --reps 10 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 1; }
  grep sources $OUT/lat.log | cut -c1-110
done
