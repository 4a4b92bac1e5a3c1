set -o pipefail
mkdir -p gpurun_out
OPENR_SPF_WAVE_PRED=1 OPENR_SPF_BFS_WAVE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wave or grid" > gpurun_out/wave_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/wave_tests.log | head; tail -30 gpurun_out/wave_tests.log; exit 1; }
tail -2 gpurun_out/wave_tests.log
for p in 0 1 0 1; do
OPENR_SPF_WAVE_PRED=$p OPENR_SPF_BFS_WAVE=1 timeout -k 10 200 python -u scripts/batch_latency.py --sizes 640,1250,2500 --reps 10 > gpurun_out/wave_bl.log 2>&1 || { tail -20 gpurun_out/wave_bl.log; exit 1; }
echo PRED=$p; cut -c1-110 gpurun_out/wave_bl.log | grep sources
done
