set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_update.py tests/test_gpu_configs.py -k "wave or grid or update or overload or config3 or config1" > gpurun_out/wave_tests.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/wave_tests.log | head; tail -30 gpurun_out/wave_tests.log; exit 1; }
tail -2 gpurun_out/wave_tests.log
OPENR_SPF_BFS_WAVE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "grid or random or lean" > gpurun_out/wave_tests2.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/wave_tests2.log | head; tail -30 gpurun_out/wave_tests2.log; exit 1; }
tail -2 gpurun_out/wave_tests2.log
for sp in 0 1; do
OPENR_SPF_WAVE_SPEC=$sp OPENR_SPF_BFS_WAVE=1 timeout -k 10 200 python -u scripts/batch_latency.py --sizes 640,1250,2500,5000,10000 --reps 10 > gpurun_out/wave_bl$sp.log 2>&1 || { tail -20 gpurun_out/wave_bl$sp.log; exit 1; }
echo "SPEC=$sp"; cut -c1-120 gpurun_out/wave_bl$sp.log | grep sources
done
