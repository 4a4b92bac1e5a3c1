set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/sweep.py --topology grid100 --variants "FAM=lvl;WGS=9;WGS=10,BLK=128" --rounds 5 > gpurun_out/sweep.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/sweep.py --topology fabric --variants "FAM=code;WGS=8;WGS=4;BLK=256" --rounds 3 > gpurun_out/sweepf.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/sweepf.log; exit $rc
