set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=r01c TOPO=grid100 bash scripts/round_profile.sh && TAG=r01c TOPO=fabric bash scripts/round_profile.sh
