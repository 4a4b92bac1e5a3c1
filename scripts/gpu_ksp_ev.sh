# KSP2 evidence on HEAD: KSP parity tests, then the all-pairs line + rocprof (+ PMC).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multirank.py -m gpu -k "ksp or kth or config5" > gpurun_out/ksp_tests.log 2>&1 || { tail -30 gpurun_out/ksp_tests.log; exit 1; }
tail -1 gpurun_out/ksp_tests.log
cd "$R" && TAG=r03j bash scripts/workload_profile.sh ksp2 || exit $?
