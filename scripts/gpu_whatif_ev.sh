# What-if evidence on HEAD: config-4 parity tests, bench line + rocprof + PMC.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "whatif" > gpurun_out/whatif_tests.log 2>&1 || { tail -30 gpurun_out/whatif_tests.log; exit 1; }
tail -1 gpurun_out/whatif_tests.log
cd "$R" && TAG=r03i bash scripts/workload_profile.sh whatif || exit $?
# KSP2 trace counters (OPENR_SPF_PROF=1) on a 256-source sample
OPENR_SPF_PROF=1 timeout -k 10 200 python -u bench.py --workload ksp2 --topology fabric --ksp-sources 256 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ksp_stats.log 2>&1 || exit 1
grep ksp_stats gpurun_out/ksp_stats.log | tail -4
