# Round evidence on HEAD: G100 bench line + rocprof + PMC, what-if and KSP2 lines + rocprof
# + PMC, full GPU suite. Output under gpurun_out/r03h/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG=r03h TOPO=grid100 bash scripts/round_profile.sh || exit $?
cd "$R" && TAG=r03h bash scripts/workload_profile.sh whatif ksp2 || exit $?
cd "$R" && SKIP_BENCH=1 bash scripts/gpu_check.sh || exit $?
