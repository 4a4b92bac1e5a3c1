# Round evidence on one box: smoke + full GPU suite, then the G100 and fabric bench lines
# with their rocprofv3 kernel-trace summaries and PMC traffic (TAG names the output dir).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
SKIP_BENCH=1 bash scripts/gpu_check.sh || exit $?
for T in ${TOPOS:-grid100 fabric}; do
  TAG=${TAG:-r02} TOPO=$T bash scripts/round_profile.sh || exit $?
done
