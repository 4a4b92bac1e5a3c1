#!/bin/bash
# Round 4 bench evidence: G100 and fabric all-sources (PMC, bench line, rocprof summary),
# then KSP2 (all pairs) and the fabric update loop. Output under gpurun_out/r04/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
TAG=r04 TOPO=grid100 bash scripts/round_profile.sh || exit $?
TAG=r04 TOPO=fabric bash scripts/round_profile.sh || exit $?
TAG=r04 ROUND=r04 bash scripts/workload_profile.sh ksp2 update || exit $?
