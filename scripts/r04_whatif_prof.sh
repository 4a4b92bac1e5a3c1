#!/bin/bash
# rocprofv3 kernel trace of the what-if step (7 waves per SIMD).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/whatif_prof" -o run --output-format csv -- python3 -u "$R/bench.py" --workload whatif --no-cpu-baseline --no-ucmp --steps 10 > "$R/gpurun_out/whatif_prof.log" 2>&1 || { tail -20 "$R/gpurun_out/whatif_prof.log"; exit 1; }
f=$(find "$R/gpurun_out/whatif_prof" -name "*kernel_stats.csv" | head -1); echo "$f"; head -12 "$f" | cut -c1-220
