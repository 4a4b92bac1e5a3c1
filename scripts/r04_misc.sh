#!/bin/bash
# Round 4: resident set of the routes workload by stage; the config-1 line (G10 all-sources,
# GPU + faithful CPU at 1 and 16 threads).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/rss_probe.py > gpurun_out/rss.log 2>&1; rc=$?; echo "rss rc=$rc"; cat gpurun_out/rss.log | grep -v amdgpu.ids
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python3 -u bench.py --topology grid10 > gpurun_out/grid10.log 2>&1; rc=$?; echo "grid10 rc=$rc"; tail -c 2500 gpurun_out/grid10.log
exit $rc
