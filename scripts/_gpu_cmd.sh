set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ksp_probe_trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/ksp_probe.py > $GRAFT_REPO_ROOT/gpurun_out/ksp_probe_trace.log 2>&1; rc=$?
f=$(find $GRAFT_REPO_ROOT/gpurun_out/ksp_probe_trace -name "*kernel_stats.csv" | head -1); cut -c1-120 $f | head -8; exit $rc
