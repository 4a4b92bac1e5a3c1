# ELL-row locality probe: G100 all-sources kernel time under node renumberings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/perm_probe.py > gpurun_out/perm_probe.log 2>&1; rc=$?; grep order gpurun_out/perm_probe.log; exit $rc
