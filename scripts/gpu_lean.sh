set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sweep.py --topology grid100 --variants "XS=0;XS=1" --rounds 8 > gpurun_out/xs_sweep.log 2>&1; rc=$?; grep -E "variant|Error|error" gpurun_out/xs_sweep.log | cut -c1-120; exit $rc
