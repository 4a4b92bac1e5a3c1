set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/sweep.py --topology fabric --variants "G=1;G=2;G=4;G=8;G=16" --rounds 5 > gpurun_out/g_sweep.log 2>&1 || { tail -20 gpurun_out/g_sweep.log; exit 1; }
grep -E "variant" gpurun_out/g_sweep.log | cut -c1-110 | tail -6
