set -o pipefail
O=gpurun_out/r06/g8; mkdir -p $O
OPENR_SPF_PROF=1 timeout -k 10 300 python3 -u bench.py --workload ksp2 --ksp-sources 512 --steps 1 --warmup 0 --no-cpu-baseline > $O/kspstats.log 2>&1 || { tail $O/kspstats.log; exit 1; }
grep -E "ksp_stats|ms_per_step" $O/kspstats.log | cut -c1-400
