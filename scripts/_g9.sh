set -o pipefail
O=gpurun_out/r06/g9; mkdir -p $O
for pf in 0 1 0 1; do
OPENR_SPF_KSP_PREFETCH=$pf timeout -k 10 300 python3 -u bench.py --workload ksp2 --ksp-sources 1024 --steps 2 --warmup 1 --no-cpu-baseline > $O/k_$pf.log 2>&1 || { tail $O/k_$pf.log; exit 1; }
echo "prefetch=$pf $(grep -o '"ms_per_step": [0-9.]*' $O/k_$pf.log) $(grep -o '"ok": [a-z]*' $O/k_$pf.log)"
done
