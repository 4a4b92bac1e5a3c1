# KSP2 chunk size A/B (pairs per chunk: the k=2 trace reads its chunk's second-SPF rows;
# a chunk whose rows fit the Infinity Cache keeps those reads off HBM).
set -o pipefail
mkdir -p gpurun_out
for c in 0 65536 32768 16384 8192 0; do
  if [ $c = 0 ]; then unset OPENR_SPF_KSP_CHUNK; else export OPENR_SPF_KSP_CHUNK=$c; fi
  timeout -k 10 200 python -u bench.py --workload ksp2 --topology fabric --ksp-sources 512 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_kspc_$c.log 2>&1 || { tail -20 gpurun_out/b_kspc_$c.log; exit 1; }
  grep '^{' gpurun_out/b_kspc_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ksp chunk $c', round(d['ms_per_step'],2))"
done
