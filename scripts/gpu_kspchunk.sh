# KSP2 chunk budget A/B (MiB of second-SPF rows + ignore slots per chunk; default 2048).
set -o pipefail
mkdir -p gpurun_out
for c in 2048 4096 8192 16384 2048; do
  OPENR_SPF_KSP_CHUNK_MB=$c timeout -k 10 200 python -u bench.py --workload ksp2 --topology fabric --ksp-sources 512 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_kspm_$c.log 2>&1 || { tail -20 gpurun_out/b_kspm_$c.log; exit 1; }
  grep '^{' gpurun_out/b_kspm_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ksp chunk MB $c', round(d['ms_per_step'],2))"
done
