#!/bin/bash
# KSP2 fabric sample (512 sources x all destinations): step time, tracer counters, and a
# rocprofv3 kernel-trace summary of the same command.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
N=${KSP_SOURCES:-512}
timeout -k 10 300 python3 -u bench.py --workload ksp2 --ksp-sources $N --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ksp_s.log 2>&1 || { tail -5 gpurun_out/ksp_s.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ksp_s.log
if [ "${PROF:-0}" = 1 ]; then
  OPENR_SPF_PROF=1 timeout -k 10 300 python3 -u bench.py --workload ksp2 --ksp-sources $N --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/ksp_p.log 2>&1 || { tail -5 gpurun_out/ksp_p.log; exit 1; }
  grep -v '^{' gpurun_out/ksp_p.log | tail -30
  cd /tmp && export TMPDIR=/tmp
  rm -rf "$R/gpurun_out/ksp_prof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ksp_prof" -o run --output-format csv -- python3 -u "$R/bench.py" --workload ksp2 --ksp-sources $N --no-cpu-baseline --steps 3 --warmup 1 > "$R/gpurun_out/ksp_prof.log" 2>&1 || { tail -5 "$R/gpurun_out/ksp_prof.log"; exit 1; }
  f=$(find "$R/gpurun_out/ksp_prof" -name "*kernel_stats.csv" | head -1); cut -c1-60,200-330 "$f" | head -12
fi
