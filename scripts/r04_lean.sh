#!/bin/bash
# Round-4 lean pass iteration: parity (configs, lean overflow paths, level rows), then the
# G100 full batch and shard timings.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py \
  tests/test_gpu_rccl.py "tests/test_gpu_parity.py::test_lean_pass_depth_overflow" \
  "tests/test_gpu_parity.py::test_lean_pass_half_overflow" "tests/test_gpu_parity.py::test_ring_overflow_rerun_list" \
  > gpurun_out/lean_tests.log 2>&1; rc=$?
echo "lean tests rc=$rc"; grep -E "FAIL|Error|error|passed|failed" gpurun_out/lean_tests.log | tail -12
case $rc in 0) ;; *) tail -40 gpurun_out/lean_tests.log; exit $rc;; esac
OPENR_SPF_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gather > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
grep bfs_ell gpurun_out/prof.log | tail -1
timeout -k 10 240 python3 -u scripts/sweep.py --topology grid100 --rounds 6 \
  --variants "LWGS=0;LWGS=8;LWGS=7" > gpurun_out/occ.log 2>&1 || { tail -20 gpurun_out/occ.log; exit 1; }
cat gpurun_out/occ.log
timeout -k 10 200 python3 -u scripts/batch_latency.py --topology grid100 --sizes 1250,2500,5000,10000 --reps 5 > gpurun_out/lat.log 2>&1 || { tail -20 gpurun_out/lat.log; exit 1; }
tail -4 gpurun_out/lat.log
