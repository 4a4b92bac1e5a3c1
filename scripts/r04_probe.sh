#!/bin/bash
# Round-4 probe of the G100 level pass: occupancy sweep, per-phase cycles, SQ counters of
# the default full-batch kernel and of the 1 250-source shard kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 tests/cpp/build/linkstate_test gpu > gpurun_out/linkstate_test.log 2>&1; rc=$?; echo "linkstate_test rc=$rc"; grep -E "FAIL|failures|mismatch" gpurun_out/linkstate_test.log | tail -8
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py "tests/test_gpu_configs.py::test_config3_grid100_all_sources" > gpurun_out/new_tests.log 2>&1; rc=$?; echo "new tests rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/new_tests.log | tail -12
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python3 -u bench.py --workload decision --steps 10 --warmup 2 --decision-cases grid:100:sp,grid:10000:sp,fabric:5000:sp,grid:1024:ksp2 > gpurun_out/decision.log 2>&1; rc=$?; echo "decision rc=$rc"; tail -c 3000 gpurun_out/decision.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 240 python3 -u scripts/sweep.py --topology grid100 --rounds 6 \
  --variants "LWGS=10;LWGS=9;LWGS=8;LWGS=7;LWGS=6;LWGS=5" > gpurun_out/occ.log 2>&1 || { tail -20 gpurun_out/occ.log; exit 1; }
cat gpurun_out/occ.log
OPENR_SPF_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
grep bfs_ell gpurun_out/prof.log | tail -2
KFILTER=bfs_ell SQ_TAG=full BENCH_ARGS="--topology grid100" bash scripts/sq_counters.sh || exit 1
SQ_CMD="scripts/batch_latency.py --topology grid100 --sizes 1250 --reps 3" KFILTER=bfs_wave SQ_TAG=shard bash scripts/sq_counters.sh || exit 1
