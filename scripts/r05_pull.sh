#!/bin/bash
# Round 5: direction-optimising (pull) levels in the code family. Parity first (pull
# variants, fabric / sliced / source-class tests), then fabric all-sources launch times
# with pull off / on, interleaved in one process.
set -o pipefail
mkdir -p gpurun_out/pull
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "pull or fabric or sliced or source_classes or ring_overflow or distance_only" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/pull/tests.txt 2>&1 || { tail -40 gpurun_out/pull/tests.txt; exit 1; }
tail -3 gpurun_out/pull/tests.txt
V="OPENR_SPF_PULL=8;OPENR_SPF_PULL=0;OPENR_SPF_PULL=2;OPENR_SPF_PULL=1024;OPENR_SPF_PULL=8,OPENR_SPF_WIDE=0"
timeout -k 10 300 python -u scripts/batch_latency.py --topology fabric --sizes 4992 --variants "$V" \
  > gpurun_out/pull/latency.jsonl 2>&1 || { tail -30 gpurun_out/pull/latency.jsonl; exit 1; }
cat gpurun_out/pull/latency.jsonl
