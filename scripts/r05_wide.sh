#!/bin/bash
# Round 5: the wide pass for the fabric's degree-84 class. Parity of every sliced-class
# test (wide / sliced), then fabric all-sources launch times with the wide pass at 256 and
# 512 threads and with the sliced pass, interleaved in one process.
set -o pipefail
mkdir -p gpurun_out/wide
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fabric or sliced or source_classes or ring_overflow" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/wide/tests.txt 2>&1 || { tail -40 gpurun_out/wide/tests.txt; exit 1; }
tail -3 gpurun_out/wide/tests.txt
V="OPENR_SPF_WIDE=1;OPENR_SPF_WIDE=2;OPENR_SPF_WIDE=0"
timeout -k 10 300 python -u scripts/batch_latency.py --topology fabric --sizes 4992 --variants "$V" \
  > gpurun_out/wide/latency.jsonl 2>&1 || { tail -30 gpurun_out/wide/latency.jsonl; exit 1; }
cat gpurun_out/wide/latency.jsonl
