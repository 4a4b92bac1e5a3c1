#!/bin/bash
# Round 5: 512-thread workgroups for the code family's high-degree classes. Parity of the
# fabric / KSP2 / class tests, then fabric all-sources and fabric KSP2 with the 512- and
# 256-thread shapes.
set -o pipefail
mkdir -p gpurun_out/block
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "fabric or sliced or source_classes or ksp or distance_only or config2 or config5" -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/block/tests.txt 2>&1 || { tail -40 gpurun_out/block/tests.txt; exit 1; }
tail -3 gpurun_out/block/tests.txt
timeout -k 10 300 python -u scripts/batch_latency.py --topology fabric --sizes 4992 --variants "OPENR_SPF_BFS_BLOCK=512;OPENR_SPF_BFS_BLOCK=256" \
  > gpurun_out/block/latency.jsonl 2>&1 || { tail -30 gpurun_out/block/latency.jsonl; exit 1; }
cat gpurun_out/block/latency.jsonl
for b in 512 256; do
  OPENR_SPF_BFS_BLOCK=$b timeout -k 10 300 python -u bench.py --workload ksp2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/block/ksp2_$b.log 2>&1 || { tail -30 gpurun_out/block/ksp2_$b.log; exit 1; }
  echo "ksp2 block $b: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/block/ksp2_$b.log)"
done
