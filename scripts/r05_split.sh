#!/bin/bash
# Round-5 shard experiment: wave-pass parity for the split variants, then
# the shard-size kernel times of the three variants interleaved. The split variants were
# removed after this measurement: run it on commit 919d97c.
set -o pipefail
mkdir -p gpurun_out/split
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wave_pass" -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/split/tests.txt 2>&1 || { tail -30 gpurun_out/split/tests.txt; exit 1; }
tail -3 gpurun_out/split/tests.txt
V="OPENR_SPF_BFS_WAVE=1,OPENR_SPF_BFS_WAVE_SPLIT=0;OPENR_SPF_BFS_WAVE=1,OPENR_SPF_BFS_WAVE_SPLIT=1;OPENR_SPF_BFS_WAVE=1,OPENR_SPF_BFS_WAVE_SPLIT=2"
timeout -k 10 300 python -u scripts/batch_latency.py --topology grid100 --sizes 625,1250,2500,3334 --variants "$V" \
  > gpurun_out/split/latency.jsonl 2>&1 || { tail -30 gpurun_out/split/latency.jsonl; exit 1; }
cat gpurun_out/split/latency.jsonl
