#!/bin/bash
# Round 5: route-DB node recycling. The C++ decision suite on the GPU engine, then the
# all-node route build with the default allocator settings and without heap trimming.
set -o pipefail
mkdir -p gpurun_out/routes
timeout -k 10 300 tests/cpp/build/decision_test gpu > gpurun_out/routes/decision_test.log 2>&1 || { grep FAIL gpurun_out/routes/decision_test.log | head; tail -3 gpurun_out/routes/decision_test.log; exit 1; }
tail -1 gpurun_out/routes/decision_test.log
i=0
for T in "" "glibc.malloc.trim_threshold=4294967296:glibc.malloc.mmap_threshold=33554432:glibc.malloc.top_pad=67108864"; do
  i=$((i+1))
  GLIBC_TUNABLES=$T timeout -k 10 300 python3 -u bench.py --workload routes --steps 3 --warmup 1 > gpurun_out/routes/recycle_$i.log 2>&1 || { tail -20 gpurun_out/routes/recycle_$i.log; exit 1; }
  echo "variant $i [$T]: $(grep -o '"ms_per_step": [0-9.]*\|"checksum": "[0-9a-f]*"\|"peak_rss_mb": [0-9.]*' gpurun_out/routes/recycle_$i.log | tr '\n' ' ')"
done
