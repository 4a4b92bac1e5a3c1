#!/bin/bash
# Round 5: all-node route build (bench.py --workload routes) under glibc malloc tunables:
# default, no trimming / no mmap for large blocks, and a larger per-thread cache.
set -o pipefail
mkdir -p gpurun_out/routes
i=0
for T in "" "glibc.malloc.trim_threshold=4294967296:glibc.malloc.mmap_threshold=33554432:glibc.malloc.top_pad=67108864" \
         "glibc.malloc.trim_threshold=4294967296:glibc.malloc.mmap_threshold=33554432:glibc.malloc.top_pad=67108864:glibc.malloc.tcache_count=2048"; do
  i=$((i+1))
  GLIBC_TUNABLES=$T timeout -k 10 300 python3 -u bench.py --workload routes --steps 3 --warmup 1 > gpurun_out/routes/malloc_$i.log 2>&1 || { tail -20 gpurun_out/routes/malloc_$i.log; exit 1; }
  echo "variant $i [$T]: $(grep -o '"ms_per_step": [0-9.]*\|"checksum": "[0-9a-f]*"\|"peak_rss_mb": [0-9.]*' gpurun_out/routes/malloc_$i.log | tr '\n' ' ')"
done
