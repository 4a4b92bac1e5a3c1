#!/bin/bash
# Round 5 experiment: the code family's lean edge loop with 8 edges per lane (k8), the next
# step's edge loads issued before this step's LDS work (pf4), and both (pf8), against the
# default (4 edges, no prefetch). Fabric all-sources launch time + fabric parity per variant.
# The variant libraries (_variants/<name>/, untracked) were compile-time builds of
# spf_bfs.hip whose experiment macros were removed after this measurement.
set -o pipefail
O=gpurun_out/lean_var; mkdir -p $O
cp openr_amd/lib/libopenr_spf.so $O/default.so
for v in default k8 pf4 pf8; do
  if [ $v = default ]; then cp $O/default.so openr_amd/lib/libopenr_spf.so; else cp _variants/$v/libopenr_spf.so openr_amd/lib/libopenr_spf.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "fabric_small or fabric_5000 or source_classes" -x -q --timeout 120 --timeout-method thread > $O/tests_$v.txt 2>&1 || { echo "$v tests failed"; tail -5 $O/tests_$v.txt; exit 1; }
  timeout -k 10 200 python -u scripts/batch_latency.py --topology fabric --sizes 4992 --reps 30 > $O/lat_$v.jsonl 2>&1 || { tail -5 $O/lat_$v.jsonl; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.txt) $(grep -o '"median_ms": [0-9.]*' $O/lat_$v.jsonl)"
done
cp $O/default.so openr_amd/lib/libopenr_spf.so
