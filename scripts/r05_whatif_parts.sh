#!/bin/bash
# Round 5 experiment: what-if in parts (repair of part p+1 overlapping the re-solves of
# part p on a side stream). Parity on the whole workload, then the bench step per P.
# The OPENR_SPF_WHATIF_PARTS path and its test were removed after this measurement (slower).
set -o pipefail
O=gpurun_out/wparts; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "whatif_parts" -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for P in 1 2 3 4 1; do
  OPENR_SPF_WHATIF_PARTS=$P timeout -k 10 300 python -u bench.py --workload whatif --steps 20 --warmup 3 --no-cpu-baseline --no-ucmp > $O/bench_$P.log 2>&1 || { tail -10 $O/bench_$P.log; exit 1; }
  echo "P=$P $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_mean": [0-9.]*' $O/bench_$P.log | tr '\n' ' ')"
done
