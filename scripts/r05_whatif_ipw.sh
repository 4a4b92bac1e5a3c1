#!/bin/bash
# Round 5 experiment: what-if work items per resident workgroup (the OPENR_SPF_WHATIF_IPW
# knob existed only for this sweep; 8 stays the code's value).
set -o pipefail
O=gpurun_out/ipw; mkdir -p $O
for I in 8 2 3 4 6 12 8; do
  OPENR_SPF_WHATIF_IPW=$I timeout -k 10 300 python -u bench.py --workload whatif --steps 20 --warmup 3 --no-cpu-baseline --no-ucmp > $O/bench_$I.log 2>&1 || { tail -10 $O/bench_$I.log; exit 1; }
  echo "IPW=$I $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_mean": [0-9.]*' $O/bench_$I.log | tr '\n' ' ')"
done
