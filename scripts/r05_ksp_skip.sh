#!/bin/bash
# KSP2 pairs with an empty k = 2 answer by construction (ksp_select_pairs): parity tests,
# then the all-pairs fabric bench with the skip on and off. Output: gpurun_out/r05/kspskip/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r05/kspskip"; mkdir -p "$OUT"
stop() { case $1 in 0) ;; *) echo "step failed rc=$1; stopping"; exit $1;; esac; }
export TMPDIR=/tmp
cd "$R" && timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "ksp2" tests/test_gpu_configs.py::test_config5_fabric_ksp2_all_destinations \
  tests/test_gpu_configs.py::test_config5_fabric_ksp2_more_sources > "$OUT/tests.txt" 2>&1; stop $?
tail -2 "$OUT/tests.txt"
for S in ${SKIPS:-1 0}; do
  OPENR_SPF_KSP_SKIP=$S OPENR_SPF_KSP_RESUME=${RESUME:-1} OPENR_SPF_KSP_PULL=${PULL:-1} OPENR_SPF_KSP_PACK=${PACK:-1} timeout -k 10 300 python3 -u bench.py --workload ksp2 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_skip${S}_resume${RESUME:-1}_pull${PULL:-1}_pack${PACK:-1}.log" 2>&1; stop $?
  echo "skip=$S $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_skip${S}_resume${RESUME:-1}_pull${PULL:-1}_pack${PACK:-1}.log")"
done
