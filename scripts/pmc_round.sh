#!/bin/bash
# PMC HBM traffic of a round (FETCH_SIZE / WRITE_SIZE, one rocprofv3 run each, via
# scripts/pmc_traffic.sh): every engine kernel of a G100 / fabric all-sources step, of a
# KSP2 step on 64 fabric sources, and the what-if repair kernel. Each summary goes to
# gpurun_out/$ROUND/pmc_traffic_<name>.json and, on the box, to profiles/$ROUND/ so that
# bench lines run later in the same call cite it (bench.py PMC_ROUNDS). Commit the
# gpurun_out copies under profiles/$ROUND/. Arguments: names to run (default: all).
#   ROUND=r06 bash scripts/pmc_round.sh grid100 whatif
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
ROUND="${ROUND:-r06}"
stop() { case $1 in 0) ;; *) echo "step failed rc=$1; stopping"; exit $1;; esac; }
mkdir -p "$R/gpurun_out/$ROUND" "$R/profiles/$ROUND"
for spec in "grid100|PMC_AGG=1|--topology grid100|" "fabric|PMC_AGG=1|--topology fabric|" \
            "ksp2|PMC_AGG=1|--workload ksp2 --ksp-sources 64|" \
            "whatif|PMC_KERNEL=whatif_group|--workload whatif --no-ucmp --no-delta|"; do
  name=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; rest=${rest#*|}; args=${rest%%|*}
  [ $# -gt 0 ] && ! [[ " $* " == *" $name "* ]] && continue
  env $envs PMC_TAG="$ROUND/pmc/$name" BENCH_ARGS="$args" bash "$R/scripts/pmc_traffic.sh" > "$R/gpurun_out/$ROUND/pmc_$name.log" 2>&1; stop $?
  cp "$R/gpurun_out/pmc_$ROUND/pmc/$name/pmc_traffic.json" "$R/gpurun_out/$ROUND/pmc_traffic_$name.json"
  cp "$R/gpurun_out/$ROUND/pmc_traffic_$name.json" "$R/profiles/$ROUND/pmc_traffic_$name.json"
  echo "$name: $(grep -o '"hbm_bytes_per_[a-z]*": [0-9.e+]*' "$R/gpurun_out/$ROUND/pmc_traffic_$name.json")"
done
