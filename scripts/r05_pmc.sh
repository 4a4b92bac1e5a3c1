#!/bin/bash
# Round 5 PMC traffic passes (FETCH_SIZE / WRITE_SIZE, one rocprofv3 run each): every engine
# kernel of a G100 / fabric all-sources step and of a KSP2 step on 64 fabric sources. Copy
# gpurun_out/r05/pmc/<name>/pmc_traffic.json to profiles/r05/pmc_traffic_<name>.json before
# recording bench lines (they cite only tracked evidence). Arguments: the names to run
# (default: all).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
stop() { case $1 in 0) ;; *) echo "step failed rc=$1; stopping"; exit $1;; esac; }
for spec in "grid100|PMC_AGG=1|--topology grid100" "fabric|PMC_AGG=1|--topology fabric" \
            "ksp2|PMC_AGG=1|--workload ksp2 --ksp-sources 64"; do
  name=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; args=${rest#*|}
  [ $# -gt 0 ] && ! [[ " $* " == *" $name "* ]] && continue  # names given: only those
  env $envs PMC_TAG="r05/pmc/$name" BENCH_ARGS="$args" bash "$R/scripts/pmc_traffic.sh" > "$R/gpurun_out/pmc_$name.log" 2>&1; stop $?
  mkdir -p "$R/gpurun_out/r05/pmc/$name" && cp "$R/gpurun_out/pmc_r05/pmc/$name/pmc_traffic.json" "$R/gpurun_out/r05/pmc/$name/pmc_traffic.json"
  echo "$name: $(grep -o '"hbm_bytes_per_[a-z]*": [0-9.e+]*' "$R/gpurun_out/r05/pmc/$name/pmc_traffic.json")"
done
