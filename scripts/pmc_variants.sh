#!/bin/bash
# SQ counter pass per sweep variant (one rocprofv3 run each).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmcv_${PMC_TAG:-x}"
mkdir -p "$OUT"
CTRS="${PMC_CTRS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU}"
cd /tmp && export TMPDIR=/tmp
i=0
IFS=';' read -ra VARS <<< "${VARIANTS:-MS=0,G=2;LANES=8,G=1}"
for v in "${VARS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$OUT/v$i" -o run --output-format csv -- \
    python3 "$R/scripts/sweep.py" --topology ${TOPO:-grid100} --variants "$v" --rounds 1 > "$OUT/v$i.log" 2>&1
  rc=$?; echo "variant[$i] ($v) rc=$rc"; tail -1 "$OUT/v$i.log"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
