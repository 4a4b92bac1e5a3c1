#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over one sweep variant.
#   PMC_TAG=r01 SWEEP_ARGS='--topology grid100 --variants G=2 --rounds 1' bash scripts/pmc.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_${PMC_TAG:-x}"
mkdir -p "$OUT"
SARGS="${SWEEP_ARGS:---topology grid100 --variants G=2 --rounds 1}"
cd /tmp && export TMPDIR=/tmp
i=0
IFS='|' read -ra PMCGRP <<< "${PMC_LIST:-FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU|SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT}"
for grp in "${PMCGRP[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- \
    python3 "$R/scripts/sweep.py" $SARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pmc[$i] ($grp) rc=$rc"
  case $rc in 0) ;; *) tail -5 "$OUT/p$i.log"; exit $rc;; esac
done
exit 0
