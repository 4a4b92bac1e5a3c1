#!/bin/bash
# Host bulk-load timing (and optional gprof flat profile) of LinkState on a benchmark
# topology's encoded adj: values. CPU only.
#   TOPO=fabric PG=1 bash scripts/bulkload_prof.sh
set -eo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
TOPO="${TOPO:-fabric}"
OUT="${OUT:-/tmp/bulkload_$TOPO}"
mkdir -p "$OUT"
python3 - "$R" "$TOPO" "$OUT" <<'PY'
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from openr_amd import adjdb, topology
g = topology.fabric(5000) if sys.argv[2] == "fabric" else topology.grid_fast(100)
data, off = adjdb.AdjDbBatch.from_columns(adjdb.columns_for_graph(g)).encode_all()
np.asarray(data, dtype=np.uint8).tofile(sys.argv[3] + "/data.bin")
np.asarray(off, dtype=np.uint64).tofile(sys.argv[3] + "/off.bin")
PY
H="$R/openr_amd/csrc/host"
PGFLAG=""; [ -n "$PG" ] && PGFLAG="-pg"
g++ -O2 -g $PGFLAG -std=c++17 -I"$H" -I"$R/include" "$R/scripts/bulkload_bench.cpp" "$H/LinkState.cpp" \
  "$H/AdjDbCodec.cpp" -L"$R/openr_amd/lib" -lopenr_spf -Wl,-rpath,"$R/openr_amd/lib" -pthread -o "$OUT/bulkload"
cd "$OUT" && ./bulkload "$OUT" "${ITERS:-10}"
if [ -n "$PG" ]; then gprof -b -p bulkload gmon.out | head -20 | cut -c1-160; fi
