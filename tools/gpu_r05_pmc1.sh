#!/bin/bash
# r05: instruction-cache and issue counters of single-root searches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/pmc1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SPECS="tic_tac_toe connect_four hex hex:numpy pig"
i=0
for C in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 "$R/tools/single_search.py" 1000 $SPECS > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
done
find "$OUT" -name "*counter_collection.csv" | head
