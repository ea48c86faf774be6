#!/bin/bash
# r06: k_rollouts' 1024-bit superko-log Bloom filter for batches of at most
# 131072 playouts (in-tree, OS_ROLL_BLOOM1K=1) against 512 bits
# (build_ab/lib_rb0.so): the C5 per-rank share and C5 A/B, interleaved twice;
# then rocprof, PMC and the default bench on these sources (call F).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06/rbloom
bash tools/r06_ab.sh rbloom/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur rb0 || exit 1
bash tools/r06_ab.sh rbloom/c5 "--config c5" cur rb0 || exit 1
rm -f build_ab/lib_rb0.so
bash tools/r06_callF.sh
