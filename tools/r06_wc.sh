#!/bin/bash
# r06: k_lsearch's write-combined streams, timed: the MT19937 words
# (OS_LS_WC=0: word by word, build_ab/lib_lsw0.so) and the superko log
# (OS_LS_LOGWC=0: entry by entry, build_ab/lib_lsl0.so) against the in-tree
# library (both combined), g9 interleaved twice.  A flush is a branch that
# one lane of a 32-lane wave takes on most moves.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06/wc
bash tools/r06_ab.sh wc/g9 "--config g9" cur lsw0 lsl0 || exit 1
echo "r06_wc done"
