#!/bin/bash
# r05 A/B: k_lsearch's MT streams stored 16 words at a time (wc1, in-tree)
# against word by word (wc0).  GPU tests of the lane kernels on the in-tree
# build first, then the g9 line and FETCH / WRITE passes per build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_wc
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "go or big or lane or stateful or python or az" > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/g9_ab.sh ${AB_TAGS:-wc0 wc1} || exit 1
