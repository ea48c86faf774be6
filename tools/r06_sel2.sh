#!/bin/bash
# r06: lowest() and select96 with a branch-free word choice (in-tree,
# OS_SELECT96_FLAT=1) against a branch per word (build_ab/lib_sel0.so): g9 and C5, interleaved
# twice, then the go GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06/sel2
bash tools/r06_ab.sh sel2/g9 "--config g9" cur sel0 || exit 1
bash tools/r06_ab.sh sel2/c5 "--config c5" cur sel0 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "go" \
  > gpurun_out/r06/sel2/pytest_go.log 2>&1 || { tail -20 gpurun_out/r06/sel2/pytest_go.log; exit 1; }
tail -1 gpurun_out/r06/sel2/pytest_go.log
echo "r06_sel2 done"
