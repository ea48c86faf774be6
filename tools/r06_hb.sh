#!/bin/bash
# r06: the captured stones' Zobrist terms by for_each_bit (in-tree,
# OS_GO_HASH_BITS=1) against lowest / clear per stone (build_ab/lib_hb0.so):
# g9 and C5, interleaved twice, then the go GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06/hb
bash tools/r06_ab.sh hb/g9 "--config g9" cur hb0 || exit 1
bash tools/r06_ab.sh hb/c5 "--config c5" cur hb0 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "go" \
  > gpurun_out/r06/hb/pytest_go.log 2>&1 || { tail -20 gpurun_out/r06/hb/pytest_go.log; exit 1; }
tail -1 gpurun_out/r06/hb/pytest_go.log
echo "r06_hb done"
