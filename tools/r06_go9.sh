#!/bin/bash
# r06: go up to 9 x 9 on three-word bitboards (Go9).  The -m gpu suite on the
# new library, then g9 and C5 A/B against an OS_GO9=0 build (build_ab/
# lib_go9off.so), interleaved twice.  Results under gpurun_out/r06/go9/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/go9
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/r06_ab.sh go9/g9 "--config g9" cur go9off || exit 1
bash tools/r06_ab.sh go9/c5 "--config c5" cur go9off || exit 1
bash tools/r06_ab.sh go9/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur go9off || exit 1
echo "r06_go9 done"
