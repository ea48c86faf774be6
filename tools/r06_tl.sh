#!/bin/bash
# r06: go's lane apply with the points of two or more empty neighbours found
# for the whole board first (os_games.h OS_GO_TWO_LIB), so most opponent
# neighbours and new stones skip their floods, against every flood from its
# seed (build_ab/lib_tl0.so): the -m gpu suite, g9 / C5 / C5 per-rank A/B,
# then every g9 root and C5 playout against the oracle.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/tl
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/r06_ab.sh tl/g9 "--config g9" cur tl0 || exit 1
bash tools/r06_ab.sh tl/c5 "--config c5" cur tl0 || exit 1
bash tools/r06_ab.sh tl/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur tl0 || exit 1
timeout -k 10 900 python -u tools/full_parity.py --out "$OUT/full_parity.json" --only g9,c5 \
  > "$OUT/full_parity.txt" 2>&1 || { tail -5 "$OUT/full_parity.txt"; exit 1; }
tail -2 "$OUT/full_parity.txt"
echo "r06_tl done"
