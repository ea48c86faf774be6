#!/bin/bash
# r06: two filter bits per position of the root's history in front of its
# scan (os_games.h OS_GO_BASE_FILT2) against one (build_ab/lib_bf1.so): the
# -m gpu suite, g9 / C5 / C5 per-rank A/B, then every g9 root and C5 playout
# against the oracle.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/bf
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/r06_ab.sh bf/g9 "--config g9" cur bf1 || exit 1
bash tools/r06_ab.sh bf/c5 "--config c5" cur bf1 || exit 1
bash tools/r06_ab.sh bf/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur bf1 || exit 1
timeout -k 10 900 python -u tools/full_parity.py --out "$OUT/full_parity.json" --only g9,c5 \
  > "$OUT/full_parity.txt" 2>&1 || { tail -5 "$OUT/full_parity.txt"; exit 1; }
tail -2 "$OUT/full_parity.txt"
echo "r06_bf done"
