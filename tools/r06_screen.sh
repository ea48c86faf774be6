#!/bin/bash
# r06: lane-layout UCT selection screened in f32 (mcts_search, OS_LANE_SCREEN),
# k_rollouts' size-selected LDS Zobrist table and go's one-pass expansion list
# (Legal::fill).  The -m gpu suite, g9 A/B against build_ab/lib_scr0.so
# (-DOS_LANE_SCREEN=0) and build_ab/lib_fill0.so (-DOS_LEGAL_FILL=0), C5 at
# both sizes, then every g9 and C5 root / playout against the oracle
# (tools/full_parity.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/screen
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/r06_ab.sh screen/g9 "--config g9" cur scr0 fill0 || exit 1
bash tools/r06_ab.sh screen/c5 "--config c5" cur || exit 1
bash tools/r06_ab.sh screen/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur || exit 1
timeout -k 10 900 python -u tools/full_parity.py --out "$OUT/full_parity.json" --only g9,c5 \
  > "$OUT/full_parity.txt" 2>&1 || { tail -5 "$OUT/full_parity.txt"; exit 1; }
tail -3 "$OUT/full_parity.txt"
echo "r06_screen done"
