#!/bin/bash
# r06: k_lsearch<Go9>'s superko-log Bloom filter at 1024 bits per lane
# (in-tree, OS_LS_BLOOM1K=1) against 512 (build_ab/lib_bl0.so): g9 A/B
# interleaved twice, the go GPU tests, then every g9 root against the oracle.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/bloom
mkdir -p "$OUT"
bash tools/r06_ab.sh bloom/g9 "--config g9" cur bl0 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "go" \
  > "$OUT/pytest_go.log" 2>&1 || { tail -20 "$OUT/pytest_go.log"; exit 1; }
tail -1 "$OUT/pytest_go.log"
timeout -k 10 900 python -u tools/full_parity.py --out "$OUT/full_parity.json" --only g9 \
  > "$OUT/full_parity.txt" 2>&1 || { tail -5 "$OUT/full_parity.txt"; exit 1; }
tail -2 "$OUT/full_parity.txt"
echo "r06_bloom done"
