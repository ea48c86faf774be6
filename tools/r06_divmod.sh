#!/bin/bash
# r06: the shuffle's pair split (x / b1, x % b1) by an f32 reciprocal and one
# correction (os_rng.h small_divmod) against the compiler's integer division
# (build_ab/lib_dm0.so, -DOS_SHUFFLE_DIVMOD=0): the -m gpu suite, g9 A/B,
# then every g9 root against the oracle.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/divmod
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/r06_ab.sh divmod/g9 "--config g9" cur dm0 || exit 1
timeout -k 10 900 python -u tools/full_parity.py --out "$OUT/full_parity.json" --only g9 \
  > "$OUT/full_parity.txt" 2>&1 || { tail -5 "$OUT/full_parity.txt"; exit 1; }
tail -2 "$OUT/full_parity.txt"
echo "r06_divmod done"
