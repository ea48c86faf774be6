#!/bin/bash
# r05 A/B: hex fill four moves per step (in-tree, OS_HEX_TAKE4=1) against one
# (build_ab/lib_take1.so).  GPU tests of hex first, full-size C4 parity, then
# C4 timings interleaved and single-bot hex latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_take4
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "hex or python or parity" > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python -u tools/full_parity.py --only c4 --out "$OUT/full_parity_c4.json" 2>&1 | tee "$OUT/full_parity.log" | grep -v "checked" || exit 1
bash tools/gpu_ab_cfg.sh c4 3 take1 cur || exit 1
timeout -k 10 300 python -u tools/step_latency.py --reps 7 --games hex --out "$OUT/lat_cur" > "$OUT/lat_cur.log" 2>&1 || exit 1
OS_AMD_LIB=$R/build_ab/lib_take1.so timeout -k 10 300 python -u tools/step_latency.py --reps 7 --games hex --out "$OUT/lat_take1" > "$OUT/lat_take1.log" 2>&1 || exit 1
grep "^| hex" "$OUT"/lat_*/step_latency.md
