#!/bin/bash
# r05: full -m gpu suite + single-bot step latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_d.log" 2>&1 || { tail -30 "$OUT/pytest_d.log"; exit 1; }
tail -1 "$OUT/pytest_d.log"
timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out "$OUT/step_latency" \
  > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency/step_latency.md"
