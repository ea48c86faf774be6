#!/bin/bash
# GPU-box session: parity tests, then one short bench line per BASELINE config.
# Each GPU step has its own time limit; steps are chained with && so the
# script stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cfg
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c2.json" 2> "$OUT/c2.err" &&
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" &&
timeout -k 10 600 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c4.json" 2> "$OUT/c4.err" &&
timeout -k 10 600 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err"
echo "exit=$?"
