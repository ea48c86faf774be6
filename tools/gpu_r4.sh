#!/bin/bash
# Round-4 GPU session: default bench (with the parity sweep), then the -m gpu
# suite + smoke.  Every GPU step has its own limit; stop at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4
mkdir -p "$OUT"
part=${1:-all}
if [ "$part" = all ] || [ "$part" = bench ]; then
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
  echo "bench done"; cut -c1-400 "$OUT/bench.json"
fi
if [ "$part" = all ] || [ "$part" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
  tail -1 "$OUT/smoke.log"
fi
