#!/bin/bash
# Iteration session on the GPU box: parity tests, then short bench lines for
# the configs named on the command line (default: c2).  Each GPU step has its
# own time limit; steps are chained so the first failure ends the session.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/iter
mkdir -p "$OUT"
cd "$R"
CFGS=${*:-c2}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
for c in $CFGS; do
  timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline \
    > "$OUT/$c.json" 2> "$OUT/$c.err" || { echo "bench $c failed"; tail -20 "$OUT/$c.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', '%.4g'%d['value'], d['unit'], '%.2f ms'%d['ms_per_step'], d.get('parity'))"
done
