#!/bin/bash
# r05: az tests and line after the replay change (Python only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/final
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_az.py tests/test_python_az.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > "$OUT/pytest_az.log" 2>&1 || { tail -20 "$OUT/pytest_az.log"; exit 1; }
tail -1 "$OUT/pytest_az.log"
timeout -k 10 600 python -u bench.py --config az > "$OUT/az.json" 2> "$OUT/az.err" || { tail -20 "$OUT/az.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/az.json'));print('az', d['value'], d['ms_per_step'], d['parity']['bit_exact'])"
