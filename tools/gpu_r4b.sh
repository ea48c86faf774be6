#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4b
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_integration_docs.py tests/test_mcts_example.py tests/test_python_api.py tests/test_python_goldens.py -m gpu -v --timeout 200 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -1 "$OUT/pytest_new.log"
timeout -k 10 300 python -u tools/step_latency.py > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency.log"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));s=d['parity_sweep'];print({k:v['bit_exact'] if isinstance(v,dict) else v for k,v in s.items()})"
