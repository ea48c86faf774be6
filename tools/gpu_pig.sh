#!/bin/bash
# chance-node kernels without scratch: chance parity tests, pig step latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/pig
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_chance.py tests/test_selfplay.py -k "pig or chance" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/step_latency.py --reps 5 --games pig,connect_four --out "$OUT/step_latency" > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency/step_latency.md"
