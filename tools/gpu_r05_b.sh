#!/bin/bash
# r05: single-bot step latency (step and kernel in the same run) + az line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05
mkdir -p "$OUT"
timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out "$OUT/step_latency" \
  > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency/step_latency.md"
timeout -k 10 300 python -u bench.py --config az > "$OUT/az.json" 2> "$OUT/az.err" || { tail -20 "$OUT/az.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/az.json'));print('az', d['value'], d['ms_per_step'], d['parity'], d['az'])"
timeout -k 10 300 python -u bench.py --config az --az-overlap 0 > "$OUT/az_serial.json" 2> "$OUT/az_serial.err" || exit 1
python -c "import json;d=json.load(open('$OUT/az_serial.json'));print('az serial', d['value'], d['ms_per_step'])"
