#!/bin/bash
# A/B of k_az_step's searches per wave (bench.py --config az --block B).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/ab_az
mkdir -p "$OUT"
for b in ${*:-64 16 8}; do
  timeout -k 10 300 python -u bench.py --config az --steps 3 --warmup 1 --no-cpu-baseline \
    --block "$b" > "$OUT/az_b$b.json" 2> "$OUT/az_b$b.err" || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/az_b$b.json')); print('block $b', d['value'], d['ms_per_step'], d['az']['k_az_step_ms_total'], d['parity'])"
done
