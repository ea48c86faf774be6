#!/bin/bash
# go wave-layout rollout (lane labels): go parity, new tests, step latency, g9 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4c
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -k "go or Go or selfplay or integration or mcts_example" -v --timeout 200 --timeout-method thread > "$OUT/pytest_go.log" 2>&1 || { tail -40 "$OUT/pytest_go.log"; exit 1; }
tail -1 "$OUT/pytest_go.log"
timeout -k 10 300 python -u tools/step_latency.py > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency.log"
for r in 4096 16384; do
  timeout -k 10 300 python -u bench.py --config g9 --roots $r --layout wave --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/g9_wave_$r.json" 2> "$OUT/g9_wave_$r.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/g9_wave_$r.json'));print('g9 wave $r', d['value'], d['ms_per_step'], d['parity'])"
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));s=d['parity_sweep'];print(d['value'], {k:v['bit_exact'] if isinstance(v,dict) else v for k,v in s.items()})"
