#!/bin/bash
# go wave rollout + wave az kernel: parity first, then measurements.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4d
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu --deselect tests/test_mcts_example.py::test_verbose_report_matches_oracle_tree -k "go or Go or selfplay or integration or mcts_example or az or chance or pig" -v --timeout 200 --timeout-method thread > "$OUT/pytest_sel.log" 2>&1 || { grep -E "FAILED|Error|error" "$OUT/pytest_sel.log" | head -30; tail -5 "$OUT/pytest_sel.log"; exit 1; }
tail -1 "$OUT/pytest_sel.log"
timeout -k 10 300 python -u tools/step_latency.py > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency.log"
for r in 4096 16384; do
  timeout -k 10 300 python -u bench.py --config g9 --roots $r --layout wave --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/g9_wave_$r.json" 2> "$OUT/g9_wave_$r.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/g9_wave_$r.json'));print('g9 wave $r', d['value'], d['ms_per_step'], d['parity'])"
done
timeout -k 10 300 python -u bench.py --config az --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/az.json" 2> "$OUT/az.err" || exit 1
python -c "import json;d=json.load(open('$OUT/az.json'));print('az', d['value'], d['ms_per_step'], d['az'], d['parity'])"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));s=d['parity_sweep'];print(d['value'], {k:v['bit_exact'] if isinstance(v,dict) else v for k,v in s.items()})"
