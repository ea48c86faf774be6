#!/bin/bash
# Bloom-fronted superko bucket log (OS_GO_LOG_BLOOM): go parity on the GPU, C5 / g9 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/bloomlog
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_big_boards.py tests/test_selfplay.py tests/test_full_configs.py -k "go or Go or c5 or C5" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for c in c5 g9; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep > "$OUT/$c.json" 2> "$OUT/$c.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['value'], d['ms_per_step'], d['parity'])"
done
timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sweep > "$OUT/g9w.json" 2> "$OUT/g9w.err" || exit 1
python -c "import json;d=json.load(open('$OUT/g9w.json'));print('g9w', d['value'], d['ms_per_step'], d['parity']['bit_exact'])"
