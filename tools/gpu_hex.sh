#!/bin/bash
# GPU-box iteration on the hex wave kernel: hex parity tests, the layout
# probe, and the C4 bench line in the wave layout.  Each GPU step has its own
# time limit; the first failure ends the session.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/hx
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k hex --timeout 200 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/rollout_probe.py ${PROBE_ARGS:-65536 4096 256} > "$OUT/probe.txt" 2>&1 || { tail "$OUT/probe.txt"; exit 1; }
grep -i hex "$OUT/probe.txt"
timeout -k 10 300 python bench.py --config c4 --layout ${C4_LAYOUT:-wave} --steps 2 --warmup 1 \
  --no-cpu-baseline > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail "$OUT/c4.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/c4.json'));print('c4', '%.4g'%d['value'], '%.1f ms'%d['ms_per_step'], d['parity'])"
