#!/bin/bash
# r05: full -m gpu suite, then the driver's default bench command, timed.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
t0=$(date +%s)
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/default_bench.json" 2> "$OUT/default_bench.err" || { tail -20 "$OUT/default_bench.err"; exit 1; }
t1=$(date +%s)
echo "default bench wall $((t1-t0)) s"
python - "$OUT/default_bench.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print('c2', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['parity_sweep']['all_bit_exact'], d['parity_sweep']['seconds'])
c=d['configs']
for k,v in c.items():
  if isinstance(v,dict):
    print(k, v.get('value'), v.get('ms_per_step'), (v.get('roofline') or {}).get('frac'), v.get('parity'), v.get('seconds_total'), v.get('error'))
print('all', c['all_bit_exact'], c['seconds'])
PY
