#!/bin/bash
# r06: chance-node parity (pig) on the LDS LUT build, pig's single-bot step,
# then the default bench line as the driver runs it (C2 + configs).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chance or pig or python_goldens or selfplay" > $O/pytest_pig.log 2>&1
rc=$?
tail -1 $O/pytest_pig.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 5 --out $O/lat_pig > $O/lat_pig.log 2>&1 || { tail -5 $O/lat_pig.log; exit 1; }
tail -n 1 $O/lat_pig/step_latency.md
timeout -k 10 600 python -u bench.py > $O/default_bench.json 2> $O/default_bench.err || { tail -5 $O/default_bench.err; exit 1; }
python - "$O/default_bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print('C2', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['parity_sweep']['all_bit_exact'])
for k, v in d.get('configs', {}).items():
  if isinstance(v, dict):
    print(k, v.get('value'), v.get('ms_per_step'), v.get('parity', {}).get('bit_exact'))
PY
