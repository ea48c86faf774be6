#!/bin/bash
# r06: chance-node parity (pig) on the node-lane C++ playout, pig's
# single-bot step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chance or pig or python_goldens or selfplay" > $O/pytest_pig.log 2>&1
rc=$?
tail -1 $O/pytest_pig.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 7 --out $O/lat_pig > $O/lat_pig.log 2>&1 || { tail -5 $O/lat_pig.log; exit 1; }
tail -n 1 $O/lat_pig/step_latency.md
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-configs --no-parity-sweep > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['ms_per_step'], d['value'], d['parity']['bit_exact'])"
