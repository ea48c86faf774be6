#!/bin/bash
# r06: pig parity with the f32 UCT screen in the chance search, pig step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chance or pig or python_goldens or selfplay" > $O/pytest_pig.log 2>&1
rc=$?
tail -1 $O/pytest_pig.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 7 --out $O/lat_pig > $O/lat_pig.log 2>&1 || { tail -5 $O/lat_pig.log; exit 1; }
tail -n 1 $O/lat_pig/step_latency.md
