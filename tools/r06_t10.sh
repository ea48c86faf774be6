#!/bin/bash
# r06: full -m gpu suite with two-player pig on Pig2, then pig's step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 7 --out $O/lat_pig > $O/lat_pig.log 2>&1 || { tail -5 $O/lat_pig.log; exit 1; }
tail -n 1 $O/lat_pig/step_latency.md
