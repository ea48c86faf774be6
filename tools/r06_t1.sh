#!/bin/bash
# r06: full -m gpu suite, the AlphaZero bot latency rows, and pig's single-bot
# step on the turn-walk playout (cur) against the node-by-node one (pig0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_latency.py --az --reps 5 --out $O/az > $O/az.log 2>&1 || { tail -5 $O/az.log; exit 1; }
cut -c1-300 $O/az.log
timeout -k 10 300 python -u tools/step_latency.py --games pig,tic_tac_toe,connect_four --reps 7 --out $O/lat_cur > $O/lat_cur.log 2>&1 || { tail -5 $O/lat_cur.log; exit 1; }
OS_AMD_LIB=$R/build_ab/lib_pig0.so timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 7 --out $O/lat_pig0 > $O/lat_pig0.log 2>&1 || { tail -5 $O/lat_pig0.log; exit 1; }
cat $O/lat_cur/step_latency.md $O/lat_pig0/step_latency.md
