#!/bin/bash
# r06: go on the wave layout -- parity tests, 4096-root go9 search and the
# single go bot step, the parallel apply (cur) against the serial one (gopar0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/go
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "go or Go or selfplay or rollout" > $O/pytest_go.log 2>&1
rc=$?
tail -3 $O/pytest_go.log
[ $rc -eq 0 ] || exit $rc
bash tools/r06_ab.sh g9w "--config g9 --roots 4096 --layout wave --steps 3 --warmup 1 --parity-roots 8" cur gopar0 || exit 1
timeout -k 10 300 python -u tools/step_latency.py --games "go(board_size=9)" --reps 5 --out $O/lat_cur > $O/lat_cur.log 2>&1 || { tail -5 $O/lat_cur.log; exit 1; }
OS_AMD_LIB=$R/build_ab/lib_gopar0.so timeout -k 10 300 python -u tools/step_latency.py --games "go(board_size=9)" --reps 5 --out $O/lat_gopar0 > $O/lat_gopar0.log 2>&1 || { tail -5 $O/lat_gopar0.log; exit 1; }
cat $O/lat_cur/step_latency.md $O/lat_gopar0/step_latency.md
