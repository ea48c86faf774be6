#!/bin/bash
# r06: pig parity on the numpy scalar role walk; pig step, cur vs the map-scan
# build (pignpscan).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "chance or pig or python_goldens or selfplay" > $O/pytest_pig.log 2>&1
rc=$?
tail -1 $O/pytest_pig.log
[ $rc -eq 0 ] || exit $rc
for v in cur pignpscan; do
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $v != cur ] && lib=$R/build_ab/lib_$v.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 7 --out $O/lat_$v > $O/lat_$v.log 2>&1 || { tail -5 $O/lat_$v.log; exit 1; }
  tail -n 1 $O/lat_$v/step_latency.md | sed "s/^/$v /"
done
