#!/bin/bash
# r06: pig single step with two-player state arrays (pigmax2: timing A/B,
# exact for two players) against the product build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t9
mkdir -p $O
for v in cur pigmax2; do
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $v != cur ] && lib=$R/build_ab/lib_$v.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u tools/step_latency.py --games pig --reps 7 --out $O/lat_$v > $O/lat_$v.log 2>&1 || { tail -5 $O/lat_$v.log; exit 1; }
  tail -n 1 $O/lat_$v/step_latency.md | sed "s/^/$v /"
done
