#!/bin/bash
# r06: go wave apply variants (cur: lane Zobrist + one-copy neighbour loop;
# gozl0: the same with zob[] loads; gopar0: the serial apply) on 4096-root
# go9 and the single go bot; pig with / without playouts (pignoroll: timing
# only, NOT the reference's results) for attribution.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "go or Go or selfplay" > $O/pytest_go.log 2>&1
rc=$?
tail -1 $O/pytest_go.log
[ $rc -eq 0 ] || exit $rc
lat() {  # tag lib games
  OS_AMD_LIB=$2 timeout -k 10 300 python -u tools/step_latency.py --games "$3" --reps 5 --out $O/lat_$1 > $O/lat_$1.log 2>&1 || { tail -5 $O/lat_$1.log; exit 1; }
  tail -n +3 $O/lat_$1/step_latency.md | sed "s/^/$1 /"
}
CUR=$R/open_spiel-1_amd/os_amd/libos_mcts.so
bash tools/r06_ab.sh g9w3 "--config g9 --roots 4096 --layout wave --steps 3 --warmup 1 --parity-roots 8" cur gozl0 gopar0 || exit 1
lat go_cur $CUR "go(board_size=9)"
lat go_zl0 $R/build_ab/lib_gozl0.so "go(board_size=9)"
lat pig_noroll $R/build_ab/lib_pignoroll.so pig
