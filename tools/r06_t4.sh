#!/bin/bash
# r06: full -m gpu suite (go back on the serial apply; pig two-player playouts
# without the turn walk), then pig's single-bot step: cur against the turn
# walk (pigwalk) and the timing-only no-playout build (pignoroll).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -1 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
lat() {  # tag lib games
  OS_AMD_LIB=$2 timeout -k 10 300 python -u tools/step_latency.py --games "$3" --reps 5 --out $O/lat_$1 > $O/lat_$1.log 2>&1 || { tail -5 $O/lat_$1.log; exit 1; }
  tail -n +3 $O/lat_$1/step_latency.md | sed "s/^/$1 /"
}
CUR=$R/open_spiel-1_amd/os_amd/libos_mcts.so
lat pig_cur $CUR pig
lat pig_walk $R/build_ab/lib_pigwalk.so pig
lat go_cur $CUR "go(board_size=9)"
