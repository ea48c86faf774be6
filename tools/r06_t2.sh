#!/bin/bash
# r06: full -m gpu suite, then pig's single-bot step with the LDS arena (cur)
# against the HBM arena (chlds0), and go on the wave layout with the parallel
# apply (cur) against the serial one (gopar0): 4096-root go9 and the go bot.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/t2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
lat() {  # tag lib games
  OS_AMD_LIB=$2 timeout -k 10 300 python -u tools/step_latency.py --games "$3" --reps 5 --out $O/lat_$1 > $O/lat_$1.log 2>&1 || { tail -5 $O/lat_$1.log; exit 1; }
  tail -n +3 $O/lat_$1/step_latency.md | sed "s/^/$1 /"
}
CUR=$R/open_spiel-1_amd/os_amd/libos_mcts.so
lat pig_cur $CUR pig
lat pig_hbm $R/build_ab/lib_chlds0.so pig
bash tools/r06_ab.sh g9w "--config g9 --roots 4096 --layout wave --steps 3 --warmup 1 --parity-roots 8" cur gopar0 || exit 1
lat go_cur $CUR "go(board_size=9)"
lat go_serial $R/build_ab/lib_gopar0.so "go(board_size=9)"
