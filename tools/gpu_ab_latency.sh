#!/bin/bash
# A/B of single-bot step latency (tools/step_latency.py) between the in-tree
# library and build_ab/lib_TAG.so, interleaved twice.
#   tools/gpu_ab_latency.sh TAG [games]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
T=$1; G=${2:-tic_tac_toe,connect_four}
OUT=$R/gpurun_out/r05/ab_lat_$T
mkdir -p "$OUT"
for i in 1 2; do
  for v in cur $T; do
    lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
    [ $v != cur ] && lib=$R/build_ab/lib_$v.so
    OS_AMD_LIB=$lib timeout -k 10 300 python -u tools/step_latency.py --reps 9 --games "$G" \
      --out "$OUT/${v}_$i" > "$OUT/${v}_$i.log" 2>&1 || { tail -5 "$OUT/${v}_$i.log"; exit 1; }
    echo "== $v $i"; grep "^|" "$OUT/${v}_$i/step_latency.md" | tail -n +3 | cut -d'|' -f2,4,5,7,8
  done
done
