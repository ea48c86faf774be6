#!/bin/bash
# r05 A/B: hex fill loop unrolled 4 (in-tree) / 8 against not unrolled (take1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_unroll
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "hex" > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/gpu_ab_cfg.sh c4 3 take1 cur unr8 || exit 1
for v in cur take1; do
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $v != cur ] && lib=$R/build_ab/lib_$v.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u tools/step_latency.py --reps 7 --games hex,tic_tac_toe --out "$OUT/lat_$v" > "$OUT/lat_$v.log" 2>&1 || exit 1
done
grep "^| hex\|^| tic" "$OUT"/lat_*/step_latency.md
