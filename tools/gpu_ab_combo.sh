#!/bin/bash
# r05 A/B: OS_UNI_SEL=0 + OS_UNI_MT=1 (build_ab/lib_combo.so) against the
# in-tree build on every wave-layout config and the single-bot latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_combo
mkdir -p "$OUT"
bash tools/gpu_ab_cfg.sh c2 20 cur combo || exit 1
bash tools/gpu_ab_cfg.sh c3 2 cur combo || exit 1
bash tools/gpu_ab_cfg.sh c4 3 cur combo || exit 1
AB_TAG=wave AB_EXTRA="--layout wave --roots 4096" bash tools/gpu_ab_cfg.sh g9 3 cur combo || exit 1
bash tools/gpu_ab_cfg.sh sp 5 cur combo || exit 1
for v in cur combo; do
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $v != cur ] && lib=$R/build_ab/lib_$v.so
  OS_AMD_LIB=$lib timeout -k 10 400 python -u tools/step_latency.py --reps 7 --out "$OUT/lat_$v" > "$OUT/lat_$v.log" 2>&1 || exit 1
done
grep "^| " "$OUT"/lat_*/step_latency.md | grep -v "game\|---" | cut -d'|' -f1,2,4,7
