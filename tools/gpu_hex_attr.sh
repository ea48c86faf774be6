#!/bin/bash
# Timing-only attribution of C4's hex playout (results NOT bit-exact for the
# A/B builds): in-tree build, OS_AB_HEX=1 (no end relaxation), OS_AB_HEX=2
# (no fill loop).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/hex_attr
mkdir -p "$OUT"
for v in cur hexab1 hexab2; do
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $v != cur ] && lib=$R/build_ab/lib_$v.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 \
    --no-cpu-baseline --parity-roots 0 --no-configs --no-parity-sweep > "$OUT/$v.json" 2> "$OUT/$v.err" || { tail -5 "$OUT/$v.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));print('$v', '%.3f'%d['roofline']['kernel_ms_per_launch'])"
done
