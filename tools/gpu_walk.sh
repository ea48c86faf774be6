#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/walk
mkdir -p "$OUT"
for tag in main nowalk; do
  lib=$R/build_ab/lib_$tag.so; [ $tag = main ] && lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  for c in c5 g9; do
    OS_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/${c}_$tag.json" 2> "$OUT/${c}_$tag.err" || exit 1
    python -c "import json;d=json.load(open('$OUT/${c}_$tag.json'));print('$c $tag', d['value'], d['ms_per_step'])"
  done
done
