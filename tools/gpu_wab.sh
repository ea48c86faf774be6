#!/bin/bash
# g9 wave (4096 roots) A/B: current, label lookup with branches, two-step legal.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/wab
mkdir -p "$OUT"
for tag in main labat legal2 main; do
  lib=$R/build_ab/lib_$tag.so; [ $tag = main ] && lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 4 > "$OUT/g9w_$tag.json" 2> "$OUT/g9w_$tag.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/g9w_$tag.json'));print('g9w $tag', d['value'], d['ms_per_step'], d['parity']['bit_exact'])"
done
for tag in main legal2; do
  lib=$R/build_ab/lib_$tag.so; [ $tag = main ] && lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/c5_$tag.json" 2> "$OUT/c5_$tag.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/c5_$tag.json'));print('c5 $tag', d['value'], d['ms_per_step'])"
done
