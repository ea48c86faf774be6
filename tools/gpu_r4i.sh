#!/bin/bash
# az k_waz_step occupancy A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4i
mkdir -p "$OUT"
for tag in main noatom; do
  lib=$R/build_ab/lib_$tag.so; [ $tag = main ] && lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  OS_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --config az --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 8 > "$OUT/az_$tag.json" 2> "$OUT/az_$tag.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/az_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['az']['search_only_sims_per_s'], d['parity']['bit_exact'])"
done
echo r4i-done
