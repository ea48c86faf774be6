#!/bin/bash
# r06 timing attribution (not bit-exact): g9 with k_lsearch's playouts
# skipped (build_ab/lib_noroll.so, -DOS_AB_LANE_NOROLL=1: every leaf scores 0)
# against the in-tree library, to size the tree part of the step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/noroll
mkdir -p "$OUT"
for v in cur noroll cur noroll; do
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ "$v" != cur ] && lib=$R/build_ab/lib_$v.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config g9 --no-cpu-baseline --no-configs \
    --no-parity-sweep --parity-roots 0 > "$OUT/$v.json" 2> "$OUT/$v.err" || { tail -5 "$OUT/$v.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$v.json'));print('$v', d['ms_per_step'])"
done
echo "r06_noroll done"
