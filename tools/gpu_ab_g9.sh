#!/bin/bash
# r05 A/B: g9 (go9 lane search, 65536 x 256) on A/B builds, interleaved.
#   tools/gpu_ab_g9.sh TAG...   (cur = the in-tree library; others build_ab/lib_TAG.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_g9
mkdir -p "$OUT"
for i in 1 2; do
  for v in "$@"; do
    lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
    [ $v != cur ] && lib=$R/build_ab/lib_$v.so
    OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config g9 --steps 3 --warmup 1 \
      --no-cpu-baseline --parity-roots 8 --no-configs --no-parity-sweep > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -5 "$OUT/$v$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v$i', d['ms_per_step'], d['parity']['bit_exact'], d['parity']['timed_run_bit_exact'])"
  done
done
