#!/bin/bash
# A/B of library builds on one bench config, interleaved twice.
#   tools/gpu_ab_cfg.sh CONFIG STEPS TAG...   (cur = the in-tree library;
#   others build_ab/lib_TAG.so).  Output: gpurun_out/r05/ab_CONFIG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
C=$1; S=$2; shift 2
OUT=$R/gpurun_out/r05/ab_$C${AB_TAG:+_$AB_TAG}
mkdir -p "$OUT"
for i in 1 2; do
  for v in "$@"; do
    lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
    [ $v != cur ] && lib=$R/build_ab/lib_$v.so
    OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $C --steps $S --warmup 1 $AB_EXTRA \
      --no-cpu-baseline --parity-roots 8 --no-configs --no-parity-sweep > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -5 "$OUT/$v$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$C $v$i', '%.3f'%d['roofline']['kernel_ms_per_launch'], d['parity']['bit_exact'], d['parity'].get('timed_run_bit_exact'))"
  done
done
