#!/bin/bash
# r05 A/B: C3 (breakthrough 65536 x 2048) on two builds, interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_c3
mkdir -p "$OUT"
for i in 1 2; do
  for v in base cur; do
    lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
    [ $v = base ] && lib=$R/build_ab/lib_base.so
    OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 \
      --no-cpu-baseline --parity-roots 8 --no-configs > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -5 "$OUT/$v$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v$i', d['ms_per_step'], d['parity']['bit_exact'], d['parity']['timed_run_bit_exact'])"
  done
done
