#!/bin/bash
# r06 A/B: one bench config on several libraries, interleaved twice.
#   tools/r06_ab.sh OUTNAME "BENCH ARGS" TAG...
#   TAG cur = the in-tree library; others build_ab/lib_TAG.so.
# Prints ms_per_step and the parity flags per run; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
NAME=$1; shift
ARGS=$1; shift
OUT=$R/gpurun_out/r06/$NAME
mkdir -p "$OUT"
for i in 1 2; do
  for v in "$@"; do
    lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
    [ "$v" != cur ] && lib=$R/build_ab/lib_$v.so
    OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py $ARGS --no-cpu-baseline \
      --no-configs --no-parity-sweep > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -5 "$OUT/$v$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));p=d.get('parity',{});print('$NAME $v$i', d['ms_per_step'], d['value'], p.get('bit_exact'), p.get('timed_run_bit_exact'))"
  done
done
