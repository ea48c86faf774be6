#!/bin/bash
# r05: C2 under compile-time knob variants (build_ab/lib_TAG.so) against the
# in-tree build, twice each, interleaved with the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/knobs
mkdir -p "$OUT"
run() {
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $1 != cur ] && lib=$R/build_ab/lib_$1.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 \
    --no-cpu-baseline --parity-roots 8 --no-configs --no-parity-sweep > "$OUT/$1_$2.json" 2> "$OUT/$1_$2.err" || { tail -5 "$OUT/$1_$2.err"; return 1; }
  python -c "import json;d=json.load(open('$OUT/$1_$2.json'));print('$1 $2', '%.3f'%d['roofline']['kernel_ms_per_launch'], d['parity']['bit_exact'], d['parity']['timed_run_bit_exact'])"
}
for i in 1 2; do
  for v in cur "$@"; do run $v $i || exit 1; done
done
