#!/bin/bash
# A/B of library builds under build_ab/ (lib_<tag>.so) on the bench workload.
# Each run has its own time limit; stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab
mkdir -p "$OUT"
cd "$R"
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --parity-roots 8"}
for tag in "$@"; do
  OS_AMD_LIB=$R/build_ab/lib_$tag.so timeout -k 10 300 python bench.py $ARGS \
    > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || exit 1
  python -c "import json,sys; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', '%.4e'%d['value'], '%.3f ms'%d['roofline']['kernel_ms_per_launch'], d['parity']['bit_exact'])"
done
