#!/bin/bash
# C5 traffic A/B (k_rollouts<Go> buffer layouts, OS_ROLL_AOS): per build tag
# the c5 bench line and one FETCH_SIZE/WRITE_SIZE pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/c5ab
for tag in "$@"; do
  BENCH_ARGS="--config c5 --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 8" \
    bash tools/ab.sh "$tag" || exit 1
  cd /tmp && export TMPDIR=/tmp
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do  # one TCC counter set per run
    i=$((i+1))
    OS_AMD_LIB=$R/build_ab/lib_$tag.so timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c \
      -d "$R/gpurun_out/c5ab/$tag/p$i" -o run --output-format csv -- \
      python3 "$R/bench.py" --config c5 --steps 1 --warmup 1 --no-cpu-baseline --parity-roots 0 \
      > "$R/gpurun_out/c5ab/$tag/p$i.log" 2>&1 || exit 1
  done
  cd "$R"
done
echo c5ab-done
