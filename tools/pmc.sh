#!/bin/bash
# rocprofv3 PMC passes over bench.py (kernel-trace + counters only; never
# combined with sys/runtime traces).  One pass per counter group.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
i=0
while [ $# -gt 0 ]; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $1 -d "$OUT/p$i" -o run \
    --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || exit 1
  shift
done
echo pmc-done
