#!/bin/bash
# r05 measurement set (one gpurun call per part, each step under its own limit):
#   tests   full -m gpu suite + smoke
#   bench   the driver's default command (+ its rocprof kernel stats), sp and az
#           lines (+ rocprof), C5 per-rank line, 4096-root go9 wave line, step latency
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/final
mkdir -p "$OUT"
case "$1" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
    tail -1 "$OUT/pytest_gpu.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
    tail -1 "$OUT/smoke.log"
    ;;
  bench)
    t0=$(date +%s)
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/default_bench.json" \
      2> "$OUT/default_bench.err" || { tail -20 "$OUT/default_bench.err"; exit 1; }
    echo "default bench wall $(( $(date +%s) - t0 )) s"
    for c in sp az; do
      timeout -k 10 600 python -u bench.py --config $c > "$OUT/$c.json" 2> "$OUT/$c.err" || { tail -20 "$OUT/$c.err"; exit 1; }
      echo "bench $c done"
    done
    timeout -k 10 300 python -u bench.py --config c5 --roots 131072 --steps 10 --warmup 3 \
      --no-cpu-baseline --no-parity-sweep > "$OUT/c5_131072.json" 2> "$OUT/c5_131072.err" || exit 1
    timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 2 \
      --warmup 1 --no-cpu-baseline --no-parity-sweep > "$OUT/g9_wave_4096.json" 2> "$OUT/g9_wave_4096.err" || exit 1
    timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out "$OUT/step_latency" \
      > "$OUT/step_latency.log" 2>&1 || exit 1
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_default" -o run --output-format csv -- \
      python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/rocprof_default.log" 2>&1 || exit 1
    for c in sp az; do
      EXTRA=""
      [ "$c" = az ] && EXTRA="--az-graph 0"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_$c" -o run --output-format csv -- \
        python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 0 $EXTRA \
        > "$OUT/rocprof_$c.log" 2>&1 || exit 1
    done
    find "$OUT" -name "*kernel_trace.csv" -delete
    echo "bench part done"
    ;;
  rocprof)
    # one rocprof run per config, without the parity prefixes and the sweep,
    # so each timed kernel's average is that of the line's own launches
    cd /tmp && export TMPDIR=/tmp
    for c in ${2:-c2 c3 c4 c5 g9}; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_$c" -o run --output-format csv -- \
        python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 0 \
        --no-parity-sweep --no-configs > "$OUT/rocprof_$c.log" 2>&1 || exit 1
      echo "rocprof $c done"
    done
    find "$OUT" -name "*kernel_trace.csv" -delete
    ;;
esac
