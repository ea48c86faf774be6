#!/bin/bash
# Round-6 measurement on the GPU box, in parts (one gpurun call each; every
# GPU step under its own time limit, stopping at the first failure).  Results
# under gpurun_out/r06/final/.
#   tools/r06_final.sh tests     full -m gpu suite + smoke
#   tools/r06_final.sh bench     the driver's default command
#                                (bench.py --gpus 1 --steps 20 --warmup 5),
#                                plus the sp and az lines
#   tools/r06_final.sh rocprof [CFG...]
#                                rocprofv3 --kernel-trace --stats per config,
#                                and the steady-state per-launch summary
#                                (tools/kernel_steady.py: first launch dropped)
#   tools/r06_final.sh pmc CFG...  PMC passes (tools/pmc_configs.sh)
#   tools/r06_final.sh extras    C5 per-rank line, 4096-root go9 wave line,
#                                single-bot step latency, AZ bot latency
#   tools/r06_final.sh parity [CFG...]  tools/full_parity.py
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/final
mkdir -p "$OUT"
part=$1; shift
CFGS="c2 c3 c4 c5 sp az g9"
case "$part" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || { tail -5 "$OUT/pytest_gpu.log"; exit 1; }
    tail -1 "$OUT/pytest_gpu.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > "$OUT/smoke.log" 2>&1 || exit 1
    tail -1 "$OUT/smoke.log"
    ;;
  bench)
    timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/default_bench.json" \
      2> "$OUT/default_bench.err" || { tail -5 "$OUT/default_bench.err"; exit 1; }
    echo "default bench done"
    for c in sp az; do
      timeout -k 10 600 python -u bench.py --config "$c" > "$OUT/$c.json" 2> "$OUT/$c.err" || exit 1
      echo "bench $c done"
    done
    ;;
  rocprof)
    cd /tmp && export TMPDIR=/tmp
    for c in ${*:-$CFGS}; do
      EXTRA=""
      [ "$c" = az ] && EXTRA="--az-graph 0"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_$c" -o run \
        --output-format csv -- python3 "$R/bench.py" --config "$c" --steps 5 --warmup 2 \
        --no-cpu-baseline --parity-roots 0 --no-parity-sweep --no-configs $EXTRA \
        > "$OUT/rocprof_$c.log" 2>&1 || exit 1
      tr=$(find "$OUT/rocprof_$c" -name "*kernel_trace.csv" | head -1)
      st=$(find "$OUT/rocprof_$c" -name "*kernel_stats.csv" | head -1)
      cp "$st" "$OUT/${c}_kernel_stats.csv"
      python3 "$R/tools/kernel_steady.py" "$tr" --skip 1 --out "$OUT/${c}_kernel_steady.json" \
        > "$OUT/${c}_kernel_steady.txt" || exit 1
      head -2 "$OUT/${c}_kernel_steady.txt"
      python3 - "$OUT/rocprof_$c.log" "$OUT/${c}_rocprof_line.json" <<'PY'
import json, sys
for line in open(sys.argv[1]):
  line = line.strip()
  if line.startswith("{") and '"metric"' in line:
    open(sys.argv[2], "w").write(line + "\n")
PY
      rm -rf "$OUT/rocprof_$c"
    done
    ;;
  pmc)
    bash "$R/tools/pmc_configs.sh" "$@" || exit 1
    ;;
  extras)
    timeout -k 10 300 python -u bench.py --config c5 --roots 131072 --steps 10 --warmup 3 \
      --no-cpu-baseline --no-parity-sweep --no-configs > "$OUT/c5_131072.json" \
      2> "$OUT/c5_131072.err" || exit 1
    timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 2 \
      --warmup 1 --no-cpu-baseline --no-parity-sweep --no-configs > "$OUT/g9_wave_4096.json" \
      2> "$OUT/g9_wave_4096.err" || exit 1
    timeout -k 10 600 python -u tools/step_latency.py --reps 7 --out "$OUT/step_latency" \
      > "$OUT/step_latency.log" 2>&1 || exit 1
    timeout -k 10 300 python -u tools/step_latency.py --az --reps 5 --out "$OUT/step_latency" \
      > "$OUT/az_latency.log" 2>&1 || exit 1
    cat "$OUT/step_latency/step_latency.md" "$OUT/step_latency/az_step_latency.md"
    ;;
  parity)
    ONLY=""
    [ $# -gt 0 ] && ONLY="--only $(echo "$@" | tr ' ' ',')"
    timeout -k 10 1100 python -u tools/full_parity.py --out "$OUT/full_parity.json" $ONLY \
      > "$OUT/full_parity.txt" 2>&1 || { tail -5 "$OUT/full_parity.txt"; exit 1; }
    tail -12 "$OUT/full_parity.txt"
    ;;
esac
echo "r06_final $part done"
