#!/bin/bash
# End-of-round measurement on the GPU box, in three parts (one gpurun call
# each, every step under its own time limit, stopping at the first failure):
#   tools/gpu_final.sh tests    full -m gpu suite + smoke
#   tools/gpu_final.sh bench    one bench line per config (with cpu_baseline)
#                               + rocprofv3 --kernel-trace --stats of each
#   tools/gpu_final.sh pmc CFG...  PMC passes (tools/pmc_configs.sh)
#   tools/gpu_final.sh extras   C5 per-rank line, 4096-root go9 wave line,
#                               single-bot step latency (tools/step_latency.py)
# Results under gpurun_out/final/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/final
mkdir -p "$OUT"
part=$1; shift
CFGS="c2 c3 c4 c5 sp az g9"
case "$part" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1 || exit 1
    tail -1 "$OUT/pytest_gpu.log"
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
      > "$OUT/smoke.log" 2>&1 || exit 1
    tail -1 "$OUT/smoke.log"
    ;;
  bench)
    for c in ${*:-$CFGS}; do
      timeout -k 10 600 python -u bench.py --config "$c" > "$OUT/$c.json" 2> "$OUT/$c.err" || exit 1
      echo "bench $c done"
    done
    cd /tmp && export TMPDIR=/tmp
    for c in ${*:-$CFGS}; do
      EXTRA=""
      [ "$c" = az ] && EXTRA="--az-graph 0"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_$c" -o run \
        --output-format csv -- python3 "$R/bench.py" --config "$c" --steps 3 --warmup 1 \
        --no-cpu-baseline --parity-roots 0 --no-parity-sweep $EXTRA > "$OUT/rocprof_$c.log" 2>&1 || exit 1
      echo "rocprof $c done"
    done
    ;;
  pmc)
    bash "$R/tools/pmc_configs.sh" "$@" || exit 1
    ;;
  extras)
    # per-rank C5 line (8-GPU share of the 2^20 playouts), the 4096-root go9
    # wave line, and the single-bot step latency table
    timeout -k 10 300 python -u bench.py --config c5 --roots 131072 --steps 10 --warmup 3 \
      --no-cpu-baseline --no-parity-sweep > "$OUT/c5_131072.json" 2> "$OUT/c5_131072.err" || exit 1
    timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 2 \
      --warmup 1 --no-cpu-baseline --no-parity-sweep > "$OUT/g9_wave_4096.json" \
      2> "$OUT/g9_wave_4096.err" || exit 1
    timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out "$OUT/step_latency" \
      > "$OUT/step_latency.log" 2>&1 || exit 1
    ;;
esac
echo "gpu_final $part done"
