#!/bin/bash
# GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; steps are chained with && so the
# script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
STEP=${1:-all}

run_tests() {
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
}
run_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
}
run_bench() {
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
}
run_prof() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
     -d "$OUT/prof" -o run --output-format csv -- \
     python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
     > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err")
}

case "$STEP" in
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  all) run_tests && run_smoke && run_bench && run_prof ;;
  quick) run_smoke && run_bench && run_prof ;;
esac
echo "exit=$?"
