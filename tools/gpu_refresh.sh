#!/bin/bash
# GPU-box session that regenerates the committed evidence for the current
# kernels: GPU parity tests, smoke, one bench line per BASELINE config (with
# the CPU baseline), and a `rocprofv3 --kernel-trace --stats` summary of each
# config's bench command.  Every GPU step has its own time limit and the steps
# are chained with &&, so the first failure ends the session.
#   tools/gpu_refresh.sh [configs...]        (default: c2 c3 c4 c5)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/refresh
mkdir -p "$OUT"
cd "$R"
CFGS=${*:-c2 c3 c4 c5}
step_tests() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 && tail -1 "$OUT/pytest_gpu.log" &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
  echo smoke-ok
}
step_cfg() {
  local c=$1
  timeout -k 10 600 python bench.py --config $c --steps 3 --warmup 1 \
    > "$OUT/$c.json" 2> "$OUT/$c.err" &&
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', '%.4g'%d['value'], d['unit'], '%.2f ms'%d['ms_per_step'], d.get('parity'))" &&
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
     -d "$OUT/prof_$c" -o run --output-format csv -- \
     python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline \
     > "$OUT/prof_$c.json" 2> "$OUT/prof_$c.err")
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then step_tests || { echo "tests failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }; fi
for c in $CFGS; do
  step_cfg $c || { echo "config $c failed"; tail -20 "$OUT/$c.err" "$OUT/prof_$c.err"; exit 1; }
done
echo refresh-done
