#!/bin/bash
# One GPU-box session of named steps, each under its own time limit, chained
# so that the first failure ends the call (no GPU step runs after a failure).
#   tools/gpu_step.sh tests|smoke|c2|c3w|c3l|c4|c5|sp|prof_c2|prof_c3|boxinfo ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
B="--steps ${STEPS:-3} --warmup 1"
step() {
  case "$1" in
    boxinfo) { nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null;
               python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } \
               > "$OUT/boxinfo.txt" 2>&1 ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
             --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    c2) timeout -k 10 400 python bench.py $B $EXTRA > "$OUT/c2.json" 2> "$OUT/c2.err" ;;
    c3w) timeout -k 10 600 python bench.py --config c3 --layout wave $B --no-cpu-baseline $EXTRA > "$OUT/c3w.json" 2> "$OUT/c3w.err" ;;
    c3l) timeout -k 10 600 python bench.py --config c3 --layout lane $B --no-cpu-baseline $EXTRA > "$OUT/c3l.json" 2> "$OUT/c3l.err" ;;
    c3) timeout -k 10 600 python bench.py --config c3 $B $EXTRA > "$OUT/c3.json" 2> "$OUT/c3.err" ;;
    c4) timeout -k 10 600 python bench.py --config c4 $B $EXTRA > "$OUT/c4.json" 2> "$OUT/c4.err" ;;
    c5) timeout -k 10 600 python bench.py --config c5 $B $EXTRA > "$OUT/c5.json" 2> "$OUT/c5.err" ;;
    sp) timeout -k 10 600 python bench.py --config sp $B $EXTRA > "$OUT/sp.json" 2> "$OUT/sp.err" ;;
    prof_*) c=${1#prof_}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
         -d "$OUT/prof_$c" -o run --output-format csv -- \
         python3 "$R/bench.py" --config $c --steps 3 --warmup 1 --no-cpu-baseline \
         > "$OUT/prof_$c.json" 2> "$OUT/prof_$c.err") ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "== $s $(date +%T)"
  step "$s" || { echo "step $s failed rc=$?"; exit 1; }
done
echo "all steps ok"
