#!/bin/bash
# r05: numpy-policy parity subset, single-search phase profile, step latency.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_np.log" 2>&1 || { tail -30 "$OUT/pytest_np.log"; exit 1; }
tail -1 "$OUT/pytest_np.log"
(cd tools && OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 300 python -u phase_single.py 1000 > "$OUT/phase_single.txt" 2>&1) || { tail -20 "$OUT/phase_single.txt"; exit 1; }
grep PHASE1 "$OUT/phase_single.txt"
timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out "$OUT/step_latency" \
  > "$OUT/step_latency.log" 2>&1 || { tail -20 "$OUT/step_latency.log"; exit 1; }
cat "$OUT/step_latency/step_latency.md"
