#!/bin/bash
# r05: az step kernel breakdown (rocprof) + breakthrough phase profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/e
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/az" -o run --output-format csv -- \
  python3 "$R/bench.py" --config az --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 0 \
  > "$OUT/az.log" 2>&1 || { tail -5 "$OUT/az.log"; exit 1; }
find "$OUT/az" -name "*kernel_stats.csv" -exec cp {} "$OUT/az_kernel_stats.csv" \;
head -20 "$OUT/az_kernel_stats.csv" | cut -c1-160
cd "$R/tools" && OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 300 python -u phase_probe.py 4096 2048 breakthrough > "$OUT/phase_bt.txt" 2>&1 || { tail -5 "$OUT/phase_bt.txt"; exit 1; }
grep PHASE "$OUT/phase_bt.txt"
