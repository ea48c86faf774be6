#!/bin/bash
# r05: phase profiles on the phase-timing build (build_ab/lib_phase.so):
# single searches (all games) and 4096-root batches of connect_four and go9.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/phase
mkdir -p "$OUT"
OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 300 python -u tools/phase_single.py 1000 \
  > "$OUT/phase_single.txt" 2>&1 || { tail -5 "$OUT/phase_single.txt"; exit 1; }
OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 300 python -u tools/phase_probe.py 4096 1024 connect_four \
  > "$OUT/phase_c2.txt" 2>&1 || { tail -5 "$OUT/phase_c2.txt"; exit 1; }
OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 300 python -u tools/phase_probe.py 4096 1024 go \
  > "$OUT/phase_go4096.txt" 2>&1 || { tail -5 "$OUT/phase_go4096.txt"; exit 1; }
grep PHASE "$OUT"/*.txt
