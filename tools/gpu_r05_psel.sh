#!/bin/bash
# r05: selection sub-phases (build_ab/lib_psel.so: OS_PHASE_TIMING + OS_PHASE_SEL);
# for non-go games the go_* columns are sel_load / sel_score / sel_apply / sel_path.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/psel
mkdir -p "$OUT"
OS_AMD_LIB=$R/build_ab/lib_psel.so timeout -k 10 300 python -u tools/phase_single.py 1000 \
  > "$OUT/phase_single.txt" 2>&1 || { tail -5 "$OUT/phase_single.txt"; exit 1; }
OS_AMD_LIB=$R/build_ab/lib_psel.so timeout -k 10 300 python -u tools/phase_probe.py 4096 1024 connect_four \
  > "$OUT/phase_c2.txt" 2>&1 || { tail -5 "$OUT/phase_c2.txt"; exit 1; }
grep PHASE "$OUT"/*.txt
