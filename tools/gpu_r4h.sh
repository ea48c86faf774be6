#!/bin/bash
# az wave residency; SQ instruction mix of go wave search (4096 roots).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4h
mkdir -p "$OUT"
OS_AMD_LIB=$R/build_ab/lib_wt.so timeout -k 10 200 python -u tools/az_wave_times.py 16384 128 > "$OUT/azwt.txt" 2>&1 || { tail -5 "$OUT/azwt.txt"; exit 1; }
grep AZWT "$OUT/azwt.txt"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d "$OUT/g9w$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config g9 --layout wave --roots 4096 --steps 1 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/g9w$i.log" 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P -d "$OUT/azw$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config az --steps 1 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 0 --az-graph 0 > "$OUT/azw$i.log" 2>&1 || exit 1
done
echo r4h-done
