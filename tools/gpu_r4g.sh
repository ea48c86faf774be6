#!/bin/bash
# az phase breakdown (sampled), C5 / g9 Bloom + lazy-atari A/B, SQ instruction mix of go wave search.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4g
mkdir -p "$OUT"
OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 200 python -u tools/az_phase_probe.py 16384 128 wave > "$OUT/azphase_wave.txt" 2>&1 || { tail -5 "$OUT/azphase_wave.txt"; exit 1; }
grep AZPHASE "$OUT/azphase_wave.txt"
for tag in main bloom0 lazy0 both0; do
  lib=$R/build_ab/lib_$tag.so; [ $tag = main ] && lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  OS_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-sweep > "$OUT/c5_$tag.json" 2> "$OUT/c5_$tag.err" || exit 1
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config g9 --layout lane --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 8 > "$OUT/g9_$tag.json" 2> "$OUT/g9_$tag.err" || exit 1
  python -c "import json;a=json.load(open('$OUT/c5_$tag.json'));b=json.load(open('$OUT/g9_$tag.json'));print('$tag c5', a['value'], a['ms_per_step'], a['parity']['bit_exact'], 'g9', b['value'], b['ms_per_step'], b['parity'])"
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d "$OUT/g9w$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config g9 --layout wave --roots 4096 --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/g9w$i.log" 2>&1 || exit 1
done
echo r4g-done
