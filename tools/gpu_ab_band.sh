#!/bin/bash
# r05 A/B: UCT screen settled by one band ballot (in-tree, OS_SCREEN_BAND=1)
# against the identity test always (build_ab/lib_band0.so).  GPU suite on the
# in-tree build first, then C2 / C4 / C3 timings interleaved, then the
# selection sub-phases of the band build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_band
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run() {  # tag config steps warmup run
  lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  [ $1 != cur ] && lib=$R/build_ab/lib_$1.so
  OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $2 --steps $3 --warmup $4 \
    --no-cpu-baseline --parity-roots 8 --no-parity-sweep --no-configs > "$OUT/$2_$1_$5.json" 2> "$OUT/$2_$1_$5.err" || { tail -5 "$OUT/$2_$1_$5.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$2_$1_$5.json'));print('$2 $1 $5', '%.3f'%d['roofline']['kernel_ms_per_launch'], '%.3f'%d['ms_per_step'], d['parity']['bit_exact'], d['parity'].get('timed_run_bit_exact'))"
}
A=${AB_BASE:-band0}
for i in 1 2 3; do run $A c2 20 5 $i || exit 1; run cur c2 20 5 $i || exit 1; done
if [ -z "$AB_C2_ONLY" ]; then
  for i in 1 2; do run $A c4 3 1 $i || exit 1; run cur c4 3 1 $i || exit 1; done
  run $A c3 2 1 1 || exit 1; run cur c3 2 1 1 || exit 1
fi
OS_AMD_LIB=$R/build_ab/lib_psel.so timeout -k 10 300 python -u tools/phase_single.py 1000 \
  > "$OUT/phase_single.txt" 2>&1 || exit 1
OS_AMD_LIB=$R/build_ab/lib_psel.so timeout -k 10 300 python -u tools/phase_probe.py 4096 1024 connect_four \
  > "$OUT/phase_c2.txt" 2>&1 || exit 1
grep PHASE "$OUT"/phase*.txt | grep -v "go(board"
