#!/bin/bash
# C2 / C4 pacing-interval A/B (OS_PACE_EVERY 32 default, 64, 128).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/pace
mkdir -p "$OUT"
for tag in main pe64 pe128 main; do
  lib=$R/build_ab/lib_$tag.so; [ $tag = main ] && lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
  for c in c2 c4; do
    OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-parity-sweep --parity-roots 4 > "$OUT/${c}_$tag.json" 2> "$OUT/${c}_$tag.err" || exit 1
    python -c "import json;d=json.load(open('$OUT/${c}_$tag.json'));print('$c $tag', d['value'], d['ms_per_step'], d['parity']['bit_exact'])"
  done
done
timeout -k 10 300 python -u bench.py --config c5 --roots 131072 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-sweep > "$OUT/c5_131072.json" 2> "$OUT/c5_131072.err" || exit 1
python -c "import json;d=json.load(open('$OUT/c5_131072.json'));print('c5 per-rank 131072', d['value'], d['ms_per_step'], d['parity'])"
mkdir -p gpurun_out/r4n
timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out gpurun_out/r4n/step_latency > gpurun_out/r4n/step_latency.log 2>&1 || { tail -20 gpurun_out/r4n/step_latency.log; exit 1; }
cat gpurun_out/r4n/step_latency/step_latency.md
