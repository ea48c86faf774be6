#!/bin/bash
# Round-4 final, part 4: full -m gpu suite + smoke, C5 per-rank line, single-bot step latency table.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_final.sh tests || exit 1
mkdir -p gpurun_out/r4final
timeout -k 10 300 python -u bench.py --config c5 --roots 131072 --steps 10 --warmup 3 --no-cpu-baseline --no-parity-sweep > gpurun_out/r4final/c5_131072.json 2> gpurun_out/r4final/c5_131072.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r4final/c5_131072.json'));print('c5 per-rank 131072', d['value'], d['ms_per_step'], d['parity'])"
timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out gpurun_out/r4final/step_latency > gpurun_out/r4final/step_latency.log 2>&1 || { tail -20 gpurun_out/r4final/step_latency.log; exit 1; }
cat gpurun_out/r4final/step_latency/step_latency.md
