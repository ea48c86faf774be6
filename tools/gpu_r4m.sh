#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_gow.sh gow1 || exit 1
mkdir -p gpurun_out/r4m
timeout -k 10 500 python -u tools/step_latency.py --reps 7 --out gpurun_out/r4m/step_latency > gpurun_out/r4m/step_latency.log 2>&1 || { tail -20 gpurun_out/r4m/step_latency.log; exit 1; }
cat gpurun_out/r4m/step_latency/step_latency.md
