#!/bin/bash
# r06 final, call D (after the Pig2 change moved the kernel-source hash):
# rocprof kernel statistics + steady summaries, PMC passes, the driver's
# default bench, full-size parity -- all on the final sources.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_final.sh rocprof c2 c3 c4 c5 sp az g9 && \
bash tools/r06_final.sh pmc c2 c3 c4 c5 sp az g9 && \
python3 tools/pmc_merge.py && \
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final/default_bench_d.json 2> gpurun_out/r06/final/default_bench_d.err && \
bash tools/r06_final.sh parity
