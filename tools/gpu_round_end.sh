#!/bin/bash
# End-of-round check on the final tree: full -m gpu suite + smoke, then the
# default bench line (C2, with the parity sweep) as the driver runs it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_final.sh tests || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/final/default_bench.json 2> gpurun_out/final/default_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/final/default_bench.json'));print('default', d['metric'], d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['parity_sweep']['all_bit_exact'], d['roofline']['pmc_source'])"
