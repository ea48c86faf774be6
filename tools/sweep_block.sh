#!/bin/bash
# Block-size sweep of bench.py (no CPU baseline), one JSON line per setting.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for b in "$@"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --block $b \
    > gpurun_out/sweep_$b.json 2> gpurun_out/sweep_$b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep_$b.json'));print('block',$b,'value %.3e'%d['value'],'kernel_ms %.2f'%d['roofline']['kernel_ms_per_launch'],'parity',d['parity']['bit_exact'])"
done
