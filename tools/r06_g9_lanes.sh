#!/bin/bash
# r06: go9 search (256 sims) by root count, layout and k_lsearch block width.
# One line per run: roots layout block ms_per_step sims/s bit_exact.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/g9_lanes
mkdir -p "$OUT"
run() {  # roots layout block steps
  local tag=$1_$2_$3
  timeout -k 10 300 python -u bench.py --config g9 --roots $1 --layout $2 --block $3 --steps $4 \
    --warmup 1 --parity-roots 8 --no-cpu-baseline --no-configs --no-parity-sweep \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', round(d['ms_per_step'],2), '%.3e'%d['value'], d['parity']['bit_exact'], d['parity']['timed_run_bit_exact'])"
}
for n in 4096 8192; do run $n wave 0 3; done
for n in 4096 8192 16384 32768 65536; do
  for b in 16 32 64; do run $n lane $b 3; done
done
run 131072 lane 32 2
run 131072 lane 64 2
