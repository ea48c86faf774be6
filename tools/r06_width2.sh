#!/bin/bash
# r06: k_lsearch<Go9> width (searches per wave) on the final sources, g9 at
# 65536 and 32768 roots, 16 / 32 / 64 lanes (bench.py --block).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/width2
mkdir -p "$OUT"
for roots in 65536 32768; do
  for b in 16 32 64; do
    timeout -k 10 300 python -u bench.py --config g9 --roots $roots --block $b --steps 2 --warmup 1 \
      --no-cpu-baseline --no-configs --no-parity-sweep > "$OUT/g9_${roots}_$b.json" \
      2> "$OUT/g9_${roots}_$b.err" || { tail -5 "$OUT/g9_${roots}_$b.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/g9_${roots}_$b.json'));p=d.get('parity',{});print('g9 $roots $b', d['ms_per_step'], d['value'], p.get('bit_exact'), p.get('timed_run_bit_exact'))"
  done
done
echo "r06_width2 done"
