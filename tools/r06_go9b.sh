#!/bin/bash
# r06 Go9 follow-ups: C5 with k_rollouts at five waves per SIMD
# (build_ab/lib_rocc5.so, -DOS_ROLL_OCC=5), and g9's k_lsearch width
# (16 / 32 / 64 searches per wave) at 32768 and 65536 roots.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/go9b
mkdir -p "$OUT"
bash tools/r06_ab.sh go9b/c5 "--config c5" cur rocc5 || exit 1
bash tools/r06_ab.sh go9b/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur rocc5 || exit 1
for roots in 65536 32768; do
  for b in 16 32 64; do
    timeout -k 10 300 python -u bench.py --config g9 --roots $roots --block $b --steps 2 --warmup 1 \
      --no-cpu-baseline --no-configs --no-parity-sweep > "$OUT/g9_${roots}_$b.json" \
      2> "$OUT/g9_${roots}_$b.err" || { tail -5 "$OUT/g9_${roots}_$b.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/g9_${roots}_$b.json'));p=d.get('parity',{});print('g9 $roots $b', d['ms_per_step'], d['value'], p.get('bit_exact'), p.get('timed_run_bit_exact'))"
  done
done
echo "r06_go9b done"
