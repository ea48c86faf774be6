#!/bin/bash
# go phase profile (new lane-label rollout), az wave-vs-lane A/B, g9 traffic attribution.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4e
mkdir -p "$OUT"
OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 200 python -u tools/phase_probe.py 64 256 go > "$OUT/phase_go.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/phase_go.txt"
for lay in wave lane; do
  timeout -k 10 300 python -u bench.py --config az --az-layout $lay --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 8 > "$OUT/az_$lay.json" 2> "$OUT/az_$lay.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/az_$lay.json'));print('az $lay', d['value'], d['ms_per_step'], d['az']['k_az_step_ms_total'], d['az']['search_only_sims_per_s'], d['parity']['bit_exact'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_az" -o run --output-format csv -- python3 "$R/bench.py" --config az --steps 2 --warmup 1 --no-cpu-baseline --parity-roots 0 --az-graph 0 > "$OUT/rocprof_az.log" 2>&1 || exit 1
cd "$R"
find "$OUT/rocprof_az" -name "*kernel_stats.csv" -exec head -5 {} \;
timeout -k 10 900 bash tools/g9_ab.sh default nomt nolog none > "$OUT/g9ab.log" 2>&1 || { tail -5 "$OUT/g9ab.log"; exit 1; }
tail -6 "$OUT/g9ab.log"
