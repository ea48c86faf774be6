#!/bin/bash
# az phase breakdown (wave/lane), C5 line (Bloom superko) + traffic, per-rank lines (c5 131072, c4 8192).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4f
mkdir -p "$OUT"
for lay in wave lane; do
  OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 200 python -u tools/az_phase_probe.py 16384 128 $lay > "$OUT/azphase_$lay.txt" 2>&1 || { tail -5 "$OUT/azphase_$lay.txt"; exit 1; }
  grep AZPHASE "$OUT/azphase_$lay.txt"
done
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-sweep > "$OUT/c5.json" 2> "$OUT/c5.err" || exit 1
timeout -k 10 300 python -u bench.py --config c5 --roots 131072 --steps 5 --warmup 2 --no-cpu-baseline --no-parity-sweep > "$OUT/c5_131072.json" 2> "$OUT/c5_131072.err" || exit 1
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep > "$OUT/c4_8192.json" 2> "$OUT/c4_8192.err" || exit 1
for f in c5 c5_131072 c4_8192; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'] if 'kernel_ms_per_launch' in d['roofline'] else '', d['roofline']['frac'], d.get('parity'))"; done
cd /tmp && export TMPDIR=/tmp
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $c -d "$OUT/c5p$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/c5p$i.log" 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5stats" -o run --output-format csv -- \
    python3 "$R/bench.py" --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep > "$OUT/c5stats.log" 2>&1 || exit 1
echo r4f-done
