#!/bin/bash
# go wave search: parity (test_gpu_parity go cases), 4096-root g9 wave line, SQ instruction mix.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/${1:-gow}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "go" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 8 > "$OUT/g9w.json" 2> "$OUT/g9w.err" || exit 1
python -c "import json;d=json.load(open('$OUT/g9w.json'));print('g9w4096', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['parity']['timed_run_bit_exact'])"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d "$OUT/pmc" -o run --output-format csv -- \
  python3 "$R/bench.py" --config g9 --layout wave --roots 4096 --steps 1 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/pmc.log" 2>&1 || exit 1
cd "$R" && python3 tools/pmc_sum.py k_wsearch "$OUT/pmc"
