#!/bin/bash
# external-evaluator search: GPU tests and the az bench line (+ rocprof stats).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/final
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_az.py tests/test_dirichlet.py > "$OUT/pytest_az.log" 2>&1 || { tail -30 "$OUT/pytest_az.log"; exit 1; }
tail -1 "$OUT/pytest_az.log"
timeout -k 10 600 python -u bench.py --config az > "$OUT/az.json" 2> "$OUT/az.err" || exit 1
python -c "import json;d=json.load(open('$OUT/az.json'));print('az', d['value'], d['ms_per_step'], d['az']['search_only_sims_per_s'], d['parity']['bit_exact'], d['roofline']['pmc_source'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_az" -o run --output-format csv -- python3 "$R/bench.py" --config az --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 0 --no-parity-sweep --az-graph 0 > "$OUT/rocprof_az.log" 2>&1 || exit 1
echo az-done
