#!/bin/bash
# r06 final, call C: the new searches-per-wave GPU test, the default bench
# again (its line now reads the fresh PMC records), then full-size parity of
# every config on the final sources.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/r06/final
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_capi.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_capi.log 2>&1 || { tail -20 $O/pytest_capi.log; exit 1; }
tail -1 $O/pytest_capi.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/default_bench_fresh_pmc.json 2> $O/default_bench_fresh_pmc.err || { tail -5 $O/default_bench_fresh_pmc.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/default_bench_fresh_pmc.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['pmc_source'])"
bash tools/r06_final.sh parity
