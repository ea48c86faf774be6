#!/bin/bash
# az (fused heads, threaded prepare); go wave rollout with lane neighbourhoods.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r4l
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_az.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --config az --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 8 > "$OUT/az.json" 2> "$OUT/az.err" || exit 1
python -c "import json;d=json.load(open('$OUT/az.json'));print('az', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['az'], d['parity']['bit_exact'])"
timeout -k 10 300 python -u bench.py --config g9 --layout wave --roots 4096 --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 8 > "$OUT/g9w.json" 2> "$OUT/g9w.err" || exit 1
python -c "import json;d=json.load(open('$OUT/g9w.json'));print('g9w4096', d['value'], d['ms_per_step'], d['parity'])"
OS_AMD_LIB=$R/build_ab/lib_phase.so timeout -k 10 200 python -u tools/phase_probe.py 64 256 go > "$OUT/phase_go.txt" 2>&1 || exit 1
grep PHASE "$OUT/phase_go.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rocprof_az" -o run --output-format csv -- python3 "$R/bench.py" --config az --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sweep --parity-roots 0 > "$OUT/rocprof_az.log" 2>&1 || exit 1
echo r4l-done
