#!/bin/bash
# Node-cache A/B: parity of the wave kernels with the cache, then C2 / C3 timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
OS_AMD_LIB=$R/build_ab/lib_nc256.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_arena.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nc_parity.log 2>&1 || exit 1
tail -2 gpurun_out/nc_parity.log
bash tools/ab.sh nc0 nc128 nc256 nc512 nc0 nc256 || exit 1
BENCH_ARGS="--config c3 --steps 1 --warmup 1 --no-cpu-baseline --parity-roots 8" bash tools/ab.sh nc0 nc256 || exit 1
BENCH_ARGS="--config c4 --steps 2 --warmup 1 --no-cpu-baseline --parity-roots 8" bash tools/ab.sh nc0 nc256
