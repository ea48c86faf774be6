#!/bin/bash
# GPU suite, then the search bench with the page pool vs the reserved arena
# (and optionally build_ab/lib_$BASE.so on the reserved arena).
set -e
mkdir -p gpurun_out/arena
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/arena/gpu_tests.log 2>&1
tail -1 gpurun_out/arena/gpu_tests.log
run() {  # cfg arena tag [lib]
  OS_AMD_LIB=${4:-} timeout -k 10 300 python bench.py --config $1 --arena $2 --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 8 > gpurun_out/arena/${1}_$3.json 2> gpurun_out/arena/${1}_$3.err
  python -c "import json; d=json.load(open('gpurun_out/arena/${1}_$3.json')); a=d.get('arena',{}); print('$1', '$3', '%.4e'%d['value'], '%.2f ms'%d['roofline']['kernel_ms_per_launch'], d['parity']['bit_exact'], 'arena %.2f of %.2f GB, pages %d/%d' % (a.get('arena_bytes',0)/1e9, a.get('reserved_bytes',0)/1e9, a.get('pages_used',0), a.get('pool_pages_or_chunk_roots',0)))"
}
for cfg in ${CFGS:-c3 c2}; do
  for i in 1 2; do
    [ -n "$BASE" ] && run $cfg reserved base $PWD/build_ab/lib_$BASE.so
    run $cfg reserved reserved
    run $cfg paged paged
  done
done
