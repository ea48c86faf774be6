# A/B of the OS_PACE issue-priority pacing: default build (paced) against
# diag/lib_p0.so (OS_PACE=0) on sp; the paced playout loop (diag/lib_rp1.so)
# on c5; then the GPU parity tests of the paced kernels.
set -e
B() { python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('  value %.4g ms/step %.3f parity %s' % (d['value'], d['ms_per_step'], d.get('parity')))"; }
for c in sp c5; do
  for L in open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_p0.so diag/lib_rp1.so; do
    [ $c = sp ] && [ $L = diag/lib_rp1.so ] && continue
    echo "== $c $L"
    OS_AMD_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline | B
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_selfplay.py tests/test_full_configs.py tests/test_arena.py 2>&1 | tail -3
