# A/B: OS_SCREEN_LOG=1 (diag/lib_sl.so) against the default build on C2 and
# C4, then the wave-search parity tests on the variant.
set -e
for L in open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_sl.so open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_sl.so; do
  echo "== c2 $L"
  OS_AMD_LIB=$L timeout -k 10 100 python -u tools/c2_scaling.py connect_four 1024 1024 4096 4096
done
B() { python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('  value %.4g ms/step %.3f parity %s' % (d['value'], d['ms_per_step'], d.get('parity')))"; }
for L in open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_sl.so; do
  echo "== c4 $L"
  OS_AMD_LIB=$L timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 16 | B
done
OS_AMD_LIB=diag/lib_sl.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_selfplay.py tests/test_uct_screen.py tests/test_full_configs.py tests/test_arena.py 2>&1 | tail -2
