# A/B: OS_SEL_PREFETCH=1 (diag/lib_pf.so) against the default build on C2,
# then the wave-search parity tests on the variant.
set -e
for L in open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_pf.so open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_pf.so; do
  echo "== c2 $L"
  OS_AMD_LIB=$L timeout -k 10 100 python -u tools/c2_scaling.py connect_four 1024 1024 4096 4096
done
OS_AMD_LIB=diag/lib_pf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_selfplay.py 2>&1 | tail -2
