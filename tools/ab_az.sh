# A/B of k_az_step builds (default vs diag/lib_azold.so) and searches per wave.
set -e
B() { python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('  value %.4g ms/step %.3f k_az_step %.3f ms/launch x %d parity %s' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['az']['launches_per_step'], d.get('parity',{}).get('bit_exact')))"; }
for L in open_spiel-1_amd/os_amd/libos_mcts.so diag/lib_azold.so; do
  for b in 64 16; do
    echo "== az $L block $b"
    OS_AMD_LIB=$L timeout -k 10 300 python -u bench.py --config az --steps 3 --warmup 1 --no-cpu-baseline --block $b | B
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_az.py 2>&1 | tail -2
