# Default build: C2 / C4 times and the full GPU suite.
set -e
timeout -k 10 100 python -u tools/c2_scaling.py connect_four 1024 1024 4096 4096
B() { python3 -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('  value %.4g ms/step %.3f parity %s' % (d['value'], d['ms_per_step'], d.get('parity')))"; }
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --parity-roots 16 | B
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
