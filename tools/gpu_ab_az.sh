#!/bin/bash
# A/B of the az graph replay (round 5): first the pending check read behind
# the next queued batch (OS_AZ_SERIAL_CHECK, since removed), then the first
# replay batch running to max_simulations + 1 rounds (OS_AZ_FIRST=8 keeps
# the old batch of 8; tags: serial = old form, overlap = new form).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r05/ab_az
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_az.py -x -q --timeout 200 --timeout-method thread -k graph \
  > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2 3; do
  for v in serial overlap; do
    E=""; [ $v = serial ] && E="OS_AZ_FIRST=8"
    env $E timeout -k 10 300 python -u bench.py --config az --steps 10 --warmup 2 --no-cpu-baseline \
      --parity-roots 8 > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -5 "$OUT/$v$i.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v$i', '%.4e'%d['value'], '%.3f'%d['ms_per_step'], d['parity']['bit_exact'])"
  done
done
