#!/bin/bash
# r06 timing attribution (not bit-exact): go's superko bucket walk dropped
# (build_ab/lib_nowalk.so, -DOS_GO_NOWALK=1) against the in-tree library, g9
# and C5, to size what the walk behind the Bloom filter still costs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/r06/nowalk
mkdir -p "$OUT"
for cfg in g9 c5; do
  for v in cur nowalk cur nowalk; do
    lib=$R/open_spiel-1_amd/os_amd/libos_mcts.so
    [ "$v" != cur ] && lib=$R/build_ab/lib_$v.so
    OS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-configs \
      --no-parity-sweep --parity-roots 0 > "$OUT/${cfg}_$v.json" 2> "$OUT/${cfg}_$v.err" || { tail -5 "$OUT/${cfg}_$v.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/${cfg}_$v.json'));print('$cfg $v', d['ms_per_step'])"
  done
done
echo "r06_nowalk done"
