#!/bin/bash
# PMC passes (tools/pmc.sh) over the bench command of each named config;
# results land in gpurun_out/pmc_<config>/.  Summarise afterwards on the host
# with tools/pmc_summary.py.
#   tools/pmc_configs.sh [configs...]        (default: c2 c4)
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=${*:-c2 c4}
P1="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD"
for c in $CFGS; do
  rm -rf "$R/gpurun_out/pmc"
  EXTRA=""
  [ "$c" = az ] && EXTRA="--az-graph 0"  # eager rounds: one traced dispatch per k_az_step
  BENCH_ARGS="--config $c --steps 2 --warmup 1 --no-cpu-baseline --parity-roots 0 $EXTRA" \
    bash "$R/tools/pmc.sh" "$P1" "$P2" FETCH_SIZE WRITE_SIZE || exit 1
  rm -rf "$R/gpurun_out/pmc_$c"
  mv "$R/gpurun_out/pmc" "$R/gpurun_out/pmc_$c"
  echo "pmc $c done"
done
