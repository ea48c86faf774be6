#!/bin/bash
# PMC passes (tools/pmc.sh) over the bench command of each named config;
# results land in gpurun_out/pmc_<config>/.  Summarise afterwards on the host
# with tools/pmc_summary.py.
#   tools/pmc_configs.sh [configs...]        (default: c2 c4)
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=${*:-c2 c4}
PMC_SUMMARY=${PMC_SUMMARY-1}  # summarise on the box (traces of many-launch configs exceed the copy-back)
P1="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD"
for c in $CFGS; do
  rm -rf "$R/gpurun_out/pmc"
  EXTRA=""
  [ "$c" = az ] && EXTRA="--az-graph 0"  # eager rounds: one traced dispatch per k_az_step
  BENCH_ARGS="--config $c --steps 2 --warmup 1 --no-cpu-baseline --parity-roots 0 --no-parity-sweep --no-configs $EXTRA" \
    bash "$R/tools/pmc.sh" "$P1" "$P2" FETCH_SIZE WRITE_SIZE || exit 1
  rm -rf "$R/gpurun_out/pmc_$c"
  mv "$R/gpurun_out/pmc" "$R/gpurun_out/pmc_$c"
  if [ -n "$PMC_SUMMARY" ]; then
    # Summarise on the box and keep only the counter CSVs (the traces of the
    # many-launch configs would exceed what gpurun copies back).
    case $c in
      c2|c3|c4) K=k_wsearch ;; c5) K=k_rollouts ;; sp) K=k_wselfplay ;;
      az) K=k_waz_step ;; g9) K=k_lsearch ;;
    esac
    case $c in
      c2|sp|az) G=connect_four ;; c3) G=breakthrough ;; c4) G=hex ;; c5|g9) G=go ;;
    esac
    python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_$c" $K $G \
      "$R/gpurun_out/pmc_rec_$c.json" > /dev/null || exit 1
    find "$R/gpurun_out/pmc_$c" -type f ! -name "run_counter_collection.csv" ! -name "*.log" -delete
    gzip -f "$R/gpurun_out/pmc_$c"/p*/run_counter_collection.csv
  fi
  echo "pmc $c done"
done
