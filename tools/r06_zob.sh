#!/bin/bash
# r06: k_rollouts with go's Zobrist table in LDS (cur) against the table read
# through the caches (build_ab/lib_zob0.so, -DOS_ROLL_ZOB_LDS=0); C5 and its
# per-rank share, interleaved twice, then the rollout GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06/zob
bash tools/r06_ab.sh zob/c5 "--config c5" cur zob0 || exit 1
bash tools/r06_ab.sh zob/c5r "--config c5 --roots 131072 --steps 10 --warmup 3" cur zob0 || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rollout" \
  > gpurun_out/r06/zob/pytest_rollout.log 2>&1 || { tail -20 gpurun_out/r06/zob/pytest_rollout.log; exit 1; }
tail -1 gpurun_out/r06/zob/pytest_rollout.log
echo "r06_zob done"
