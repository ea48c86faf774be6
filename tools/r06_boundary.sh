#!/bin/bash
# r06: host-boundary (PCIe-inclusive) rates of C2 / C3 / g9 on the final
# sources (tools/boundary_rate.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06/boundary
timeout -k 10 600 python -u tools/boundary_rate.py 5 --out gpurun_out/r06/boundary/boundary_rate.json \
  > gpurun_out/r06/boundary/boundary_rate.log 2>&1 || { tail -5 gpurun_out/r06/boundary/boundary_rate.log; exit 1; }
tail -5 gpurun_out/r06/boundary/boundary_rate.log
echo "r06_boundary done"
