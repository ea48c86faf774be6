#!/bin/bash
# r06 final (second pass, after the late go work), call F: rocprof kernel
# statistics and PMC passes of every config on the final sources, the PMC
# records merged (tools/pmc_merge.py), then the driver's default bench and the
# sp / az lines, which read those records.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_final.sh rocprof c2 c3 c4 c5 sp az g9 && \
bash tools/r06_final.sh pmc c2 c3 c4 c5 sp az g9 && \
python3 tools/pmc_merge.py && \
bash tools/r06_final.sh bench
