#!/bin/bash
# r06 final, call B: rocprofv3 kernel statistics (+ steady-state summaries)
# and the PMC passes of every config, on the final kernel sources.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_final.sh rocprof c2 c3 c4 c5 sp az g9 && bash tools/r06_final.sh pmc c2 c3 c4 c5 sp az g9
