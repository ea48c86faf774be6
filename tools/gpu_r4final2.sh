#!/bin/bash
# Round-4 final, part 2: go parity subset + g9 wave line, then the PMC passes of every config.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_bloomlog.sh || exit 1
bash tools/gpu_final.sh pmc c2 c3 c4 c5 sp az g9 || exit 1
