#!/bin/bash
# Round-4 final, part 1: go parity subset + g9 wave line, then every config's bench line and rocprof stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_bloomlog.sh || exit 1
bash tools/gpu_final.sh bench || exit 1
