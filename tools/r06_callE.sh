#!/bin/bash
# r06 final, call E: the extras (C5 per-rank line, go9 wave line, the single
# bot step-latency tables) on the final sources.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_final.sh extras
