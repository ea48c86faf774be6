#!/bin/bash
# r06 final, call A: tests + smoke, the driver's bench command + sp / az
# lines, extras (C5 per-rank, go9 wave, step latency tables).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_final.sh tests && bash tools/r06_final.sh bench && bash tools/r06_final.sh extras
