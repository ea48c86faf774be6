#!/bin/bash
# r06 final (second pass), call G: the full -m gpu suite and smoke, every
# config's full-size parity against the oracle, and the extras (C5 per-rank
# line, 4096-root go9 wave line, single-bot and AZ step latency).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r06_final.sh tests && bash tools/r06_final.sh parity && bash tools/r06_final.sh extras
