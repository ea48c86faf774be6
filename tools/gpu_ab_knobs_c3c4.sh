#!/bin/bash
# r05 knob sweep on breakthrough (C3) and hex (C4): which per-game uniformity
# re-assertions pay outside connect_four.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_ab_cfg.sh c3 2 cur uroll0 uroll1 umt1 usel0 || exit 1
bash tools/gpu_ab_cfg.sh c4 3 cur uroll0 uroll1 umt1 usel0 || exit 1
