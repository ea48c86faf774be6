#!/bin/bash
# r05 A/B: per-game selection re-assertion (connect_four mode 0, others 2;
# build_ab/lib_c4sel.so) against the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_ab_cfg.sh c2 20 cur c4sel || exit 1
bash tools/gpu_ab_cfg.sh sp 5 cur c4sel || exit 1
bash tools/gpu_ab_cfg.sh c4 3 cur c4sel || exit 1
