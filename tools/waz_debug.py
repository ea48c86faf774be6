#!/usr/bin/env python3
"""k_waz_step debug run (bounds-checked build, OS_WAZ_CHECK=1): one small
external-evaluator search batch per case on the wave layout, compared with the
oracle.  A failed check ends its search with status 100 + site (no access out
of range), reported by the fetch."""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import oracle_lib  # noqa: E402
from os_amd import engine as E  # noqa: E402
from os_amd.az import ExternalEvaluatorSearch  # noqa: E402
import test_az  # noqa: E402

CASES = [("connect_four", 80, 20, True, "fused", (1.0, 0.25)),
         ("connect_four", 3, 40, True, "separate", (0.0, 0.0)),
         ("tic_tac_toe", 3, 40, False, "fused", (0.0, 0.0)),
         ("breakthrough(rows=6,columns=6)", 3, 30, True, "fused", (0.0, 0.0))]
which = sys.argv[1:] or [str(i) for i in range(len(CASES))]
for i in map(int, which):
  game, R, sims, puct, req, (alpha, eps) = CASES[i]
  acts, offs = E.make_roots(game, R, seed_base=5, max_plies=4)
  seeds = np.arange(R, dtype=np.uint32) + 9
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  kw = dict(puct=puct, uct_c=1.25, max_simulations=sims, dirichlet_alpha=alpha,
            dirichlet_epsilon=eps)
  ref = og.mcts_external(acts, offs, seeds, test_az._oracle_eval_fn(game), max_children=A, **kw)
  search = ExternalEvaluatorSearch(game)
  try:
    got = search.run(acts, offs, seeds, test_az._gpu_toy_evaluator(A), requests=req,
                     layout="wave", **kw)
    torch.cuda.synchronize()
  except Exception as e:  # a failed check is reported here
    print("case", i, game, "ERROR", e, flush=True)
    continue
  mc = search.eng.max_children
  bad = {}
  for k in E.OUTPUT_KEYS:
    r = ref[k][:, :mc] if ref[k].ndim == 2 else ref[k]
    rows = np.nonzero((got[k] != r).reshape(R, -1).any(axis=1))[0]
    if len(rows):
      bad[k] = rows[:8].tolist()
  print("case", i, game, "steps", search.steps, "bad", bad, flush=True)
  if bad:
    r0 = min(min(v) for v in bad.values())
    for k in E.OUTPUT_KEYS:
      print("  ", k, "got", np.asarray(got[k][r0]).tolist()[:10], "ref",
            np.asarray(ref[k][r0]).tolist()[:10])
