"""Diagnostic: external-evaluator searches with the bench's random MLP --
sims per search, root outcomes, fused vs separate agreement, run-to-run
determinism.  python tools/diag_az.py [R]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from os_amd import engine as E  # noqa: E402
from os_amd.az import ExternalEvaluatorSearch  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
game = "connect_four"
acts, offs = E.make_roots(game, R, seed_base=1000, max_plies=4)
seeds = np.arange(R, dtype=np.uint32)
s = ExternalEvaluatorSearch(game)
net = bench._az_network(int(np.prod(s.obs_shape)), s.num_actions, torch, torch.device("cuda", 0))
kw = dict(puct=True, max_simulations=128, uct_c=1.25, dirichlet_alpha=1.0, dirichlet_epsilon=0.25)
outs = {}
for mode in ("separate", "fused", "fused"):
  o = s.run(acts, offs, seeds, net, requests=mode, **kw)
  st = s.eng.stats()
  rn = o["root_n"]
  print(mode, "steps", s.steps, "requests", s.requests, "sims", st["sims"],
        "root_n<128:", int((rn < 128).sum()), "root_out!=2:", int((o["root_out"] != 2).sum()),
        "nchild==1:", int((o["nchild"] == 1).sum()), "root_n hist", np.bincount(rn // 16)[:10],
        flush=True)
  if mode in outs:
    print("fused run-to-run equal:", all(np.array_equal(outs[mode][k], o[k]) for k in E.OUTPUT_KEYS))
  outs[mode] = o
bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(outs["separate"][k], outs["fused"][k])]
print("separate vs fused mismatches:", bad)
if bad:
  d = np.nonzero(outs["separate"]["root_n"] != outs["fused"]["root_n"])[0]
  print("first differing roots", d[:10], outs["separate"]["root_n"][d[:10]], outs["fused"]["root_n"][d[:10]])
