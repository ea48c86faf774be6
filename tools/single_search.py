#!/usr/bin/env python3
"""One warm single-root search per (game, policy) -- the launch a single bot's
step makes -- for PMC passes (tools/gpu_r05_pmc1.sh).
  python tools/single_search.py [sims] [game[:policy]] ...
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402


def main():
  sims = int(sys.argv[1])
  for spec in sys.argv[2:]:
    gs, _, pol = spec.partition(":")
    p = _lib.POLICY_NUMPY if pol == "numpy" else _lib.POLICY_CPP
    eng = E.Engine(gs)
    kw = dict(max_simulations=sims, policy=p)
    if p == _lib.POLICY_NUMPY:
      kw["max_memory_mb"] = 0
    acts, offs = np.zeros(0, np.int64), np.array([0, 0], np.int64)
    for _ in range(2):
      eng.prepare(acts, offs, [3], [7 if p == _lib.POLICY_CPP else 3], **kw)
      eng.run_async()
      eng.fetch()
    print(spec, eng.last_sims(), flush=True)
    eng.close()


if __name__ == "__main__":
  main()
