#!/usr/bin/env python3
"""pig: lane (k_mcts) vs wave (k_wsearch_chance) layout, device time of one
search batch of R roots x 1000 sims (HIP events on the launch stream)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402


def main():
  import torch
  gs = sys.argv[1] if len(sys.argv) > 1 else "pig"
  for R in (1, 64, 1024):
    for name, lay in (("lane", _lib.LAYOUT_LANE), ("wave", _lib.LAYOUT_WAVE)):
      eng = E.Engine(gs)
      acts, offs = E.make_roots(gs, R, seed_base=7, max_plies=0)
      seeds = np.arange(R, dtype=np.uint32) + 3
      eng.prepare(acts, offs, seeds, seeds + np.uint32(7), uct_c=2.0, max_simulations=1000,
                  layout=lay)
      st = torch.cuda.current_stream()
      ts = []
      for _ in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        eng.run_async(st.cuda_stream)
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
      out = eng.fetch()
      print("PIG %s R=%d %s: %.2f ms (sims %d)" % (gs, R, name, float(np.median(ts[1:])),
                                                  eng.last_sims()), flush=True)


if __name__ == "__main__":
  main()
