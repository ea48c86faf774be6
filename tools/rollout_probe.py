#!/usr/bin/env python3
"""Layout probe: playouts/s (rollout kernels) and sims/s (search kernels) per
game and per kernel layout (wave-per-search vs lane-per-search)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402

GAMES = ("tic_tac_toe", "connect_four", "breakthrough", "hex", "go(board_size=9)")
LAYOUTS = (("wave", _lib.LAYOUT_WAVE), ("lane", _lib.LAYOUT_LANE))


def probe_rollouts(n):
  for gs in GAMES:
    eng = E.Engine(gs)
    seeds = np.arange(n, dtype=np.uint32)
    for name, lay in LAYOUTS:
      eng.rollouts([], seeds[:1024], layout=lay)
      t0 = time.perf_counter()
      out = eng.rollouts([], seeds, layout=lay)
      dt = time.perf_counter() - t0
      print("ROLLOUT %-18s %-4s n=%d %8.3f ms  %.3e playouts/s  mean_r0=%.4f" %
            (gs, name, n, dt * 1e3, n / dt, out[:, 0].mean()), flush=True)


def probe_search(roots, sims):
  import torch
  for gs in GAMES:
    eng = E.Engine(gs)
    acts, offs = E.make_roots(gs, roots, seed_base=1, max_plies=6)
    seeds = np.arange(roots, dtype=np.uint32) + 7
    for name, lay in LAYOUTS:
      try:
        eng.prepare(acts, offs, seeds, seeds + 100000, max_simulations=sims,
                    layout=lay)
        eng.run_async()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run_async()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        eng.fetch()
        s = eng.last_sims()
        print("SEARCH  %-18s %-4s roots=%d sims=%d %8.3f ms  %.3e sims/s" %
              (gs, name, roots, sims, dt * 1e3, s / dt), flush=True)
      except Exception as e:  # report and keep probing the other cases
        print("SEARCH  %-18s %-4s FAILED %s" % (gs, name, e), flush=True)


def main():
  n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
  probe_rollouts(n)
  probe_search(int(sys.argv[2]) if len(sys.argv) > 2 else 4096,
               int(sys.argv[3]) if len(sys.argv) > 3 else 256)


if __name__ == "__main__":
  main()
