#!/usr/bin/env python3
"""Rollout-kernel probe: playouts/s per game from the initial position."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import engine as E  # noqa: E402


def main():
  n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
  for gs in ("connect_four", "breakthrough", "hex", "go(board_size=9)"):
    eng = E.Engine(gs)
    seeds = np.arange(n, dtype=np.uint32)
    eng.rollouts([], seeds[:1024])
    t0 = time.perf_counter()
    out = eng.rollouts([], seeds)
    dt = time.perf_counter() - t0
    print("ROLLOUT %-18s n=%d %.3f ms  %.3e playouts/s  mean_r0=%.3f" %
          (gs, n, dt * 1e3, n / dt, out[:, 0].mean()), flush=True)


if __name__ == "__main__":
  main()
