#!/usr/bin/env python3
"""C2 kernel time against the number of concurrent searches (latency vs issue).

  python tools/c2_scaling.py [game] [sims] [roots...]

For each root count R (the first R of BASELINE's C2 roots, seeds as bench.py):
kernel time (HIP events on the launch stream, median of 3), sims run, and the
per-search spread of simulations actually run.  R = 256 puts one wave on every
fourth SIMD, so its time is the slowest single search running alone; R = 4096
is the C2 workload (4 waves per SIMD).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import engine as E  # noqa: E402


def main():
  import torch
  gs = sys.argv[1] if len(sys.argv) > 1 else "connect_four"
  sims = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
  counts = [int(x) for x in sys.argv[3:]] or [64, 256, 1024, 2048, 4096, 8192]
  eng = E.Engine(gs)
  st = torch.cuda.current_stream()
  for R in counts:
    acts, offs = E.make_roots(gs, R, seed_base=1000, max_plies=8)
    bs = np.arange(R, dtype=np.uint32)
    es = bs + np.uint32(1 << 20)
    times = []
    for _ in range(3):
      eng.prepare(acts, offs, bs, es, uct_c=2.0, max_simulations=sims, solve=True)
      a = torch.cuda.Event(enable_timing=True)
      b = torch.cuda.Event(enable_timing=True)
      a.record(st)
      eng.run_async(st.cuda_stream)
      b.record(st)
      torch.cuda.synchronize()
      out = eng.fetch()
      times.append(a.elapsed_time(b))
    ms = float(np.median(times))
    n = out["root_n"].astype(np.int64)
    tot = eng.last_sims()
    print("R=%6d  %8.3f ms  %.3e sims/s  root_n min/med/max %d/%d/%d  full=%d/%d" % (
        R, ms, tot / ms * 1e3, n.min(), int(np.median(n)), n.max(),
        int((n >= sims).sum()), R), flush=True)


if __name__ == "__main__":
  main()
