#!/usr/bin/env python3
"""Quick GPU parity + timing probe (development tool, run via gpurun)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_lib as O  # noqa: E402
from os_amd import engine as E  # noqa: E402


def cmp(a, b):
  return [k for k in E.OUTPUT_KEYS if not np.array_equal(a[k], b[k])]


def main():
  cases = [("tic_tac_toe", 32, 1000, 4), ("connect_four", 64, 1024, 8),
           ("breakthrough", 16, 300, 6), ("hex(board_size=5)", 16, 300, 6),
           ("hex", 8, 300, 4), ("go(board_size=7,komi=4.5)", 8, 200, 6),
           ("go(board_size=9)", 8, 128, 6)]
  for gs, R, sims, plies in cases:
    eng = E.Engine(gs)
    acts, offs = E.make_roots(gs, R, 1000, plies)
    bs = np.arange(R, dtype=np.uint32)
    es = bs + (1 << 20)
    t0 = time.time()
    og = eng.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims)
    t1 = time.time()
    ref = O.Game(gs).mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                                max_children=eng.max_children)
    bad = cmp(og, ref)
    print("PARITY", gs, R, sims, "OK" if not bad else "MISMATCH %s" % bad,
          "gpu_s=%.3f" % (t1 - t0), flush=True)
    if bad:
      for r in range(R):
        if not all(np.array_equal(og[k][r], ref[k][r]) for k in E.OUTPUT_KEYS):
          print("  first bad root", r, "gpu", og["child_n"][r][:og["nchild"][r]],
                "ref", ref["child_n"][r][:ref["nchild"][r]], flush=True)
          break
  # timing at the C2 config
  gs = "connect_four"
  eng = E.Engine(gs)
  R = 4096
  acts, offs = E.make_roots(gs, R, 1000, 8)
  bs = np.arange(R, dtype=np.uint32)
  es = bs + (1 << 20)
  for block in (64, 32, 16, 8):
    eng.prepare(acts, offs, bs, es, uct_c=2.0, max_simulations=1024,
                block_size=block)
    eng.run_async()
    o = eng.fetch()
    t0 = time.time()
    eng.run_async()
    o = eng.fetch()
    t1 = time.time()
    sims = eng.last_sims()
    print("TIMING c4 R=%d block=%d sims=%d wall=%.4fs sims/s=%.3e" %
          (R, block, sims, t1 - t0, sims / (t1 - t0)), flush=True)
  # spot parity of the full-size run on 64 roots
  sub = 64
  ref = O.Game(gs).mcts_batch(acts[:offs[sub]], offs[:sub + 1], bs[:sub], es[:sub],
                              uct_c=2.0, max_simulations=1024, max_children=7)
  bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(o[k][:sub], ref[k])]
  print("PARITY c4 full-run first 64 roots:", "OK" if not bad else bad, flush=True)


if __name__ == "__main__":
  main()
