#!/usr/bin/env python3
"""Per-phase cycle breakdown of the wave search kernel.

Run with OS_AMD_LIB pointing at a -DOS_PHASE_TIMING=1 build:
  OS_AMD_LIB=build_ab/lib_phase.so python tools/phase_probe.py [roots] [sims]
Prints, per game, s_memtime cycles per simulation per wave in each phase.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402

PHASES = ("select", "expand", "rollout", "backup", "solver", "tail", "twist", "total",
          "go_legal", "go_apply", "go_insert", "go_score", "x_own", "x_opp", "x_mover", "x_rest")
GAMES = (("connect_four", 8), ("tic_tac_toe", 4), ("breakthrough", 6), ("hex", 6),
         ("go(board_size=9)", 6))


def main():
  import torch
  roots = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
  sims = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
  buf = np.zeros(len(PHASES), np.uint64)
  only = sys.argv[3] if len(sys.argv) > 3 else ""
  for gs, plies in GAMES:
    if only not in gs:
      continue
    eng = E.Engine(gs)
    acts, offs = E.make_roots(gs, roots, seed_base=1000, max_plies=plies)
    seeds = np.arange(roots, dtype=np.uint32)
    s = sims if gs in ("connect_four", "tic_tac_toe") else max(64, sims // 4)
    eng.prepare(acts, offs, seeds, seeds + np.uint32(1 << 20), max_simulations=s)
    _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))  # reset
    eng.run_async()
    torch.cuda.synchronize()
    n = _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))
    if n < 0:
      _lib.check(n)
    eng.fetch()
    total_sims = eng.last_sims()
    per = buf.astype(np.float64) / max(total_sims, 1)
    st = eng.stats()
    print("PHASE %-18s sims=%d/root  cycles/sim: %s  | scanned/sim %.1f rng/sim %.1f" % (
        gs, s, " ".join("%s=%.0f" % (p, v) for p, v in zip(PHASES, per)),
        st["scanned"] / total_sims, st["rng_words"] / total_sims), flush=True)


if __name__ == "__main__":
  main()
