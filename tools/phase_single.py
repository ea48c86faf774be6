#!/usr/bin/env python3
"""Per-phase cycles of ONE search (a single bot's step) on the wave layout.

Run with OS_AMD_LIB pointing at a -DOS_PHASE_TIMING=1 build (tools/abbuild.sh):
  OS_AMD_LIB=build_ab/lib_phase.so python tools/phase_single.py [sims]
Prints, per game and policy, s_memtime cycles per simulation in each phase
(one root from the initial position, seeds 3 / 7 as tools/step_latency.py).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402
from phase_probe import PHASES  # noqa: E402

GAMES = ("tic_tac_toe", "connect_four", "breakthrough", "hex", "go(board_size=9)")


def main():
  import torch
  sims = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
  buf = np.zeros(len(PHASES), np.uint64)
  for gs in GAMES:
    for pol, name in ((_lib.POLICY_CPP, "cpp"), (_lib.POLICY_NUMPY, "numpy")):
      eng = E.Engine(gs)
      acts, offs = np.zeros(0, np.int64), np.array([0, 0], np.int64)
      kw = dict(max_simulations=sims, policy=pol)
      if pol == _lib.POLICY_NUMPY:
        kw["max_memory_mb"] = 0
      eng.prepare(acts, offs, [3], [7 if pol == _lib.POLICY_CPP else 3], **kw)
      eng.run_async()  # warm
      eng.fetch()
      _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))  # reset
      ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      ev0.record()
      eng.run_async()
      ev1.record()
      torch.cuda.synchronize()
      n = _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))
      if n < 0:
        _lib.check(n)
      eng.fetch()
      s = max(eng.last_sims(), 1)
      per = buf.astype(np.float64) / s
      print("PHASE1 %-18s %-5s %.3f ms  cycles/sim: %s" % (
          gs, name, ev0.elapsed_time(ev1),
          " ".join("%s=%.0f" % (p, v) for p, v in zip(PHASES, per) if v)), flush=True)
      eng.close()


if __name__ == "__main__":
  main()
