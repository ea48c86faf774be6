#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_waz_step (one wave per search).

Run with OS_AMD_LIB pointing at a -DOS_PHASE_TIMING=1 build:
  OS_AMD_LIB=build_ab/lib_phase.so python tools/az_phase_probe.py [roots] [sims] [layout]
Prints s_memtime cycles per wave-launch in each phase of the kernel
(prologue, descent, expansion, backup, request writes), over one search batch
with bench.py's random-init evaluator.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
sys.path.insert(0, ROOT)
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402

NAMES = {"select": "descent", "expand": "expand", "rollout": "prologue", "backup": "backup",
         "tail": "writes", "total": "total"}
PHASES = ("select", "expand", "rollout", "backup", "solver", "tail", "twist", "total",
          "go_legal", "go_apply", "go_insert", "go_score")


def main():
  import torch
  import bench
  from os_amd.az import ExternalEvaluatorSearch
  roots = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
  sims = int(sys.argv[2]) if len(sys.argv) > 2 else 128
  layout = sys.argv[3] if len(sys.argv) > 3 else "wave"
  game = sys.argv[4] if len(sys.argv) > 4 else "connect_four"
  acts, offs = E.make_roots(game, roots, seed_base=1000, max_plies=4)
  seeds = np.arange(roots, dtype=np.uint32)
  search = ExternalEvaluatorSearch(game)
  obs = int(np.prod(search.obs_shape))
  net = bench._az_network(obs, search.num_actions, torch, torch.device("cuda:0"))
  kw = dict(puct=True, max_simulations=sims, uct_c=1.25, dirichlet_alpha=1.0,
            dirichlet_epsilon=0.25, layout=layout)
  search.run(acts, offs, seeds, net, **kw)  # warm
  buf = np.zeros(len(PHASES), np.uint64)
  torch.cuda.synchronize()
  _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))  # reset
  search.run(acts, offs, seeds, net, time_steps=True, **kw)
  torch.cuda.synchronize()
  n = _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))
  if n < 0:
    _lib.check(n)
  waves = search.steps * ((roots + 63) // 64)  # the kernel samples one search in 64
  per = buf.astype(np.float64) / max(waves, 1)
  print("AZPHASE %s %s roots=%d sims=%d launches=%d kernel_ms/launch=%.4f  cycles/wave-launch: %s" % (
      game, layout, roots, sims, search.steps, search.step_ms() / max(search.steps, 1),
      " ".join("%s=%.0f" % (NAMES[p], v) for p, v in zip(PHASES, per) if p in NAMES)),
      flush=True)


if __name__ == "__main__":
  main()
