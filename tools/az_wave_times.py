#!/usr/bin/env python3
"""Residency of k_waz_step's waves in one launch (OS_WAVE_TIMES=1 build).

  OS_AMD_LIB=build_ab/lib_wt.so python tools/az_wave_times.py [roots] [sims]

The kernel records (start, end, hardware slot) of every search's wave in the
launch that runs its 21st simulation.  Prints the launch span, wave lifetimes,
and how many waves each SIMD / CU held at once (the occupancy actually reached).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
sys.path.insert(0, ROOT)
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402

K_PHASES = 12
K_WT = 16384


def max_overlap(st, en):
  ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
  ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
  return int(np.cumsum(ev[:, 1]).max())


def main():
  import torch
  import bench
  from os_amd.az import ExternalEvaluatorSearch
  R = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
  sims = int(sys.argv[2]) if len(sys.argv) > 2 else 128
  game = "connect_four"
  acts, offs = E.make_roots(game, R, seed_base=1000, max_plies=4)
  seeds = np.arange(R, dtype=np.uint32)
  search = ExternalEvaluatorSearch(game)
  net = bench._az_network(int(np.prod(search.obs_shape)), search.num_actions, torch,
                          torch.device("cuda:0"))
  kw = dict(puct=True, max_simulations=sims, uct_c=1.25, dirichlet_alpha=1.0,
            dirichlet_epsilon=0.25, layout="wave")
  search.run(acts, offs, seeds, net, **kw)
  buf = np.zeros(K_PHASES + 3 * K_WT, np.uint64)
  torch.cuda.synchronize()
  _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))  # clear
  search.run(acts, offs, seeds, net, time_steps=True, **kw)
  torch.cuda.synchronize()
  _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))
  n = min(R, K_WT)
  wt = buf[K_PHASES:K_PHASES + 3 * n].reshape(n, 3)
  ok = wt[:, 0] != 0
  wt = wt[ok]
  t0 = wt[:, 0].astype(np.int64)
  t1 = wt[:, 1].astype(np.int64)
  base = t0.min()
  start = (t0 - base) / 100.0
  end = (t1 - base) / 100.0
  life = end - start
  hw = wt[:, 2].astype(np.uint64)
  hwid = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
  xcc = ((hw >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64)
  simd = (hwid >> 4) & 3
  cu = (hwid >> 8) & 15
  sh = (hwid >> 12) & 1
  se = (hwid >> 13) & 7
  slot = ((xcc * 8 + se) * 2 + sh) * 16 + cu
  key = slot * 4 + simd
  q = [0, 10, 50, 90, 100]
  print("AZWT waves recorded %d of %d; launch span %.1f us; kernel ms/launch %.4f" % (
      ok.sum(), R, end.max(), search.step_ms() / max(search.steps, 1)))
  print("AZWT start us pct %s: %s" % (q, np.percentile(start, q).round(1)))
  print("AZWT life us  pct %s: %s" % (q, np.percentile(life, q).round(1)))
  occ_simd = [max_overlap(start[key == k], end[key == k]) for k in np.unique(key)]
  occ_cu = [max_overlap(start[slot == k], end[slot == k]) for k in np.unique(slot)]
  print("AZWT distinct SIMDs %d CUs %d; max resident waves per SIMD hist %s; per CU hist %s" % (
      len(occ_simd), len(occ_cu), np.bincount(occ_simd).tolist(), np.bincount(occ_cu).tolist()))


if __name__ == "__main__":
  main()
