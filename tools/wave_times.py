#!/usr/bin/env python3
"""Per-wave start/end times of the wave search (OS_WAVE_TIMES=1 build).

  OS_AMD_LIB=diag/lib_wt.so python tools/wave_times.py [game] [roots] [sims]

Prints the distribution of wave lifetimes and end times (s_memrealtime,
100 MHz), and how waves were placed on XCDs / CUs / SIMDs.  Shows how much of
the launch is the tail (SIMDs with fewer than their share of waves left).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
from os_amd import _lib  # noqa: E402
from os_amd import engine as E  # noqa: E402

K_PHASES = 12
K_WT = 16384


def _dbg(buf):
  rc = _lib.lib.os_debug_phase_cycles(_lib.ptr(buf), len(buf))
  if rc < 0:
    _lib.check(rc)


def main():
  import torch
  gs = sys.argv[1] if len(sys.argv) > 1 else "connect_four"
  R = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
  sims = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
  buf = np.zeros(K_PHASES + 3 * K_WT, np.uint64)
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, seed_base=1000, max_plies=8)
  bs = np.arange(R, dtype=np.uint32)
  es = bs + np.uint32(1 << 20)
  for rep in range(2):
    eng.prepare(acts, offs, bs, es, uct_c=2.0, max_simulations=sims, solve=True)
    _dbg(buf)  # clear
    eng.run_async()
    torch.cuda.synchronize()
    _dbg(buf)
    out = eng.fetch()
  n = min(R, K_WT)
  wt = buf[K_PHASES:K_PHASES + 3 * n].reshape(n, 3)
  t0 = wt[:, 0].astype(np.int64)
  t1 = wt[:, 1].astype(np.int64)
  base = t0.min()
  start = (t0 - base) / 100.0  # us (100 MHz)
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
  simd_key = slot * 4 + simd
  print("%s R=%d sims=%d: launch span %.1f us" % (gs, R, sims, end.max()))
  q = [0, 10, 50, 90, 99, 100]
  print("start us  pct %s: %s" % (q, np.percentile(start, q).round(1)))
  print("end us    pct %s: %s" % (q, np.percentile(end, q).round(1)))
  print("life us   pct %s: %s" % (q, np.percentile(life, q).round(1)))
  print("mean life / span = %.3f" % (life.mean() / end.max()))
  _, per_simd = np.unique(simd_key, return_counts=True)
  _, per_cu = np.unique(slot, return_counts=True)
  print("distinct SIMDs %d, waves per SIMD hist %s" % (
      len(per_simd), np.bincount(per_simd).tolist()))
  print("distinct CUs %d, waves per CU hist %s" % (len(per_cu), np.bincount(per_cu).tolist()))
  print("waves per XCC %s" % np.bincount(xcc, minlength=8).tolist())
  # how long each SIMD's last wave ran after its own second-to-last finished
  order = np.argsort(simd_key, kind="stable")
  sk = simd_key[order]
  ends = end[order]
  tails = []
  for k in np.unique(sk):
    e = np.sort(ends[sk == k])
    if len(e) >= 2:
      tails.append(e[-1] - e[-2])
  tails = np.array(tails)
  print("per-SIMD last-wave solo tail us pct %s: %s" % (q, np.percentile(tails, q).round(1)))
  sims_run = out["root_n"].astype(np.int64)[:n]
  rate = life / np.maximum(sims_run, 1)
  print("us per sim pct %s: %s" % (q, np.percentile(rate, q).round(3)))
  plies = np.diff(np.asarray(offs, np.int64))[:n]
  for k in range(int(plies.max()) + 1):
    m = plies == k
    if m.any():
      print("  root plies %d: %4d roots, life us mean %.0f max %.0f, us/sim mean %.3f" % (
          k, m.sum(), life[m].mean(), life[m].max(), rate[m].mean()))
  os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
  np.savez(os.path.join(ROOT, "gpurun_out", "wt_%s_%d.npz" % (gs.split("(")[0], R)),
           start=start, end=end, sims=sims_run, plies=plies, hw=hw)
  slowest = np.argsort(end)[-5:]
  for i in slowest:
    print("  slow root %d: start %.1f end %.1f sims %d simd-key %d" % (
        i, start[i], end[i], sims_run[i], simd_key[i]))


if __name__ == "__main__":
  main()
