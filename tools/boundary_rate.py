#!/usr/bin/env python3
"""Host-boundary (PCIe-inclusive) rate of the search configs: the C-ABI call
a caller makes with HOST buffers, `os_mcts_batch` (root histories, seeds in;
children / root statistics out), timed end to end -- root replay on the host,
uploads, the search, downloads -- against the kernel alone.  The bench's
`value` is the kernel-resident rate (inputs already in HBM); this is the
figure DESIGN.md §5 quotes beside it.

  python tools/boundary_rate.py [reps] [--out gpurun_out/boundary_rate.json]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))

import bench  # noqa: E402
from os_amd import engine as E  # noqa: E402


def main():
  import torch
  reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5
  out_path = os.path.join(ROOT, "gpurun_out", "boundary_rate.json")
  if "--out" in sys.argv:
    out_path = sys.argv[sys.argv.index("--out") + 1]
  res = {}
  for cfg in ("c2", "c3", "g9"):
    _, game, R, sims, plies = bench.CONFIGS[cfg]
    acts, offs = E.make_roots(game, R, seed_base=1000, max_plies=plies)
    gid = np.arange(R, dtype=np.uint32)
    bot, ev = gid, gid + np.uint32(bench.EVAL_OFFSET)
    eng = E.Engine(game)
    kw = dict(uct_c=2.0, max_simulations=sims, n_rollouts=1, max_memory_mb=1000, solve=True)
    eng.mcts_batch(acts, offs, bot, ev, **kw)  # warm (arena sized, code loaded)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
      t0 = time.perf_counter()
      eng.mcts_batch(acts, offs, bot, ev, **kw)  # host in, host out
      times.append(time.perf_counter() - t0)
    # the kernel alone: prepared batch, timed on the device
    eng.prepare(acts, offs, bot, ev, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kms = []
    for _ in range(reps):
      e0.record()
      eng.run_async(torch.cuda.current_stream().cuda_stream)
      e1.record()
      e1.synchronize()
      kms.append(e0.elapsed_time(e1))
    eng.fetch()
    sims_run = eng.last_sims()
    call_s = float(np.median(times))
    kern_s = float(np.median(kms)) / 1e3
    res[cfg] = {"game": game, "roots": R, "sims_per_root": sims, "sims_run": sims_run,
                "call_ms": call_s * 1e3, "kernel_ms": kern_s * 1e3,
                "boundary_sims_per_s": sims_run / call_s, "kernel_sims_per_s": sims_run / kern_s,
                "boundary_over_kernel": kern_s / call_s, "reps": reps,
                "input_bytes": int(acts.nbytes + offs.nbytes + bot.nbytes + ev.nbytes)}
    print(cfg, json.dumps(res[cfg]), flush=True)
    eng.close()
  os.makedirs(os.path.dirname(out_path), exist_ok=True)
  with open(out_path, "w") as f:
    json.dump(res, f, indent=1)


if __name__ == "__main__":
  main()
