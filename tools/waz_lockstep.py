#!/usr/bin/env python3
"""Debug harness: the lane (k_az_step) and wave (k_waz_step) external-evaluator
kernels stepped in lockstep on the same roots; prints the first round whose
requests (kind / observation / legal mask) differ, per search."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
from os_amd import _lib, engine as E  # noqa: E402
from os_amd._lib import check, lib, ptr  # noqa: E402
lib.os_debug_az_arena.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                  ctypes.c_void_p, ctypes.c_void_p]
import test_az  # noqa: E402

game = sys.argv[1] if len(sys.argv) > 1 else "tic_tac_toe"
R, sims = 3, int(sys.argv[2]) if len(sys.argv) > 2 else 40
req = sys.argv[3] if len(sys.argv) > 3 else "fused"
acts, offs = E.make_roots(game, R, seed_base=5, max_plies=4)
seeds = np.arange(R, dtype=np.uint32) + 9
dev = torch.device("cuda", 0)
runs = {}
for layout in ("lane", "wave"):
  eng = E.Engine(game, 0)
  A = eng.num_distinct_actions
  t = dict(kind=torch.zeros(R, dtype=torch.int32, device=dev),
           obs=torch.zeros([R] + eng.observation_shape, dtype=torch.float32, device=dev),
           legal=torch.zeros(R, A, dtype=torch.uint8, device=dev),
           prior=torch.zeros(R, A, dtype=torch.float64, device=dev),
           value=torch.zeros(R, dtype=torch.float64, device=dev),
           pending=torch.zeros(1, dtype=torch.int32, device=dev))
  p = E.make_params(uct_c=1.25, max_simulations=sims, max_memory_mb=1000, solve=True)
  check(lib.os_az_set_requests(eng._h, 1 if req == "fused" else 0))
  check(lib.os_az_set_layout(eng._h, _lib.LAYOUT_LANE if layout == "lane" else _lib.LAYOUT_WAVE))
  bs = _lib.u32(seeds)
  check(lib.os_az_prepare(eng._h, ctypes.byref(p), 1, R, ptr(_lib.i64(acts)), ptr(_lib.i64(offs)),
                          ptr(bs), 0.0, 0.0, t["kind"].data_ptr(), t["obs"].data_ptr(),
                          t["legal"].data_ptr(), t["prior"].data_ptr(), t["value"].data_ptr(),
                          t["pending"].data_ptr()))
  runs[layout] = (eng, t)
ev = test_az._gpu_toy_evaluator(runs["lane"][0].num_distinct_actions)
for step in range(4 * sims + 10):
  out = {}
  for layout, (eng, t) in runs.items():
    check(lib.os_az_step_async(eng._h, None))
    torch.cuda.synchronize()
    out[layout] = {k: t[k].cpu().numpy().copy() for k in ("kind", "obs", "legal")}
    pr, v = ev(t["obs"], t["legal"].bool(), t["kind"])
    t["prior"].copy_(pr)
    t["value"].copy_(v)
    torch.cuda.synchronize()
  a, b = out["lane"], out["wave"]
  diff = [r for r in range(R) if not (a["kind"][r] == b["kind"][r] and
                                      np.array_equal(a["obs"][r], b["obs"][r]) and
                                      np.array_equal(a["legal"][r], b["legal"][r]))]
  if diff:
    r = diff[0]
    ND = np.dtype([("first", "<u4"), ("n", "<i4"), ("w", "<f8"), ("action", "<u2"),
                   ("nchild", "u1"), ("out", "i1"), ("pad", "<u4")])
    for layout, (eng, t) in runs.items():
      nodes = np.zeros(24, ND)
      pr = np.zeros(24, np.float64)
      check(lib.os_debug_az_arena(eng._h, r, 24, nodes.ctypes.data, pr.ctypes.data))
      print(layout, "nodes", [(int(x["first"]), int(x["n"]), float(x["w"]), int(x["action"]),
                               int(x["nchild"]), int(x["out"])) for x in nodes])
      print(layout, "prior", pr.tolist())
    print("step", step, "searches differ:", diff)
    print(" lane kind", a["kind"][r], "obs", a["obs"][r].reshape(-1).tolist()[:27])
    print(" wave kind", b["kind"][r], "obs", b["obs"][r].reshape(-1).tolist()[:27])
    break
  if a["kind"].sum() == 0 and b["kind"].sum() == 0:
    print("all done at step", step, "identical requests")
    break
else:
  print("no divergence")
