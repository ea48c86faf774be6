"""TEST INFRASTRUCTURE ONLY: an `os_amd.engine.Engine` stand-in for the CPU
rehearsal of bench.py's multi-rank plumbing (`bench.py --rehearse-host`).

It runs the product search headers compiled for the host (tests/hostcheck) so
that bench.py's rank spawn, per-rank root/seed assignment and the gloo
all-reduces in bench_root_parallel / bench_playouts execute in the CPU suite.
It is never a measurement: bench.py labels every rehearsal line as such.
"""
import ctypes

import numpy as np

import hostcheck_lib as hc
import oracle_lib


class HostEngine:
  """The subset of Engine that bench.py's search / root-parallel / playout
  legs call; device addresses are host addresses of CPU torch tensors."""

  def __init__(self, game_string, device=0):
    self.game_string = game_string
    og = oracle_lib.Game(game_string)
    self.num_distinct_actions = og.num_distinct_actions
    self.max_children = og.num_distinct_actions
    self._out = None
    self._roll = None

  # ---- independent searches / root-parallel trees ----
  def prepare(self, root_actions, root_offsets, bot_seeds, eval_seeds=None, **params):
    keep = ("uct_c", "max_simulations", "n_rollouts", "max_memory_mb", "solve")
    self._prep = (np.asarray(root_actions, np.int64), np.asarray(root_offsets, np.int64),
                  np.asarray(bot_seeds, np.uint32),
                  np.asarray(eval_seeds if eval_seeds is not None else bot_seeds, np.uint32),
                  {k: v for k, v in params.items() if k in keep})

  def run_async(self, stream=None):
    acts, offs, bs, es, p = self._prep
    self._out = hc.mcts_batch(self.game_string, acts, offs, bs, es, self.max_children, **p)

  def fetch(self):
    return self._out

  def last_sims(self):
    return int(self._out["root_n"].sum())

  def stats(self):
    return None

  def set_arena_mode(self, mode):
    assert mode in ("paged", "reserved")

  def arena_info(self):
    return {"paged": 0, "reruns": 0}  # no device arena on the host

  def algorithmic_bytes(self, num_roots):
    return 0

  def root_sums_async(self, num_actions, visits_ptr, rewards_ptr, stream=None):
    o = self._out
    v = np.zeros(num_actions, np.int64)
    w = np.zeros(num_actions, np.float64)
    for r in range(len(o["nchild"])):
      k = int(o["nchild"][r])
      np.add.at(v, o["child_action"][r, :k], o["child_n"][r, :k])
      np.add.at(w, o["child_action"][r, :k], o["child_w"][r, :k])
    ctypes.memmove(visits_ptr, v.ctypes.data, v.nbytes)
    ctypes.memmove(rewards_ptr, w.ctypes.data, w.nbytes)

  # ---- playouts ----
  def rollouts_prepare(self, history, seeds, n_rollouts=1, layout=None):
    assert n_rollouts == 1
    self._roll = (np.asarray(history, np.int64), np.asarray(seeds, np.uint32))

  def rollouts_run_async(self, stream=None):
    self._returns = hc.rollouts(self.game_string, *self._roll)

  def rollouts_fetch(self):
    return self._returns

  def rollouts_outcomes_async(self, counts_ptr, stream=None):
    r = self._returns[:, 0]
    c = np.array([(r > 0).sum(), (r < 0).sum(), (r == 0).sum()], np.int64)
    ctypes.memmove(counts_ptr, c.ctypes.data, c.nbytes)
