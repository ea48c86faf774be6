"""Batched MCTS with an external evaluator on the GPU.

The reference's AlphaZero actor is `MCTSBot` driving a `VPNetEvaluator`
(open_spiel/algorithms/alpha_zero/vpevaluator.cc:70-98): every expansion asks
`Prior(state)` and every leaf asks `Evaluate(state)`, each a network inference
on (LegalActions, ObservationTensor).  Here thousands of searches advance
together in one GPU kernel (csrc/os_az.h); each `step` stops every search at
its next evaluator request and leaves the requests in device tensors, so the
caller's network (e.g. a PyTorch module on the same GPU) evaluates ONE batch
in place and writes priors / values back -- no host round trip of the data.

    search = ExternalEvaluatorSearch("connect_four")
    out = search.run(root_actions, root_offsets, bot_seeds, evaluator,
                     puct=True, max_simulations=200, uct_c=1.4)

`evaluator(obs, legal, kind)` receives torch tensors on the GPU:
obs float32 [N, C, H, W] (ObservationTensor of the player to move), legal bool
[N, A], kind int32 [N] (1 = Prior wanted, 2 = Evaluate wanted, 0 = idle), and
returns (prior float64 [N, A] action-indexed, value float64 [N] for player 0).
Entries whose kind is 0 are ignored.  Results are bit-exact with the reference
`MCTSBot(game, evaluator, uct_c, max_simulations, max_memory_mb, solve, seed,
false, child_selection_policy)` driving the same evaluator.
"""
import ctypes

import numpy as np

from . import _lib
from . import engine as E
from ._lib import check, lib, ptr

KIND_NONE, KIND_PRIOR, KIND_VALUE = 0, 1, 2


class ExternalEvaluatorSearch:
  """Many independent MCTSearch calls sharing one batched external evaluator."""

  def __init__(self, game_string, device=0):
    import torch
    self.torch = torch
    self.eng = E.Engine(game_string, device)
    self.device = torch.device("cuda", device)
    self.num_actions = self.eng.num_distinct_actions
    self.obs_shape = self.eng.observation_shape
    self.steps = 0
    self.requests = 0

  def run(self, root_actions, root_offsets, bot_seeds, evaluator, puct=True,
          max_simulations=100, uct_c=2.0, solve=True, max_memory_mb=1000,
          dirichlet_alpha=0.0, dirichlet_epsilon=0.0, stream=None, time_steps=False):
    """Runs every search to completion; returns the os_mcts_batch outputs.

    dirichlet_alpha / dirichlet_epsilon are the MCTSBot constructor's
    (mcts.h:152-159): root priors become (1 - eps) * p + eps * Dir(alpha)
    noise drawn from the bot's rng before the root's shuffle (mcts.cc:265-273).
    time_steps: record a HIP event pair around every k_az_step launch on the
    launch stream (`step_ms()` then sums them).
    """
    torch = self.torch
    offs = _lib.i64(root_offsets)
    R = len(offs) - 1
    A = self.num_actions
    dev = self.device
    kind = torch.zeros(R, dtype=torch.int32, device=dev)
    obs = torch.zeros([R] + self.obs_shape, dtype=torch.float32, device=dev)
    legal = torch.zeros(R, A, dtype=torch.uint8, device=dev)
    prior = torch.zeros(R, A, dtype=torch.float64, device=dev)
    value = torch.zeros(R, dtype=torch.float64, device=dev)
    pending = torch.zeros(1, dtype=torch.int32, device=dev)
    p = E.make_params(uct_c=uct_c, max_simulations=max_simulations,
                      max_memory_mb=max_memory_mb, solve=solve)
    acts = _lib.i64(root_actions)
    bs = _lib.u32(bot_seeds)
    check(lib.os_az_prepare(self.eng._h, ctypes.byref(p), 1 if puct else 0, R, ptr(acts),
                            ptr(offs), ptr(bs), float(dirichlet_alpha),
                            float(dirichlet_epsilon), kind.data_ptr(), obs.data_ptr(),
                            legal.data_ptr(), prior.data_ptr(), value.data_ptr(),
                            pending.data_ptr()))
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    self.steps = 0
    self.requests = 0
    self.events = []
    # The evaluator of step k is queued right behind step k, before the host
    # reads step k's request count, so the host launches the network while the
    # GPU still runs the step and queues step k + 1 while the network runs.
    # When the count comes back 0 that last evaluation answered no request:
    # step k had left nothing pending, and its outputs are never read.
    pend_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    done = torch.cuda.Event()
    while True:
      if time_steps:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
      check(lib.os_az_step_async(self.eng._h, st.cuda_stream))
      if time_steps:
        e1.record(st)
        self.events.append((e0, e1))
      self.steps += 1
      with torch.cuda.stream(st):
        pend_host.copy_(pending, non_blocking=True)
        done.record(st)
        pr, v = evaluator(obs, legal.bool(), kind)
        prior.copy_(pr)
        value.copy_(v)
      done.synchronize()  # step k and its count, not the evaluation behind it
      n = int(pend_host[0])
      if n == 0:
        break
      self.requests += n
    o = E._alloc_outputs(R, self.eng.max_children)
    check(lib.os_az_fetch(self.eng._h, self.eng.max_children, *E._out_ptrs(o)))
    return o

  def step_ms(self):
    """Summed k_az_step time of the last run(time_steps=True), ms."""
    return sum(a.elapsed_time(b) for a, b in self.events)
