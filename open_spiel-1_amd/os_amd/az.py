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
[N, A], kind int32 [N] (1 = Prior wanted, 2 = Evaluate wanted, 3 = both,
0 = idle), and returns (prior float64 [N, A] action-indexed, value float64 [N]
for player 0).  Entries whose kind is 0 are ignored.  An evaluator object may
instead provide `evaluate_into(obs, legal_u8, kind, prior, value)` and write
the responses itself (e.g. its last layer's logits through `heads_into`, the
fused policy / value heads kernel), saving the mask conversion and the two
response copies per round.  Results are bit-exact with
the reference `MCTSBot(game, evaluator, uct_c, max_simulations, max_memory_mb,
solve, seed, false, child_selection_policy)` driving the same evaluator.

requests="fused" (the default) suits an evaluator that is a pure function of
(obs, legal) -- VPNetEvaluator is (vpevaluator.cc:70-98: Prior and Evaluate
are one cached inference): each leaf asks for value AND prior at once (kind
3) and the prior is kept for the node's later expansion, so a simulation costs
one evaluator round, not two (include/os_mcts.h os_az_set_requests).
requests="separate" asks exactly what the reference asks, when it asks it.
"""
import ctypes

import numpy as np

from . import _lib
from . import engine as E
from ._lib import check, lib, ptr

KIND_NONE, KIND_PRIOR, KIND_VALUE, KIND_BOTH = 0, 1, 2, 3
_REQUESTS = {"separate": _lib.AZ_REQUESTS_SEPARATE, "fused": _lib.AZ_REQUESTS_FUSED}
_LAYOUTS = {"auto": _lib.LAYOUT_AUTO, "wave": _lib.LAYOUT_WAVE, "lane": _lib.LAYOUT_LANE}


def heads_into(logits, legal, prior, value):
  """prior / value from a network's last layer on the current stream: row r of
  `logits` (f32 or bf16 [N, A + 1]) holds A policy logits then the value
  logit; prior = softmax over the legal actions (others -1e32,
  alpha_zero/model.py:278-282), value = tanh (model.py:304), f64
  (include/os_mcts.h os_az_heads_async)."""
  import torch
  n, a = prior.shape
  if logits.dtype not in (torch.float32, torch.bfloat16):
    raise ValueError("logits must be float32 or bfloat16")
  if logits.shape[0] != n or logits.shape[1] != a + 1 or logits.stride(1) != 1:
    raise ValueError("logits must be [N, A + 1] with unit column stride")
  if legal.dtype != torch.uint8 or prior.dtype != torch.float64 or value.dtype != torch.float64:
    raise ValueError("legal uint8, prior / value float64 expected")
  # the kernel indexes legal / prior as contiguous [N, A] rows and value as [N]
  if tuple(legal.shape) != (n, a) or tuple(value.shape) != (n,):
    raise ValueError("legal must be [N, A] and value [N] like prior")
  if not (legal.is_contiguous() and prior.is_contiguous() and value.is_contiguous()):
    raise ValueError("legal, prior and value must be contiguous")
  if not (logits.device == legal.device == prior.device == value.device) or not logits.is_cuda:
    raise ValueError("logits, legal, prior and value must be on the same GPU")
  st = torch.cuda.current_stream(prior.device)
  check(lib.os_az_heads_async(logits.data_ptr(), 0 if logits.dtype == torch.float32 else 1, n, a,
                              logits.stride(0), legal.data_ptr(), prior.data_ptr(),
                              value.data_ptr(), st.cuda_stream))


class MlpNetwork:
  """Weights of a one-hidden-layer policy / value network in the layout of
  os_az_mlp_heads_async, from w1 [obs_size, hidden] and w_out [hidden, A + 1]
  (the policy logits' columns, then the value's): w1t bf16 [hidden][128]
  and wout bf16 [16][hidden], zero-padded."""

  def __init__(self, w1, w_out):
    import torch
    obs_size, hidden = w1.shape
    a1 = w_out.shape[1]
    if obs_size > 128 or hidden % 32 or hidden > 256 or a1 > 16 or w_out.shape[0] != hidden:
      raise ValueError("network shape outside os_az_mlp_heads_async's bounds")
    dev = w1.device
    self.w1t = torch.zeros(hidden, 128, dtype=torch.bfloat16, device=dev)
    self.w1t[:, :obs_size] = w1.t().to(torch.bfloat16)
    self.wout = torch.zeros(16, hidden, dtype=torch.bfloat16, device=dev)
    self.wout[:a1] = w_out.t().to(torch.bfloat16)
    self.obs_size, self.hidden, self.num_actions = obs_size, hidden, a1 - 1

  def heads_into(self, obs, legal, prior, value):
    """One evaluator round fused into one kernel on the current stream:
    relu(bf16(obs) . W1) . Wout, then softmax over the legal actions / tanh
    (os_az_mlp_heads_async)."""
    import torch
    n, a = prior.shape
    if a != self.num_actions or tuple(value.shape) != (n,) or tuple(legal.shape) != (n, a):
      raise ValueError("prior [N, A], legal [N, A], value [N] expected")
    if obs.dtype != torch.float32 or obs.numel() != n * self.obs_size or not obs.is_contiguous():
      raise ValueError("obs must be contiguous float32 [N, obs_size]")
    if legal.dtype != torch.uint8 or prior.dtype != torch.float64 or value.dtype != torch.float64:
      raise ValueError("legal uint8, prior / value float64 expected")
    if not (legal.is_contiguous() and prior.is_contiguous() and value.is_contiguous()):
      raise ValueError("legal, prior and value must be contiguous")
    st = torch.cuda.current_stream(prior.device)
    check(lib.os_az_mlp_heads_async(obs.data_ptr(), n, self.obs_size, self.w1t.data_ptr(),
                                    self.hidden, self.wout.data_ptr(), a, legal.data_ptr(),
                                    prior.data_ptr(), value.data_ptr(), st.cuda_stream))


def _evaluate(evaluator, obs, legal, kind, prior, value):
  """One evaluator round: in place when the evaluator supports it."""
  into = getattr(evaluator, "evaluate_into", None)
  if into is not None:
    into(obs, legal, kind, prior, value)
  else:
    pr, v = evaluator(obs, legal.bool(), kind)
    prior.copy_(pr)
    value.copy_(v)


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
    self._layout_wave = False

  def run(self, root_actions, root_offsets, bot_seeds, evaluator, puct=True,
          max_simulations=100, uct_c=2.0, solve=True, max_memory_mb=1000,
          dirichlet_alpha=0.0, dirichlet_epsilon=0.0, stream=None, time_steps=False,
          bot_rng=None, requests="fused", graph=False, graph_batch=8, block_size=0,
          layout="auto", policy="cpp", root_noise=None, staged=False, after_prepare=None):
    """Runs every search to completion; returns the os_mcts_batch outputs.

    The evaluator may be called once more after the last step, with every
    kind 0 (idle): its answers are then ignored.  bot_rng = (keys uint32
    [R][624], pos int32 [R]): each search continues that bot rng_ (numpy
    legacy form) instead of seeding one from bot_seeds; the advanced streams
    are left in `self.bot_rng_out` (os_az_prepare_stateful / os_az_export_rng).

    dirichlet_alpha / dirichlet_epsilon are the MCTSBot constructor's
    (mcts.h:152-159): root priors become (1 - eps) * p + eps * Dir(alpha)
    noise drawn from the bot's rng before the root's shuffle (mcts.cc:265-273).
    layout: "wave" (k_waz_step, one wavefront per search), "lane" (k_az_step,
    one lane per search; the only one with GC) or "auto" (wave unless the node
    budget can be reached).  Same results.
    block_size: searches per k_az_step workgroup (one wave; 64 when 0).
    time_steps: record a HIP event pair around every k_az_step launch on the
    launch stream (`step_ms()` then sums them).

    policy="numpy": the search of python/algorithms/mcts.py (mcts.py:292-443)
    -- RandomState.shuffle of each expansion on the bot's stream (bot_rng:
    the RandomState's (key, pos)), no single-child stop, no GC.  Its root
    noise is RandomState.dirichlet, which only the caller's RandomState can
    draw: pass it as root_noise ([R][>= max_children] float64, root r's j-th
    legal action) with dirichlet_epsilon, and the stream after the draw as
    bot_rng (dirichlet_alpha stays 0; os_az_set_noise).

    staged=True: the batch was staged ahead by `stage()` (its host work done,
    possibly while the previous batch ran); the staged arguments are used
    and the ones passed here must describe the same batch.  after_prepare: a
    callable run once the batch is on the device, before its first step (e.g.
    one that stages the next batch on a worker thread).

    graph=True: after two eager rounds, one round (k_az_step + the evaluator +
    the response copies) is captured into a HIP graph and replayed
    `graph_batch` times per host check of the pending count (fused requests:
    the first check only after max_simulations + 1 rounds, the most any
    search can ask for), so the host neither launches each op nor waits on
    every round.  The evaluator must be
    capturable (static shapes, no host synchronisation); rounds replayed after
    the last search finished see only idle (kind 0) entries.  Not with
    time_steps.
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
    if policy not in ("cpp", "numpy"):
      raise ValueError("policy must be 'cpp' or 'numpy'")
    if root_noise is not None and policy != "numpy":
      raise ValueError("root_noise is for policy='numpy' (the C++ bot's noise is drawn "
                       "by the engine from dirichlet_alpha)")
    p = E.make_params(uct_c=uct_c, max_simulations=max_simulations,
                      max_memory_mb=max_memory_mb, solve=solve, block_size=block_size,
                      policy=_lib.POLICY_NUMPY if policy == "numpy" else _lib.POLICY_CPP)
    acts = _lib.i64(root_actions)
    if requests not in _REQUESTS:
      raise ValueError("requests must be 'fused' or 'separate'")
    check(lib.os_az_set_requests(self.eng._h, _REQUESTS[requests]))
    if layout not in _LAYOUTS:
      raise ValueError("layout must be 'auto', 'wave' or 'lane'")
    check(lib.os_az_set_layout(self.eng._h, _LAYOUTS[layout]))
    if staged:
      if bot_rng is not None or root_noise is not None:
        raise ValueError("staged batches are seeded C++-policy batches")
      asked = self._batch_args(R, puct, max_simulations, uct_c, solve, max_memory_mb,
                               dirichlet_alpha, dirichlet_epsilon, block_size)
      staged_args = getattr(self, "_staged_args", None)
      if staged_args is not None and staged_args != asked:
        raise ValueError("run(staged=True) must describe the batch stage() staged: staged %r, "
                         "asked %r" % (staged_args, asked))
      # os_az_prepare_staged consumes the staged batch (and refuses a second run)
      self._staged_args = None
      check(lib.os_az_prepare_staged(self.eng._h, kind.data_ptr(), obs.data_ptr(),
                                     legal.data_ptr(), prior.data_ptr(), value.data_ptr(),
                                     pending.data_ptr()))
    elif bot_rng is None:
      bs = _lib.u32(bot_seeds)
      check(lib.os_az_prepare(self.eng._h, ctypes.byref(p), 1 if puct else 0, R, ptr(acts),
                              ptr(offs), ptr(bs), float(dirichlet_alpha),
                              float(dirichlet_epsilon), kind.data_ptr(), obs.data_ptr(),
                              legal.data_ptr(), prior.data_ptr(), value.data_ptr(),
                              pending.data_ptr()))
    else:
      keys = np.ascontiguousarray(bot_rng[0], dtype=np.uint32).reshape(R, 624)
      pos = np.ascontiguousarray(bot_rng[1], dtype=np.int32).reshape(R)
      check(lib.os_az_prepare_stateful(
          self.eng._h, ctypes.byref(p), 1 if puct else 0, R, ptr(acts), ptr(offs), ptr(keys),
          ptr(pos), float(dirichlet_alpha), float(dirichlet_epsilon), kind.data_ptr(),
          obs.data_ptr(), legal.data_ptr(), prior.data_ptr(), value.data_ptr(),
          pending.data_ptr()))
    if root_noise is not None:
      rn = np.ascontiguousarray(root_noise, dtype=np.float64)
      if rn.ndim != 2 or rn.shape[0] != R or rn.shape[1] < self.eng.max_children:
        raise ValueError("root_noise must be [R][>= max_children]")
      check(lib.os_az_set_noise(self.eng._h, ptr(rn), rn.shape[1], float(dirichlet_epsilon)))
    if after_prepare is not None:
      after_prepare()
    # the kernel the engine chose (AUTO: wave unless GC can fire)
    lay = np.zeros(1, np.int32)
    check(lib.os_az_get_layout(self.eng._h, ptr(lay)))
    self._layout_wave = int(lay[0]) == _lib.LAYOUT_WAVE
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
    if graph and time_steps:
      raise ValueError("time_steps needs eager rounds (graph=False)")
    eager_rounds = 2 if graph else None
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
        _evaluate(evaluator, obs, legal, kind, prior, value)
      done.synchronize()  # step k and its count, not the evaluation behind it
      n = int(pend_host[0])
      if n == 0:
        break
      self.requests += n
      if eager_rounds is not None and self.steps >= eager_rounds:
        # Fused requests: a search asks at most once per simulation, so it is
        # done after max_simulations + 1 rounds; the first replay batch runs
        # up to there before the host looks (rounds past a search's end are
        # idle for it).
        first = graph_batch
        if requests == "fused":
          first = max(graph_batch, max_simulations + 1 - self.steps)
        self._replay(st, evaluator, kind, obs, legal, prior, value, pending, pend_host,
                     done, graph_batch, first)
        break
    o = E._alloc_outputs(R, self.eng.max_children)
    check(lib.os_az_fetch(self.eng._h, self.eng.max_children, *E._out_ptrs(o)))
    tot = np.zeros(1, np.int64)  # every step's requests, counted on the device
    check(lib.os_az_requests(self.eng._h, ptr(tot)))
    self.requests = int(tot[0])
    if bot_rng is not None:
      keys = np.zeros((R, 624), np.uint32)
      pos = np.zeros(R, np.int32)
      check(lib.os_az_export_rng(self.eng._h, ptr(keys), ptr(pos)))
      self.bot_rng_out = (keys, pos)
    return o

  def _replay(self, st, evaluator, kind, obs, legal, prior, value, pending, pend_host, done,
              batch, first=None):
    """Captures one round into a HIP graph and replays it until no search
    is pending (checked after `first` rounds, then every `batch` rounds)."""
    torch = self.torch
    g = torch.cuda.CUDAGraph()
    st.synchronize()
    with torch.cuda.graph(g):
      cs = torch.cuda.current_stream(self.device)
      check(lib.os_az_step_async(self.eng._h, cs.cuda_stream))
      _evaluate(evaluator, obs, legal, kind, prior, value)
    n = first or batch
    with torch.cuda.stream(st):
      while True:
        for _ in range(n):
          g.replay()
          self.steps += 1
        n = batch
        pend_host.copy_(pending, non_blocking=True)
        done.record(st)
        done.synchronize()
        if int(pend_host[0]) == 0:
          break
    st.synchronize()

  def stage(self, root_actions, root_offsets, bot_seeds, puct=True, max_simulations=100,
            uct_c=2.0, solve=True, max_memory_mb=1000, dirichlet_alpha=0.0,
            dirichlet_epsilon=0.0, block_size=0):
    """The host half of the next run(staged=True) (os_az_stage): roots
    replayed, root noise drawn; no device call, so it may run on another
    thread while this search's current batch runs (ctypes releases the GIL)."""
    p = E.make_params(uct_c=uct_c, max_simulations=max_simulations,
                      max_memory_mb=max_memory_mb, solve=solve, block_size=block_size)
    acts = _lib.i64(root_actions)
    offs = _lib.i64(root_offsets)
    bs = _lib.u32(bot_seeds)
    self._stage_keep = (p, acts, offs, bs)
    self._staged_args = self._batch_args(len(offs) - 1, puct, max_simulations, uct_c, solve,
                                         max_memory_mb, dirichlet_alpha, dirichlet_epsilon,
                                         block_size)
    check(lib.os_az_stage(self.eng._h, ctypes.byref(p), 1 if puct else 0, len(offs) - 1,
                          ptr(acts), ptr(offs), ptr(bs), float(dirichlet_alpha),
                          float(dirichlet_epsilon)))

  @staticmethod
  def _batch_args(R, puct, max_simulations, uct_c, solve, max_memory_mb, dirichlet_alpha,
                  dirichlet_epsilon, block_size):
    """The search arguments a staged batch fixes (stage() vs run(staged=True))."""
    return (int(R), bool(puct), int(max_simulations), float(uct_c), bool(solve),
            int(max_memory_mb), float(dirichlet_alpha), float(dirichlet_epsilon),
            int(block_size))

  def tree(self, r=0):
    """Search r's tree after run(): os_engine_tree's flat arrays plus the
    node priors (os_az_tree_priors)."""
    t = self.eng.tree(r)
    pr = np.zeros(len(t["n"]), np.float64)
    check(lib.os_az_tree_priors(self.eng._h, r, len(pr), ptr(pr)))
    t["prior"] = pr
    return t

  def eng_az_wave(self):
    """True when the last prepared batch runs k_waz_step (os_az_set_layout)."""
    return self._layout_wave

  def step_ms(self):
    """Summed k_az_step time of the last run(time_steps=True), ms."""
    return sum(a.elapsed_time(b) for a, b in self.events)


class AlphaZeroActor:
  """AlphaZero's actor games (alpha_zero.cc:64-118 PlayGame; bots as InitAZBot,
  :120-135: MCTSBot with PUCT, Dirichlet root noise and the network
  evaluator) for many games at once.

  Every move is ONE batched external-evaluator search over all unfinished
  games (`ExternalEvaluatorSearch`, one kernel step per evaluator round), each
  game's two bots continuing their own rng_ across the game; then, per game,
  the policy pow(explore_count, 1 / temperature) over the root's children,
  normalised (NormalizePolicy); the move is SampleAction(policy, actor rng)
  while fewer than `temperature_drop` moves were played (std::mt19937 per
  game, absl::Uniform(rng, 0.0, 1.0), os_sample_action), BestChild after; the
  root value total_reward / explore_count; with `resign`, the game's cutoff
  (drawn from the actor rng first: u < cutoff_probability ? cutoff_value :
  MaxUtility + 1) ends it early with returns (value, -value).  Results equal
  the reference PlayGame run with the same evaluator and seeds.
  """

  def __init__(self, game_string, device=0):
    from . import pyspiel
    self.pyspiel = pyspiel
    self.game = pyspiel.load_game(game_string)
    self.search = ExternalEvaluatorSearch(game_string, device)

  def play(self, start_actions, start_offsets, bot_seeds, actor_seeds, evaluator, max_len=None,
           uct_c=2.0, max_simulations=50, temperature=1.0, temperature_drop=10, resign=False,
           cutoff_value=0.9, cutoff_probability=0.8, dirichlet_alpha=0.0,
           dirichlet_epsilon=0.0, solve=False, max_memory_mb=10, puct=True,
           requests="fused"):
    """Plays G games; bot_seeds [G][2], actor_seeds [G].  Returns dict(actions
    [G][L] (-1 padded), length [G], returns [G][2], policy [G][L][A] (action-
    indexed), root_value [G][L])."""
    import math
    pyspiel = self.pyspiel
    offs = np.asarray(start_offsets, np.int64)
    G = len(offs) - 1
    L = int(max_len or self.game.max_game_length())
    A = self.game.num_distinct_actions()
    acts0 = np.asarray(start_actions, np.int64)
    states = []
    for g in range(G):
      st = self.game.new_initial_state()
      for a in acts0[offs[g]:offs[g + 1]]:
        st.apply_action(int(a))
      states.append(st)
    bseeds = np.asarray(bot_seeds, np.uint32).reshape(G, 2)
    keys = np.zeros((G, 2, 624), np.uint32)
    pos = np.zeros((G, 2), np.int32)
    for g in range(G):
      for p in range(2):
        k, q = pyspiel._mt_key(int(bseeds[g, p]))
        keys[g, p], pos[g, p] = k, q
    actor = []
    for s in np.asarray(actor_seeds, np.uint32):
      k, q = pyspiel._mt_key(int(s))
      actor.append((k.copy(), np.array([q], np.int32)))

    def sample(g, probs):
      pr = np.ascontiguousarray(probs, np.float64)
      k = lib.os_sample_action(pr.ctypes.data, len(pr), actor[g][0].ctypes.data,
                               actor[g][1].ctypes.data)
      if k < 0:
        check(int(k))
      return k

    cutoff = [self.game.max_utility() + 1.0] * G
    if resign:
      for g in range(G):  # SampleAction over [(u < p), (u >= p)] is the draw u < p
        if sample(g, [cutoff_probability, 1.0 - cutoff_probability]) == 0:
          cutoff[g] = cutoff_value
    out = dict(actions=np.full((G, L), -1, np.int64), length=np.zeros(G, np.int32),
               returns=np.zeros((G, 2), np.float64), policy=np.zeros((G, L, A), np.float64),
               root_value=np.zeros((G, L), np.float64))
    live = [g for g in range(G) if not states[g].is_terminal()]
    moves = [0] * G
    self.searches = 0
    while live:
      players = [states[g].current_player() for g in live]
      ra, ro = E.roots_from_histories([states[g].history() for g in live])
      rk = np.stack([keys[g, p] for g, p in zip(live, players)])
      rp = np.array([pos[g, p] for g, p in zip(live, players)], np.int32)
      o = self.search.run(ra, ro, None, evaluator, puct=puct, max_simulations=max_simulations,
                          uct_c=uct_c, solve=solve, max_memory_mb=max_memory_mb,
                          dirichlet_alpha=dirichlet_alpha,
                          dirichlet_epsilon=dirichlet_epsilon, bot_rng=(rk, rp),
                          requests=requests)
      self.searches += len(live)
      nk, npos = self.search.bot_rng_out
      still = []
      for i, (g, p) in enumerate(zip(live, players)):
        keys[g, p], pos[g, p] = nk[i], npos[i]
        m = moves[g]
        if m >= L:
          raise RuntimeError("game %d longer than max_len" % g)
        nc = int(o["nchild"][i])
        kids = [int(a) for a in o["child_action"][i, :nc]]
        pol = [math.pow(float(n), 1.0 / temperature) for n in o["child_n"][i, :nc]]
        tot = 0.0
        for x in pol:  # NormalizePolicy: left-to-right sum in child order
          tot += x
        pol = [x / tot for x in pol]
        a = kids[sample(g, pol)] if m < temperature_drop else int(o["best_action"][i])
        rv = float(o["root_w"][i]) / int(o["root_n"][i])
        out["policy"][g, m, kids] = pol
        out["root_value"][g, m] = rv
        out["actions"][g, m] = a
        states[g].apply_action(a)
        moves[g] = m + 1
        if states[g].is_terminal():
          out["returns"][g] = states[g].returns()
        elif abs(rv) > cutoff[g]:
          out["returns"][g, p], out["returns"][g, 1 - p] = rv, -rv
        else:
          still.append(g)
      live = still
    out["length"][:] = moves
    return out
