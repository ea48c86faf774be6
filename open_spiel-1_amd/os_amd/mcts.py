"""Drop-in for open_spiel/python/algorithms/mcts.py, GPU-backed.

Public names and signatures follow the reference module (Evaluator :29-43,
RandomRolloutEvaluator :46-82, SearchNode :85-196, MCTSBot :199-443).

`MCTSBot.mcts_search` runs on the MI355X whenever the search is one the
engine implements, continuing the bot's (and the evaluator's)
`np.random.RandomState` streams in place, bit-exact with the reference module:
- a `RandomRolloutEvaluator` (one shared RandomState, as in
  mcts_test.py:41-54, or two), UCT or PUCT child selection
  (`SearchNode.uct_value` / `SearchNode.puct_value`), no Dirichlet noise, one
  of the supported games (the five, and pig with its chance nodes);
- an evaluator with a batched protocol -- `evaluate_into`, or
  `evaluate_batch(obs, legal, kind) -> (prior, value)` such as this package's
  `AlphaZeroEvaluator` -- on a deterministic two-player game: the AlphaZero
  bot of alpha_zero.py:185-192 (PUCT, Dirichlet root noise, solve=False).
  The search runs in the external-evaluator kernel (os_amd/az.py), one
  evaluator round per simulation; the root noise is drawn with the bot's own
  `RandomState.dirichlet` where mcts.py:314-316 draws it (the first use of the
  stream in a search whose evaluator draws nothing), and mixed on the device.
Searches the engine does not implement (other evaluators, a custom
`child_selection_fn`, hex / go boards above 11 x 11) run the generic host
loop below with a RuntimeWarning under `backend="auto"`; pass `backend="hip"`
to forbid that and fail loudly instead, or `backend="host"` to choose it.
"""
import math
import time
import warnings

import numpy as np

from . import _lib
from . import pyspiel


class Float32ModelError(TypeError):
  """An evaluator's model answered in a dtype other than float64: the device
  search, which computes in float64, refuses it (az_evaluator.py)."""


class Evaluator(object):
  """Evaluation function interface (mcts.py:29-43)."""

  def evaluate(self, state):
    raise NotImplementedError

  def prior(self, state):
    raise NotImplementedError


class RandomRolloutEvaluator(Evaluator):
  """Average outcome of n_rollouts uniformly random playouts (mcts.py:46-82).

  On the GPU path its RandomState is advanced by the kernel; `evaluate` is
  also available on the host for direct calls.
  """

  def __init__(self, n_rollouts=1, random_state=None):
    self.n_rollouts = n_rollouts
    self._random_state = random_state or np.random.RandomState()

  def evaluate(self, state):
    total = None
    for _ in range(self.n_rollouts):
      playout = state.clone()
      while not playout.is_terminal():
        if playout.is_chance_node():
          acts, probs = zip(*playout.chance_outcomes())
          playout.apply_action(self._random_state.choice(acts, p=probs))
        else:
          playout.apply_action(self._random_state.choice(playout.legal_actions()))
      r = np.array(playout.returns())
      total = r if total is None else total + r
    return total / self.n_rollouts

  def prior(self, state):
    if state.is_chance_node():
      return state.chance_outcomes()
    legal = state.legal_actions(state.current_player())
    p = 1.0 / len(legal)
    return [(a, p) for a in legal]


class SearchNode(object):
  """Search tree node (mcts.py:85-196; C++ mcts.h:109-137)."""

  __slots__ = ["action", "player", "prior", "explore_count", "total_reward",
               "outcome", "children"]

  def __init__(self, action, player, prior):
    self.action = action
    self.player = player
    self.prior = prior
    self.explore_count = 0
    self.total_reward = 0.0
    self.outcome = None
    self.children = []

  def uct_value(self, parent_explore_count, uct_c):
    """UCT (mcts.py:124-133 / mcts.cc:89-100)."""
    if self.outcome is not None:
      return self.outcome[self.player]
    if self.explore_count == 0:
      return float("inf")
    n = self.explore_count
    return self.total_reward / n + uct_c * math.sqrt(
        math.log(parent_explore_count) / n)

  def puct_value(self, parent_explore_count, uct_c):
    """PUCT (mcts.py:135-142 / mcts.cc:102-111)."""
    if self.outcome is not None:
      return self.outcome[self.player]
    q = self.total_reward / self.explore_count if self.explore_count else 0
    return q + uct_c * self.prior * math.sqrt(parent_explore_count) / (
        self.explore_count + 1)

  def sort_key(self):
    """Proven value, then visits, then reward (mcts.py:144-158)."""
    proven = 0 if self.outcome is None else self.outcome[self.player]
    return (proven, self.explore_count, self.total_reward)

  def best_child(self):
    return max(self.children, key=SearchNode.sort_key)

  def children_str(self, state=None):
    ordered = sorted(self.children, key=SearchNode.sort_key)
    return "\n".join(c.to_str(state) for c in reversed(ordered))

  def to_str(self, state=None):
    if state is not None and self.action is not None:
      name = state.action_to_string(state.current_player(), self.action)
    else:
      name = str(self.action)
    mean = self.explore_count and self.total_reward / self.explore_count
    solved = ("{:4.1f}".format(self.outcome[self.player])
              if self.outcome else "none")
    return ("{:>6}: player: {}, prior: {:5.3f}, value: {:6.3f}, sims: {:5d}, "
            "outcome: {}, {:3d} children").format(
                name, self.player, self.prior, mean, self.explore_count, solved,
                len(self.children))

  def __str__(self):
    return self.to_str(None)


def _outcome_vector(code, nplayers):
  """Returns() of a solved node from the engine's outcome code (os_games.h):
  the player-0 value v of a two-player game ([v, -v]); with more players
  (pig) 3 + w for a win by w (1 for w, -1 / (n - 1) for the others,
  pig.cc:94-111) and 0 for nobody (all 0)."""
  if nplayers == 2:
    return [float(code), float(-code)]
  if code >= 3:
    return [1.0 if p == code - 3 else -1.0 / (nplayers - 1) for p in range(nplayers)]
  return [0.0] * nplayers


class _TreeView(object):
  """The engine's flat arena of one search (os_engine_tree) plus what node
  construction needs; shared by every lazy node of that tree."""
  __slots__ = ("first", "n", "w", "action", "nchild", "out0", "p0", "chance", "nplayers",
               "prior")

  def __init__(self, flat, state, game):
    self.first, self.n, self.w = flat["first"], flat["n"], flat["w"]
    self.prior = flat.get("prior")  # external-evaluator trees: the node priors
    self.action, self.nchild, self.out0 = flat["action"], flat["nchild"], flat["out0"]
    self.p0 = state.current_player()
    self.chance = (game.get_type().chance_mode !=
                   pyspiel.GameType.ChanceMode.DETERMINISTIC)
    self.nplayers = game.num_players()


class _LazySearchNode(SearchNode):
  """A SearchNode whose `children` are built from the flat arena on first
  access, so a caller that reads only the root (or `best_child()`) does not
  pay for the whole tree (thousands of nodes per search)."""
  __slots__ = ("_view", "_idx", "_depth", "_state", "_parent_state", "_kids")

  def __init__(self, view, idx, depth, action, player, prior, parent_state=None,
               state=None):
    # SearchNode.__init__ is not called: `children` is the lazy property below.
    self.action, self.player, self.prior = action, player, prior
    self._view, self._idx, self._depth = view, idx, depth
    self._state, self._parent_state, self._kids = state, parent_state, None
    self.explore_count = int(view.n[idx])
    self.total_reward = float(view.w[idx])
    o = int(view.out0[idx])
    self.outcome = None if o == 2 else _outcome_vector(o, view.nplayers)

  def _node_state(self):
    if self._state is None:
      self._state = self._parent_state.child(self.action)
    return self._state

  @property
  def children(self):
    if self._kids is None:
      v, idx = self._view, self._idx
      nc = int(v.nchild[idx])
      base = int(v.first[idx])
      kids = []
      if nc:
        acts = v.action[base:base + nc].tolist()
        if v.chance:
          st = self._node_state()
          child_player = st.current_player()
          probs = dict(st.chance_outcomes()) if st.is_chance_node() else {}
          kids = [_LazySearchNode(v, base + k, self._depth + 1, a, child_player,
                                  probs.get(a, 1.0 / nc), parent_state=st)
                  for k, a in enumerate(acts)]
        else:
          child_player = v.p0 ^ (self._depth & 1)
          kids = [_LazySearchNode(v, base + k, self._depth + 1, a, child_player,
                                  1.0 / nc if v.prior is None else float(v.prior[base + k]))
                  for k, a in enumerate(acts)]
      self._kids = kids
    return self._kids

  @children.setter
  def children(self, value):
    self._kids = value


def tree_to_search_nodes(flat, state, game, root_action=None):
  """The engine's flat arena (os_engine_tree) as a SearchNode tree.

  Nodes are materialised lazily, level by level as `children` is read.  Node
  players follow from depth where turns alternate; in games with chance nodes
  (pig) they are read off the replayed states (a chance node's children have
  player PlayerId.CHANCE and the outcome probabilities as priors).  Other
  priors are the uniform 1/|legal| of RandomRolloutEvaluator.prior; outcomes
  are [v, -v] vectors as the reference stores Returns().
  """
  view = _TreeView(flat, state, game)
  return _LazySearchNode(view, 0, 0, root_action, view.p0, 1,
                         state=state if view.chance else None)


class MCTSBot(pyspiel.Bot):
  """MCTS bot (mcts.py:199-443) whose hot path runs on the MI355X."""

  def __init__(self, game, uct_c, max_simulations, evaluator, solve=True,
               random_state=None, child_selection_fn=SearchNode.uct_value,
               dirichlet_noise=None, verbose=False, backend="auto"):
    pyspiel.Bot.__init__(self)
    gt = game.get_type()
    if gt.reward_model != pyspiel.GameType.RewardModel.TERMINAL:
      raise ValueError("Game must have terminal rewards.")
    if gt.dynamics != pyspiel.GameType.Dynamics.SEQUENTIAL:
      raise ValueError("Game must have sequential turns.")
    if backend not in ("auto", "hip", "host"):
      raise ValueError("backend must be 'auto', 'hip' or 'host'")
    self._game = game
    self.uct_c = uct_c
    self.max_simulations = max_simulations
    self.evaluator = evaluator
    self.verbose = verbose
    self.solve = solve
    self.max_utility = game.max_utility()
    self._dirichlet_noise = dirichlet_noise
    self._random_state = random_state or np.random.RandomState()
    self._child_selection_fn = child_selection_fn
    self.backend = backend
    if backend == "hip" and not self._gpu_eligible():
      raise ValueError("backend='hip' needs UCT or PUCT child selection, a supported game "
                       "and either RandomRolloutEvaluator without Dirichlet noise or an "
                       "evaluator with a batched protocol (evaluate_into / evaluate_batch)")
    self._warned_host = False

  def _gpu_eligible(self):
    return self._rollout_eligible() or self._external_eligible()

  def _rollout_eligible(self):
    return (type(self.evaluator) is RandomRolloutEvaluator and
            self._child_selection_fn in (SearchNode.uct_value, SearchNode.puct_value) and
            not self._dirichlet_noise and
            isinstance(self._game, pyspiel.Game) and self._game.on_device(numpy_policy=True))

  def _device_evaluator(self):
    """The batched form of the evaluator the external-evaluator kernel drives
    (os_amd/az.py protocol), or None."""
    ev = self.evaluator
    if type(ev) is RandomRolloutEvaluator:
      return None
    if getattr(ev, "evaluate_into", None) is not None:
      return ev
    return getattr(ev, "evaluate_batch", None)

  def _external_eligible(self):
    g = self._game
    return (self._device_evaluator() is not None and
            self._child_selection_fn in (SearchNode.uct_value, SearchNode.puct_value) and
            isinstance(g, pyspiel.Game) and g.on_device(numpy_policy=True) and
            g.num_players() == 2 and
            g.get_type().chance_mode == pyspiel.GameType.ChanceMode.DETERMINISTIC)

  def restart_at(self, state):
    pass

  def step_with_policy(self, state):
    t0 = time.time()
    if self._use_gpu() and not self.verbose:
      # The engine's BestChild (mcts.py sort_key order, first maximum) is all a
      # step needs: no tree export, no SearchNode objects.
      chosen = int(self._run_gpu(state)[0]["best_action"][0])
      return [(a, 1.0 if a == chosen else 0.0)
              for a in state.legal_actions(state.current_player())], chosen
    root = self.mcts_search(state)
    best = root.best_child()
    if self.verbose:
      secs = time.time() - t0
      print("Finished {} sims in {:.3f} secs, {:.1f} sims/s".format(
          root.explore_count, secs, root.explore_count / secs))
      print("Root:")
      print(root.to_str(state))
      print("Children:")
      print(root.children_str(state))
      if best.children:
        nxt = state.clone()
        nxt.apply_action(best.action)
        print("Children of chosen:")
        print(best.children_str(nxt))
    chosen = best.action
    policy = [(a, 1.0 if a == chosen else 0.0)
              for a in state.legal_actions(state.current_player())]
    return policy, chosen

  def step(self, state):
    return self.step_with_policy(state)[1]

  def _use_gpu(self):
    """backend="auto": random-rollout searches run on the device.  A search
    over an external evaluator does too under backend="hip", but "auto" keeps
    it in the host loop: one bot searches one state, so every simulation is
    one evaluator round trip (kernel step, request to the host, the model,
    answer back), and that costs more than the host loop's whole simulation
    -- connect_four, 300 simulations, PUCT + Dirichlet (alpha_zero.py:185-192):
    60.6 ms per step on the device against 13.9 ms in the host loop
    (profiles/r06/az_step_latency.md).  The batched actor (os_amd/az.py),
    thousands of searches per round, is where the device wins."""
    if self.backend == "hip":
      return True
    return self.backend == "auto" and self._rollout_eligible()

  def mcts_search(self, state):
    if self._use_gpu():
      return tree_to_search_nodes(self._run_gpu(state)[1].tree(0), state, self._game)
    if self.backend == "auto" and not self._warned_host:
      # Never a silent CPU search: say once why this bot runs on the host.
      if self._external_eligible():
        why = ("one search over an external evaluator is faster in the host loop than "
               "one device round trip per simulation; backend='hip' runs it on the device")
      else:
        why = ("the GPU engine needs RandomRolloutEvaluator without Dirichlet noise or a "
               "batched evaluator, UCT or PUCT selection and a game it runs on the device")
      warnings.warn("MCTSBot(backend='auto') runs this search on the host CPU (%s); "
                    "pass backend='host' to silence this or backend='hip' to make it "
                    "an error" % why, RuntimeWarning, stacklevel=2)
      self._warned_host = True
    return self._search_host(state)

  # ---- GPU path -------------------------------------------------------------
  def _run_gpu(self, state):
    """One search on the device continuing the RandomState streams; returns
    (root outputs, object whose tree(0) is the search tree)."""
    if not self._rollout_eligible():
      return self._run_gpu_external(state)
    eng = pyspiel._engine_for(self._game)
    bot_rs = self._random_state
    ev_rs = self.evaluator._random_state
    shared = ev_rs is bot_rs
    b = bot_rs.get_state()
    e = None if shared else ev_rs.get_state()
    out, nb, ne = eng.mcts_stateful(
        state.history(), (b[1], b[2]), None if shared else (e[1], e[2]),
        uct_c=self.uct_c, max_simulations=self.max_simulations,
        n_rollouts=self.evaluator.n_rollouts, solve=self.solve,
        max_memory_mb=0, policy=_lib.POLICY_NUMPY,
        child_selection=(_lib.SELECT_PUCT if self._child_selection_fn is SearchNode.puct_value
                         else _lib.SELECT_UCT))
    bot_rs.set_state(("MT19937", nb[0], nb[1], b[3], b[4]))
    if not shared:
      ev_rs.set_state(("MT19937", ne[0], ne[1], e[3], e[4]))
    return out, eng

  def _run_gpu_external(self, state):
    """mcts.py's search (:395-443) with a batched evaluator, in the
    external-evaluator kernel: RandomState.shuffle expansions on the bot's
    stream, no single-child stop, no GC; one evaluator round per simulation
    (fused Evaluate + Prior for a pure evaluator)."""
    search = pyspiel._az_search_for(self._game)
    rs = self._random_state
    saved = rs.get_state()
    try:
      noise = None
      eps = 0.0
      if (self._dirichlet_noise and self.max_simulations >= 2 and not state.is_terminal()):
        # mcts.py:314-316 at the root's expansion (simulation 1): the evaluator
        # drew nothing before it, so it is the search's first use of the stream.
        eps, alpha = self._dirichlet_noise
        n = len(state.legal_actions(state.current_player()))
        noise = np.zeros((1, search.eng.max_children), np.float64)
        noise[0, :n] = rs.dirichlet([alpha] * n)
      b = rs.get_state()
      hist = np.asarray(state.history(), np.int64)
      pure = bool(getattr(self.evaluator, "pure_function", False))
      out = search.run(hist, np.array([0, len(hist)], np.int64), None, self._device_evaluator(),
                       puct=self._child_selection_fn is SearchNode.puct_value,
                       max_simulations=self.max_simulations, uct_c=self.uct_c,
                       solve=self.solve, max_memory_mb=0,
                       bot_rng=(np.asarray(b[1], np.uint32)[None], np.array([b[2]], np.int32)),
                       requests="fused" if pure else "separate", policy="numpy",
                       root_noise=noise, dirichlet_epsilon=eps)
    except BaseException:
      # no search happened: the bot's stream is where the reference's would be
      rs.set_state(saved)
      raise
    keys, pos = search.bot_rng_out
    rs.set_state(("MT19937", keys[0], int(pos[0]), b[3], b[4]))
    return out, search

  # ---- generic host path (user evaluators / selection functions) ------------
  def _descend(self, root, state):
    path = [root]
    node = root
    working = state.clone()
    while not working.is_terminal() and node.explore_count > 0:
      if not node.children:
        priors = self.evaluator.prior(working)
        if node is root and self._dirichlet_noise:
          eps, alpha = self._dirichlet_noise
          noise = self._random_state.dirichlet([alpha] * len(priors))
          priors = [(a, (1 - eps) * p + eps * z)
                    for (a, p), z in zip(priors, noise)]
        self._random_state.shuffle(priors)
        mover = working.current_player()
        node.children = [SearchNode(a, mover, p) for a, p in priors]
      if working.is_chance_node():
        acts, probs = zip(*working.chance_outcomes())
        pick = self._random_state.choice(acts, p=probs)
        node = next(c for c in node.children if c.action == pick)
      else:
        parent_n = node.explore_count
        node = max(node.children,
                   key=lambda c: self._child_selection_fn(c, parent_n, self.uct_c))
      working.apply_action(node.action)
      path.append(node)
    return path, working

  def _backup(self, path, returns, root_player, solved):
    for node in reversed(path):
      who = root_player if node.player == pyspiel.PlayerId.CHANCE else node.player
      node.total_reward += returns[who]
      node.explore_count += 1
      if not (solved and node.children):
        continue
      mover = node.children[0].player
      if mover == pyspiel.PlayerId.CHANCE:
        first = node.children[0].outcome
        if first is not None and all(np.array_equal(c.outcome, first)
                                     for c in node.children):
          node.outcome = first
        else:
          solved = False
        continue
      proven = [c for c in node.children if c.outcome is not None]
      best = None
      for c in proven:
        if best is None or c.outcome[mover] > best.outcome[mover]:
          best = c
      if best is not None and (len(proven) == len(node.children) or
                               best.outcome[mover] == self.max_utility):
        node.outcome = best.outcome
      else:
        solved = False

  def _search_host(self, state):
    root_player = state.current_player()
    root = SearchNode(None, root_player, 1)
    for _ in range(self.max_simulations):
      path, working = self._descend(root, state)
      if working.is_terminal():
        returns = working.returns()
        path[-1].outcome = returns
        solved = self.solve
      else:
        returns = self.evaluator.evaluate(working)
        solved = False
      self._backup(path, returns, root_player, solved)
      if root.outcome is not None:
        break
    return root
