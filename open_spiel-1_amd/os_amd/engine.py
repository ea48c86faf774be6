"""Batched MCTS engine on one MI355X (gfx950): Python face of libos_mcts.so.

`Engine(game_string, device)` replaces a population of the reference's
`algorithms::MCTSBot` + `RandomRolloutEvaluator` pairs
(open_spiel/algorithms/mcts.h:92-159): `mcts_batch` runs one independent
`MCTSBot::MCTSearch` (mcts.cc:325-428) per root on the GPU (one wavefront
or one lane per search), bit-exact with the reference for the
same seeds.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib, ptr

OUTPUT_KEYS = ("child_action", "child_n", "child_w", "child_out", "nchild",
               "root_n", "root_w", "root_out", "best_action", "nodes")
UNSOLVED = 2


def make_params(uct_c=2.0, max_simulations=1000, n_rollouts=1,
                max_memory_mb=1000, solve=True, policy=_lib.POLICY_CPP,
                block_size=0, arena_nodes=0, layout=_lib.LAYOUT_AUTO,
                child_selection=_lib.SELECT_UCT):
  p = _lib.MctsParams()
  p.child_selection = int(child_selection)
  p.layout = int(layout)
  p.uct_c = float(uct_c)
  p.max_simulations = int(max_simulations)
  p.n_rollouts = int(n_rollouts)
  p.max_memory_mb = int(max_memory_mb)
  p.solve = 1 if solve else 0
  p.policy = int(policy)
  p.block_size = int(block_size)
  p.arena_nodes = int(arena_nodes)
  return p


def _alloc_outputs(R, mc):
  return dict(
      child_action=np.zeros((R, mc), np.int32),
      child_n=np.zeros((R, mc), np.int32),
      child_w=np.zeros((R, mc), np.float64),
      child_out=np.zeros((R, mc), np.int8),
      nchild=np.zeros(R, np.int32),
      root_n=np.zeros(R, np.int32),
      root_w=np.zeros(R, np.float64),
      root_out=np.zeros(R, np.int8),
      best_action=np.zeros(R, np.int64),
      nodes=np.zeros(R, np.int32))


def _out_ptrs(o):
  return [ptr(o[k]) for k in OUTPUT_KEYS]


def roots_from_histories(histories):
  """[[a0, a1, ...], ...] -> (actions int64[], offsets int64[R+1])."""
  offs = np.zeros(len(histories) + 1, np.int64)
  for i, h in enumerate(histories):
    offs[i + 1] = offs[i] + len(h)
  acts = np.zeros(int(offs[-1]), np.int64)
  for i, h in enumerate(histories):
    acts[offs[i]:offs[i + 1]] = h
  return acts, offs


class Engine:
  """One engine per device (C-ABI os_engine)."""

  def __init__(self, game_string, device=0):
    h = ctypes.c_void_p()
    check(lib.os_engine_create(game_string.encode(), int(device), ctypes.byref(h)))
    self._h = h
    self.game_string = game_string
    self.device = device
    g = ctypes.c_void_p()
    check(lib.os_game_load(game_string.encode(), ctypes.byref(g)))
    info = _lib.GameInfo()
    check(lib.os_game_get_info(g, ctypes.byref(info)))
    lib.os_game_free(g)
    self.num_distinct_actions = info.num_distinct_actions
    self.max_children = info.max_children
    self.max_game_length = info.max_game_length
    shape = np.zeros(3, np.int32)
    g2 = ctypes.c_void_p()
    check(lib.os_game_load(game_string.encode(), ctypes.byref(g2)))
    lib.os_game_observation_shape(g2, ptr(shape))
    lib.os_game_free(g2)
    self.observation_shape = [int(x) for x in shape]

  def close(self):
    if getattr(self, "_h", None) and self._h.value:
      lib.os_engine_destroy(self._h)
      self._h = ctypes.c_void_p()

  def __del__(self):
    try:
      self.close()
    except Exception:  # interpreter shutdown
      pass

  def mcts_batch(self, root_actions, root_offsets, bot_seeds, eval_seeds=None,
                 **params):
    """Independent searches; returns dict of numpy arrays (child order)."""
    p = make_params(**params)
    acts = _lib.i64(root_actions)
    offs = _lib.i64(root_offsets)
    R = len(offs) - 1
    bs = _lib.u32(bot_seeds)
    es = _lib.u32(eval_seeds if eval_seeds is not None else bot_seeds)
    assert len(bs) == R and len(es) == R
    mc = self.max_children
    o = _alloc_outputs(R, mc)
    check(lib.os_mcts_batch(self._h, ctypes.byref(p), R, ptr(acts), ptr(offs),
                            ptr(bs), ptr(es), mc, *_out_ptrs(o)))
    return o

  def mcts_stateful(self, history, bot_state, eval_state=None, **params):
    """One search continuing caller-owned MT19937 streams.

    bot_state / eval_state: (key uint32[624], pos) pairs (numpy legacy
    RandomState form); the advanced states are returned.  eval_state None =>
    one shared stream (numpy policy only).
    """
    p = make_params(**params)
    acts = _lib.i64(history)
    bkey = np.array(bot_state[0], dtype=np.uint32).copy()
    bpos = np.array([bot_state[1]], dtype=np.int32)
    shared = eval_state is None
    if shared:
      ekey, epos = None, None
    else:
      ekey = np.array(eval_state[0], dtype=np.uint32).copy()
      epos = np.array([eval_state[1]], dtype=np.int32)
    mc = self.max_children
    o = _alloc_outputs(1, mc)
    check(lib.os_mcts_stateful(self._h, ctypes.byref(p), ptr(acts), len(acts),
                                  1 if shared else 0, ptr(bkey), ptr(bpos),
                                  ptr(ekey), ptr(epos), mc, *_out_ptrs(o)))
    new_eval = None if shared else (ekey, int(epos[0]))
    return o, (bkey, int(bpos[0])), new_eval

  def tree(self, r=0):
    """Flat tree of root r of the last search: dict of node arrays."""
    cnt = ctypes.c_int64()
    check(lib.os_engine_tree(self._h, r, ctypes.addressof(cnt), None, None, None,
                             None, None, None))
    n = cnt.value
    t = dict(first=np.zeros(n, np.uint32), n=np.zeros(n, np.int32),
             w=np.zeros(n, np.float64), action=np.zeros(n, np.int32),
             nchild=np.zeros(n, np.int32), out0=np.zeros(n, np.int8))
    check(lib.os_engine_tree(self._h, r, ctypes.addressof(cnt), ptr(t["first"]),
                             ptr(t["n"]), ptr(t["w"]), ptr(t["action"]),
                             ptr(t["nchild"]), ptr(t["out0"])))
    return t

  def rollouts(self, history, seeds, n_rollouts=1, layout=_lib.LAYOUT_LANE):
    """RandomRolloutEvaluator(n_rollouts, seed).Evaluate(root) per seed."""
    check(lib.os_engine_set_rollout_layout(self._h, int(layout)))
    acts = _lib.i64(history)
    s = _lib.u32(seeds)
    out = np.zeros((len(s), 2), np.float64)
    check(lib.os_rollouts_batch(self._h, ptr(acts), len(acts), len(s),
                                int(n_rollouts), ptr(s), ptr(out)))
    return out

  def rollouts_prepare(self, history, seeds, n_rollouts=1, layout=_lib.LAYOUT_LANE):
    """Device-resident rollout batch (see os_rollouts_prepare)."""
    check(lib.os_engine_set_rollout_layout(self._h, int(layout)))
    self._roll = (_lib.i64(history), _lib.u32(seeds))
    acts, s = self._roll
    check(lib.os_rollouts_prepare(self._h, ptr(acts), len(acts), len(s),
                                  int(n_rollouts), ptr(s)))

  def rollouts_run_async(self, stream=None):
    check(lib.os_rollouts_run_async(self._h, stream))

  def rollouts_fetch(self):
    out = np.zeros((len(self._roll[1]), 2), np.float64)
    check(lib.os_rollouts_fetch(self._h, ptr(out)))
    return out

  def rollouts_stats(self):
    """Counters of the last lane-layout rollout run (os_rollouts_stats)."""
    out = np.zeros(3, np.int64)
    check(lib.os_rollouts_stats(self._h, ptr(out)))
    return {"rng_words": int(out[0]), "moves": int(out[1]), "state_bytes": int(out[2])}

  def rollouts_algorithmic_bytes(self, n):
    """HBM bytes n playouts must move: one MT19937 state
    word read + written per word drawn, one position-hash log write + probe
    (16 B) per move, one root state read per playout."""
    s = self.rollouts_stats()
    return s["rng_words"] * 8 + s["moves"] * 16 + n * s["state_bytes"]

  def rollouts_outcomes_async(self, dev_counts_ptr, stream=None):
    """Writes int64[3] (p0 wins, p1 wins, draws) to a device address."""
    check(lib.os_rollouts_outcomes_async(self._h, dev_counts_ptr, stream))

  def root_sums_async(self, num_actions, dev_visits_ptr, dev_rewards_ptr, stream=None):
    """Action-indexed root visit / reward sums of the last run into device
    buffers int64[num_actions] / f64[num_actions] (root-parallel MCTS)."""
    check(lib.os_engine_root_sums_async(self._h, int(num_actions), dev_visits_ptr,
                                        dev_rewards_ptr, stream))

  # ---- self-play (two MCTSBots + one shared RandomRolloutEvaluator) ----
  def selfplay_set_options(self, actor_seeds=None, temperature=0.0, temperature_drop=0,
                           resign=False, cutoff_value=0.9, cutoff_probability=0.8):
    """AlphaZero's PlayGame move choice for the next self-play batch
    (include/os_mcts.h os_selfplay_set_options; alpha_zero.cc:64-118):
    visit-count^(1/temperature) policy sampled from each game's actor rng
    (actor_seeds[g]) before temperature_drop moves, resignation at
    |root value| > cutoff.  No actor seeds: BestChild every move."""
    o = _lib.SelfPlayOptions()
    o.temperature = float(temperature)
    o.temperature_drop = int(temperature_drop)
    o.resign = 1 if resign else 0
    o.cutoff_value = float(cutoff_value)
    o.cutoff_probability = float(cutoff_probability)
    seeds = _lib.u32(actor_seeds if actor_seeds is not None else [])
    check(lib.os_selfplay_set_options(self._h, ctypes.byref(o), len(seeds), ptr(seeds)))

  def selfplay_prepare(self, start_actions, start_offsets, bot_seeds, eval_seeds,
                       max_len=None, record_visits=True, record_observations=False,
                       record_policy=False, record_root_values=False, **params):
    """Device self-play batch (os_selfplay_prepare).  bot_seeds: [G][2]."""
    self._sp_params = make_params(**params)
    offs = _lib.i64(start_offsets)
    G = len(offs) - 1
    bs = _lib.u32(np.asarray(bot_seeds, np.uint32).reshape(-1))
    es = _lib.u32(eval_seeds)
    assert len(bs) == 2 * G and len(es) == G
    self._sp = (_lib.i64(start_actions), offs, bs, es)
    self._sp_G = G
    self._sp_len = int(max_len if max_len is not None else self.max_game_length)
    self._sp_vis = bool(record_visits)
    self._sp_obs = bool(record_observations)
    self._sp_pol = bool(record_policy)
    self._sp_val = bool(record_root_values)
    acts = self._sp[0]
    record = ((_lib.RECORD_VISITS if record_visits else 0) |
              (_lib.RECORD_OBSERVATIONS if record_observations else 0) |
              (_lib.RECORD_POLICY if record_policy else 0) |
              (_lib.RECORD_ROOT_VALUES if record_root_values else 0))
    check(lib.os_selfplay_prepare(self._h, ctypes.byref(self._sp_params), G, ptr(acts),
                                  ptr(offs), ptr(bs), ptr(es), self._sp_len, record))

  def selfplay_run_async(self, stream=None):
    check(lib.os_selfplay_run_async(self._h, stream))

  def selfplay_fetch(self):
    G, L, A = self._sp_G, self._sp_len, self.num_distinct_actions
    o = dict(actions=np.zeros((G, L), np.int64), length=np.zeros(G, np.int32),
             returns=np.zeros((G, 2), np.float64),
             visits=np.zeros((G, L, A), np.int32) if self._sp_vis else None,
             observations=(np.zeros((G, L) + tuple(self.observation_shape), np.float32)
                           if self._sp_obs else None))
    check(lib.os_selfplay_fetch(self._h, ptr(o["actions"]), ptr(o["length"]),
                                ptr(o["returns"]), ptr(o["visits"]),
                                ptr(o["observations"])))
    o["policy"] = np.zeros((G, L, A), np.float64) if self._sp_pol else None
    o["root_value"] = np.zeros((G, L), np.float64) if self._sp_val else None
    if self._sp_pol or self._sp_val:
      check(lib.os_selfplay_fetch_targets(self._h, ptr(o["policy"]), ptr(o["root_value"])))
    return o

  def selfplay(self, start_actions, start_offsets, bot_seeds, eval_seeds, max_len=None,
               record_visits=True, record_observations=False, record_policy=False,
               record_root_values=False, **params):
    """Plays G games on the device; see include/os_mcts.h os_selfplay."""
    self.selfplay_prepare(start_actions, start_offsets, bot_seeds, eval_seeds, max_len,
                          record_visits, record_observations, record_policy,
                          record_root_values, **params)
    self.selfplay_run_async()
    return self.selfplay_fetch()

  # ---- device-resident pipeline (bench) ----
  def prepare(self, root_actions, root_offsets, bot_seeds, eval_seeds=None,
              **params):
    self._prep_params = make_params(**params)
    self._prep = (_lib.i64(root_actions), _lib.i64(root_offsets),
                  _lib.u32(bot_seeds),
                  _lib.u32(eval_seeds if eval_seeds is not None else bot_seeds))
    acts, offs, bs, es = self._prep
    self._prep_R = len(offs) - 1
    check(lib.os_engine_prepare(self._h, ctypes.byref(self._prep_params),
                                self._prep_R, ptr(acts), ptr(offs), ptr(bs),
                                ptr(es)))

  def run_async(self, stream=None):
    """Launches the search kernel(s) on a hipStream_t (int handle) or NULL."""
    check(lib.os_engine_run_async(self._h, stream))

  def fetch(self):
    o = _alloc_outputs(self._prep_R, self.max_children)
    check(lib.os_engine_fetch(self._h, self.max_children, *_out_ptrs(o)))
    return o

  def layout(self):
    """Kernel layout of the last prepared batch (_lib.LAYOUT_WAVE / LAYOUT_LANE)."""
    out = np.zeros(1, np.int32)
    check(lib.os_engine_get_layout(self._h, ptr(out)))
    return int(out[0])

  def searches_per_wave(self):
    """Searches per wavefront of the last search launch (1 on the wave
    layout; the lane layout's block width)."""
    out = np.zeros(1, np.int32)
    check(lib.os_engine_get_searches_per_wave(self._h, ptr(out)))
    return int(out[0])

  def last_sims(self):
    return int(lib.os_engine_last_sims(self._h))

  STAT_KEYS = ("sims", "scanned", "backed", "expanded", "solver_scanned",
               "rng_words", "nodes", "used", "max_depth", "gc_runs")

  def stats(self):
    """Instrumentation counters of the last fetched run (summed over roots)."""
    out = np.zeros(10, np.int64)
    check(lib.os_engine_stats(self._h, ptr(out)))
    d = {k: int(v) for k, v in zip(self.STAT_KEYS, out)}
    d["node_bytes"] = int(lib.os_engine_node_bytes(self._h))
    d["state_bytes"] = int(lib.os_engine_state_bytes(self._h))
    return d

  ARENA_KEYS = ("paged", "nodes_per_page_or_root", "pool_pages_or_chunk_roots",
                "arena_bytes", "pages_used", "reruns", "overflowed_searches",
                "reserved_bytes")

  def set_arena_mode(self, mode):
    """"reserved" (worst case per root) or "paged" (a page pool sized from
    earlier fetched runs; include/os_mcts.h os_engine_set_arena_mode)."""
    modes = {"reserved": 0, "paged": 1}
    if mode not in modes:
      raise ValueError("arena mode must be 'reserved' or 'paged'")
    check(lib.os_engine_set_arena_mode(self._h, modes[mode]))

  def arena_info(self):
    """Arena of the prepared batch (os_engine_arena_info)."""
    out = np.zeros(8, np.int64)
    check(lib.os_engine_arena_info(self._h, ptr(out)))
    return {k: int(v) for k, v in zip(self.ARENA_KEYS, out)}

  def algorithmic_bytes(self, num_roots):
    """HBM bytes the search must move, from the instrumentation.

    Per simulation the algorithm reads every child scanned by UCT selection,
    reads+writes each backed-up node, writes each expanded child, reads the
    children the solver backup inspects, and reads+writes one MT19937 state
    word per word drawn; plus one root state read per search.
    """
    s = self.stats()
    nb = s["node_bytes"]
    return (s["scanned"] * nb + s["backed"] * 2 * nb + s["expanded"] * nb +
            s["solver_scanned"] * nb + s["rng_words"] * 8 +
            num_roots * s["state_bytes"])


def root_parallel(engines, root_actions, trees_per_device, seed_base=0, **params):
  """Root-parallel search over the engines' devices in one process (C-ABI
  os_root_parallel): returns (visits int64[A], rewards f64[A], sims), the
  action-indexed sums of every tree's root children.  Tree t of engine g is
  seeded seed_base + g * trees_per_device + t (evaluator: + 2^20)."""
  p = make_params(**params)
  A = engines[0].num_distinct_actions
  hs = (ctypes.c_void_p * len(engines))(*[e._h for e in engines])
  acts = _lib.i64(root_actions)
  visits = np.zeros(A, np.int64)
  rewards = np.zeros(A, np.float64)
  sims = np.zeros(1, np.int64)
  check(lib.os_root_parallel(ctypes.cast(hs, ctypes.c_void_p), len(engines), ctypes.byref(p),
                             ptr(acts), len(acts), int(trees_per_device), int(seed_base), A,
                             ptr(visits), ptr(rewards), ptr(sims)))
  for e in engines:  # each engine now holds a prepared batch of T trees (fetchable)
    e._prep_R = int(trees_per_device)
  return visits, rewards, int(sims[0])


def make_roots(game_string, num_roots, seed_base=1000, max_plies=8):
  """Benchmark roots: see os_make_roots in include/os_mcts.h."""
  g = ctypes.c_void_p()
  check(lib.os_game_load(game_string.encode(), ctypes.byref(g)))
  try:
    total = lib.os_make_roots(g, num_roots, seed_base, max_plies, None, None)
    if total < 0:
      check(int(total))
    acts = np.zeros(max(int(total), 1), np.int64)
    offs = np.zeros(num_roots + 1, np.int64)
    lib.os_make_roots(g, num_roots, seed_base, max_plies, ptr(acts), ptr(offs))
    return acts[:int(total)].copy(), offs
  finally:
    lib.os_game_free(g)


def action_indexed_visits(out, num_actions):
  """[R][A] visit counts from child-ordered outputs (root-parallel reduce)."""
  R = out["nchild"].shape[0]
  v = np.zeros((R, num_actions), np.int64)
  for r in range(R):
    nc = out["nchild"][r]
    np.add.at(v[r], out["child_action"][r, :nc], out["child_n"][r, :nc])
  return v
