"""ctypes wrapper for oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the reference-faithful CPU restatement (oracle/*.cc).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
only as the checker / CPU baseline.
"""
import ctypes
import json
import os
import subprocess

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB_PATH = os.path.join(_ROOT, "oracle", "build", "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
# int cb(const int64_t* history, int64_t n, int32_t kind, double* prior, double* value)
EVAL_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64,
                           ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                           ctypes.POINTER(ctypes.c_double))


def build():
  subprocess.check_call(["make", "-s", "-C", os.path.join(_ROOT, "oracle")])


def lib():
  global _lib
  if _lib is None:
    if not os.path.exists(_LIB_PATH):
      build()
    L = ctypes.CDLL(_LIB_PATH)
    L.oref_last_error.restype = ctypes.c_char_p
    L.oref_game_new.restype = ctypes.c_void_p
    L.oref_game_new.argtypes = [ctypes.c_char_p]
    L.oref_game_free.argtypes = [ctypes.c_void_p]
    L.oref_game_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                 ctypes.POINTER(ctypes.c_int32)]
    L.oref_state_json.restype = ctypes.c_int64
    L.oref_state_json.argtypes = [ctypes.c_void_p, _i64p, ctypes.c_int64,
                                  ctypes.c_char_p, ctypes.c_int64]
    L.oref_go_score.restype = ctypes.c_float
    L.oref_go_score.argtypes = [ctypes.c_void_p, _i64p, ctypes.c_int64]
    L.oref_rollouts.argtypes = [ctypes.c_void_p, _i64p, ctypes.c_int64,
                                ctypes.c_int64, ctypes.c_int32, _u32p, _f64p,
                                ctypes.c_void_p]
    L.oref_mcts_batch.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double,
        ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _u32p,
        _u32p, ctypes.c_int32, _i32p, _i32p, _f64p, _i8p, _i32p, _i32p, _f64p,
        _i8p, _i64p, _i32p, ctypes.c_int32, ctypes.c_int32]
    L.oref_mcts_numpy.argtypes = [
        ctypes.c_void_p, _i64p, ctypes.c_int64, ctypes.c_double, ctypes.c_int32,
        ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32, _i32p,
        _i32p, _f64p, _i8p, _i32p, _i32p, _f64p, _i8p, _i64p, _i32p, _u32p,
        ctypes.c_int32]
    L.oref_mt19937.argtypes = [ctypes.c_uint32, ctypes.c_int64, _u32p]
    L.oref_mt19937_64.argtypes = [ctypes.c_uint64, ctypes.c_int64, _u64p]
    L.oref_absl_uniform.argtypes = [ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_int64, _u64p]
    L.oref_std_shuffle.argtypes = [ctypes.c_uint32, ctypes.c_int32, _i32p]
    L.oref_time_mcts_batch.restype = ctypes.c_double
    L.oref_time_mcts_batch.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double,
        ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _u32p,
        _u32p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
    L.oref_mcts_external.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double, ctypes.c_int32,
        ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
        _u32p, EVAL_CB, ctypes.c_int32,
        _i32p, _i32p, _f64p, _i8p, _i32p, _i32p, _f64p, _i8p, _i64p, _i32p]
    L.oref_selfplay.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double,
        ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, _u32p,
        _u32p, ctypes.c_int32, _i64p, _i32p, _f64p, ctypes.c_void_p, ctypes.c_int32]
    L.oref_selfplay_az.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double, ctypes.c_int32,
        ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _u32p, _u32p, _u32p,
        ctypes.c_double, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
        ctypes.c_int32, _i64p, _i32p, _f64p, _f64p, _f64p]
    L.oref_az_actor.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double, ctypes.c_int32,
        ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
        _u32p, _u32p, ctypes.c_double, ctypes.c_int32, ctypes.c_int32, ctypes.c_double,
        ctypes.c_double, EVAL_CB, ctypes.c_int32, _i64p, _i32p, _f64p, _f64p, _f64p]
    L.oref_time_mcts_zero_eval.restype = ctypes.c_double
    L.oref_time_mcts_zero_eval.argtypes = [
        ctypes.c_void_p, ctypes.c_int64, _i64p, _i64p, ctypes.c_double, ctypes.c_int32,
        ctypes.c_int32, ctypes.c_double, ctypes.c_double, _u32p, ctypes.c_int32,
        ctypes.POINTER(ctypes.c_int64)]
    L.oref_evaluate_mcts_bots.restype = ctypes.c_int64
    L.oref_evaluate_mcts_bots.argtypes = [
        ctypes.c_void_p, ctypes.c_int32, _u32p, ctypes.c_int32, ctypes.c_uint32,
        ctypes.c_double, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32,
        _i64p, ctypes.c_int64, _f64p]
    _lib = L
  return _lib


class Game:
  """Oracle game handle (reference-faithful restatement)."""

  def __init__(self, game_string):
    self._h = lib().oref_game_new(game_string.encode())
    if not self._h:
      raise ValueError(lib().oref_last_error().decode())
    na, ml = ctypes.c_int32(), ctypes.c_int32()
    lib().oref_game_info(self._h, ctypes.byref(na), ctypes.byref(ml))
    self.num_distinct_actions = na.value
    self.max_game_length = ml.value

  def __del__(self):
    if getattr(self, "_h", None) and _lib is not None:
      _lib.oref_game_free(self._h)

  def state_info(self, history):
    a = np.ascontiguousarray(history, dtype=np.int64)
    n = lib().oref_state_json(self._h, a, len(a), None, 0)
    buf = ctypes.create_string_buffer(int(n) + 1)
    lib().oref_state_json(self._h, a, len(a), buf, n + 1)
    return json.loads(buf.value.decode())

  def go_score(self, history):
    a = np.ascontiguousarray(history, dtype=np.int64)
    return float(lib().oref_go_score(self._h, a, len(a)))

  def rollouts(self, history, seeds, n_rollouts=1):
    a = np.ascontiguousarray(history, dtype=np.int64)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
    out = np.zeros((len(seeds), 2), np.float64)
    lib().oref_rollouts(self._h, a, len(a), len(seeds), n_rollouts, seeds, out,
                        None)
    return out

  def mcts_batch(self, root_actions, root_offsets, bot_seeds, eval_seeds,
                 uct_c=2.0, max_simulations=1000, n_rollouts=1,
                 max_memory_mb=1000, solve=True, max_children=None, threads=1,
                 puct=False):
    R = len(root_offsets) - 1
    mc = max_children or self.num_distinct_actions
    out = dict(
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
    lib().oref_mcts_batch(
        self._h, R, np.ascontiguousarray(root_actions, dtype=np.int64),
        np.ascontiguousarray(root_offsets, dtype=np.int64), uct_c,
        max_simulations, n_rollouts, max_memory_mb, int(solve),
        np.ascontiguousarray(bot_seeds, dtype=np.uint32),
        np.ascontiguousarray(eval_seeds, dtype=np.uint32), mc,
        out["child_action"], out["child_n"], out["child_w"], out["child_out"],
        out["nchild"], out["root_n"], out["root_w"], out["root_out"],
        out["best_action"], out["nodes"], threads, int(bool(puct)))
    return out

  def mcts_numpy(self, history, seed, uct_c=2.0, max_simulations=1000,
                 n_rollouts=1, solve=True, puct=False):
    mc = self.num_distinct_actions
    out = dict(
        child_action=np.zeros((1, mc), np.int32),
        child_n=np.zeros((1, mc), np.int32),
        child_w=np.zeros((1, mc), np.float64),
        child_out=np.zeros((1, mc), np.int8),
        nchild=np.zeros(1, np.int32), root_n=np.zeros(1, np.int32),
        root_w=np.zeros(1, np.float64), root_out=np.zeros(1, np.int8),
        best_action=np.zeros(1, np.int64), nodes=np.zeros(1, np.int32),
        next_word=np.zeros(1, np.uint32))
    a = np.ascontiguousarray(history, dtype=np.int64)
    lib().oref_mcts_numpy(
        self._h, a, len(a), uct_c, max_simulations, n_rollouts, int(solve),
        seed, mc, out["child_action"], out["child_n"], out["child_w"],
        out["child_out"], out["nchild"], out["root_n"], out["root_w"],
        out["root_out"], out["best_action"], out["nodes"], out["next_word"],
        int(bool(puct)))
    return out

  def time_mcts_batch(self, root_actions, root_offsets, bot_seeds, eval_seeds,
                      uct_c=2.0, max_simulations=1024, n_rollouts=1,
                      max_memory_mb=1000, solve=True, threads=1):
    R = len(root_offsets) - 1
    sims = ctypes.c_int64()
    secs = lib().oref_time_mcts_batch(
        self._h, R, np.ascontiguousarray(root_actions, dtype=np.int64),
        np.ascontiguousarray(root_offsets, dtype=np.int64), uct_c,
        max_simulations, n_rollouts, max_memory_mb, int(solve),
        np.ascontiguousarray(bot_seeds, dtype=np.uint32),
        np.ascontiguousarray(eval_seeds, dtype=np.uint32), threads,
        ctypes.byref(sims))
    return secs, sims.value

  def time_mcts_zero_eval(self, root_actions, root_offsets, bot_seeds, uct_c=2.0,
                          max_simulations=100, puct=True, dirichlet_alpha=0.0,
                          dirichlet_epsilon=0.0, threads=1):
    """(seconds, sims) of MCTSBot searches with a free native evaluator."""
    R = len(root_offsets) - 1
    sims = ctypes.c_int64()
    secs = lib().oref_time_mcts_zero_eval(
        self._h, R, np.ascontiguousarray(root_actions, dtype=np.int64),
        np.ascontiguousarray(root_offsets, dtype=np.int64), uct_c, max_simulations, int(puct),
        dirichlet_alpha, dirichlet_epsilon, np.ascontiguousarray(bot_seeds, dtype=np.uint32),
        threads, ctypes.byref(sims))
    return secs, sims.value

  def mcts_external(self, root_actions, root_offsets, bot_seeds, eval_fn, puct=True,
                    uct_c=2.0, max_simulations=100, max_memory_mb=1000, solve=True,
                    max_children=None, dirichlet_alpha=0.0, dirichlet_epsilon=0.0):
    """MCTSBot with an external evaluator: eval_fn(history, kind) -> (prior
    [A] action-indexed, value for player 0); kind 1 = Prior, 2 = Evaluate."""
    R = len(root_offsets) - 1
    mc = max_children or self.num_distinct_actions
    A = self.num_distinct_actions
    out = dict(
        child_action=np.zeros((R, mc), np.int32), child_n=np.zeros((R, mc), np.int32),
        child_w=np.zeros((R, mc), np.float64), child_out=np.zeros((R, mc), np.int8),
        nchild=np.zeros(R, np.int32), root_n=np.zeros(R, np.int32),
        root_w=np.zeros(R, np.float64), root_out=np.zeros(R, np.int8),
        best_action=np.zeros(R, np.int64), nodes=np.zeros(R, np.int32))
    out["child_action"][:] = -1
    out["child_out"][:] = 2

    def cb(hist, n, kind, prior_out, value_out):
      h = [int(hist[i]) for i in range(n)]
      pr, v = eval_fn(h, int(kind))
      for a in range(A):
        prior_out[a] = float(pr[a])
      value_out[0] = float(v)
      return 0

    fn = EVAL_CB(cb)
    lib().oref_mcts_external(
        self._h, R, np.ascontiguousarray(root_actions, dtype=np.int64),
        np.ascontiguousarray(root_offsets, dtype=np.int64), uct_c, max_simulations,
        max_memory_mb, int(solve), int(puct), float(dirichlet_alpha), float(dirichlet_epsilon),
        np.ascontiguousarray(bot_seeds, dtype=np.uint32), fn, mc, out["child_action"],
        out["child_n"], out["child_w"], out["child_out"], out["nchild"], out["root_n"],
        out["root_w"], out["root_out"], out["best_action"], out["nodes"])
    return out

  def az_actor(self, start_actions, start_offsets, bot_seeds, actor_seeds, eval_fn, max_len,
               uct_c=2.0, max_simulations=50, max_memory_mb=10, solve=False, puct=True,
               dirichlet_alpha=0.0, dirichlet_epsilon=0.0, temperature=1.0,
               temperature_drop=10, resign=False, cutoff_value=0.9, cutoff_probability=0.8):
    """AlphaZero actor games (oref_az_actor): MCTSBots with the external
    evaluator eval_fn(history, kind) -> (prior [A], player-0 value)."""
    G = len(start_offsets) - 1
    A = self.num_distinct_actions
    out = dict(actions=np.zeros((G, max_len), np.int64), length=np.zeros(G, np.int32),
               returns=np.zeros((G, 2), np.float64),
               policy=np.zeros((G, max_len, A), np.float64),
               root_value=np.zeros((G, max_len), np.float64))

    def cb(hist, n, kind, prior_out, value_out):
      pr, v = eval_fn([int(hist[i]) for i in range(n)], int(kind))
      for a in range(A):
        prior_out[a] = float(pr[a])
      value_out[0] = float(v)
      return 0

    fn = EVAL_CB(cb)
    rc = lib().oref_az_actor(
        self._h, G, np.ascontiguousarray(start_actions, dtype=np.int64),
        np.ascontiguousarray(start_offsets, dtype=np.int64), uct_c, max_simulations,
        max_memory_mb, int(solve), int(puct), float(dirichlet_alpha), float(dirichlet_epsilon),
        np.ascontiguousarray(bot_seeds, dtype=np.uint32).reshape(-1),
        np.ascontiguousarray(actor_seeds, dtype=np.uint32), float(temperature),
        int(temperature_drop), int(bool(resign)), float(cutoff_value),
        float(cutoff_probability), fn, max_len, out["actions"], out["length"], out["returns"],
        out["policy"], out["root_value"])
    if rc:
      raise RuntimeError("oref_az_actor: game longer than max_len")
    return out

  def selfplay(self, start_actions, start_offsets, bot_seeds, eval_seeds, max_len,
               uct_c=2.0, max_simulations=100, n_rollouts=1, max_memory_mb=1000,
               solve=True, with_visits=True, threads=1, truncate=False):
    """Games of two MCTSBots sharing one evaluator (mcts_example.cc PlayGame).
    truncate: stop every game after max_len moves (the prefix) instead of
    raising.

    bot_seeds: [G][2]; eval_seeds: [G].  Returns dict(actions [G][max_len]
    (-1 padded), length [G], returns [G][2], visits [G][max_len][A] or None).
    """
    G = len(start_offsets) - 1
    A = self.num_distinct_actions
    out = dict(actions=np.zeros((G, max_len), np.int64),
               length=np.zeros(G, np.int32), returns=np.zeros((G, 2), np.float64),
               visits=np.zeros((G, max_len, A), np.int32) if with_visits else None)
    rc = lib().oref_selfplay(
        self._h, G, np.ascontiguousarray(start_actions, dtype=np.int64),
        np.ascontiguousarray(start_offsets, dtype=np.int64), uct_c, max_simulations,
        n_rollouts, max_memory_mb, int(solve),
        np.ascontiguousarray(bot_seeds, dtype=np.uint32).reshape(-1),
        np.ascontiguousarray(eval_seeds, dtype=np.uint32), max_len, out["actions"],
        out["length"], out["returns"],
        out["visits"].ctypes.data if with_visits else None, threads)
    if rc and not truncate:
      raise RuntimeError("oref_selfplay: game longer than max_len")
    return out


def evaluate_mcts_bots(game_string, bot_seeds, n_rollouts, eval_seed, seed, uct_c=2.0,
                       max_simulations=100, max_memory_mb=5, solve=True, num_players=2):
  """EvaluateBots over MCTSBots sharing one RandomRolloutEvaluator
  (mcts_test.cc:24-36 InitBot): (history, returns)."""
  g = Game(game_string)
  hist = np.zeros(100000, np.int64)
  ret = np.zeros(num_players, np.float64)
  n = lib().oref_evaluate_mcts_bots(
      g._h, len(bot_seeds), np.ascontiguousarray(bot_seeds, dtype=np.uint32), n_rollouts,
      eval_seed, uct_c, max_simulations, max_memory_mb, int(solve), seed, hist, len(hist), ret)
  assert n >= 0
  return [int(a) for a in hist[:n]], [float(x) for x in ret]


def selfplay_az(game_string, start_actions, start_offsets, bot_seeds, eval_seeds, actor_seeds,
                max_len, uct_c=2.0, max_simulations=100, n_rollouts=1, max_memory_mb=1000,
                solve=True, puct=False, temperature=1.0, temperature_drop=10, resign=False,
                cutoff_value=0.9, cutoff_probability=0.8):
  """AlphaZero PlayGame move choice over self-play MCTSBots (oref_selfplay_az)."""
  g = Game(game_string)
  G = len(start_offsets) - 1
  A = g.num_distinct_actions
  out = dict(actions=np.zeros((G, max_len), np.int64), length=np.zeros(G, np.int32),
             returns=np.zeros((G, 2), np.float64), policy=np.zeros((G, max_len, A), np.float64),
             root_value=np.zeros((G, max_len), np.float64))
  rc = lib().oref_selfplay_az(
      g._h, G, np.ascontiguousarray(start_actions, dtype=np.int64),
      np.ascontiguousarray(start_offsets, dtype=np.int64), uct_c, max_simulations, n_rollouts,
      max_memory_mb, int(solve), int(puct),
      np.ascontiguousarray(bot_seeds, dtype=np.uint32).reshape(-1),
      np.ascontiguousarray(eval_seeds, dtype=np.uint32),
      np.ascontiguousarray(actor_seeds, dtype=np.uint32), float(temperature),
      int(temperature_drop), int(bool(resign)), float(cutoff_value), float(cutoff_probability),
      max_len, out["actions"], out["length"], out["returns"], out["policy"], out["root_value"])
  if rc:
    raise RuntimeError("oref_selfplay_az: game longer than max_len")
  return out


def mt19937(seed, n):
  out = np.zeros(n, np.uint32)
  lib().oref_mt19937(seed, n, out)
  return out


def mt19937_64(seed, n):
  out = np.zeros(n, np.uint64)
  lib().oref_mt19937_64(seed, n, out)
  return out


def absl_uniform(seed, n, k):
  out = np.zeros(k, np.uint64)
  lib().oref_absl_uniform(seed, n, k, out)
  return out


def std_shuffle(seed, n):
  out = np.zeros(n, np.int32)
  lib().oref_std_shuffle(seed, n, out)
  return out
