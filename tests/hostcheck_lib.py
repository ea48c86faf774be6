"""ctypes wrapper for tests/hostcheck (product engine compiled for the host).

TEST INFRASTRUCTURE ONLY: lets the CPU suite check the exact search logic the
gfx950 kernel runs (csrc/os_mcts.h, os_games.h, os_rng.h) against the oracle.
"""
import ctypes
import os

import numpy as np

_ROOT = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_ROOT, "hostcheck", "build", "libhostcheck.so")
_lib = None


def lib():
  global _lib
  if _lib is None:
    L = ctypes.CDLL(_PATH)
    L.hc_last_error.restype = ctypes.c_char_p
    vp = ctypes.c_void_p
    L.hc_mcts_batch.argtypes = [ctypes.c_char_p, ctypes.c_int64, vp, vp,
                                ctypes.c_double, ctypes.c_int32, ctypes.c_int32,
                                ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                vp, vp, ctypes.c_int32] + [vp] * 10
    L.hc_rollouts.argtypes = [ctypes.c_char_p, vp, ctypes.c_int64, ctypes.c_int64,
                              vp, vp]
    L.hc_rollouts_go_bloom.argtypes = L.hc_rollouts.argtypes
    L.hc_rollouts_go_logbloom.argtypes = L.hc_rollouts.argtypes
    L.hc_rollouts_go_link16.argtypes = L.hc_rollouts.argtypes
    L.hc_rollouts_go9.argtypes = L.hc_rollouts.argtypes
    L.hc_b96_selftest.restype = ctypes.c_int64
    L.hc_b96_selftest.argtypes = [ctypes.c_uint64, ctypes.c_int64]
    L.hc_go_score.restype = ctypes.c_float
    L.hc_go_score.argtypes = [ctypes.c_char_p, vp, ctypes.c_int64]
    L.hc_mt_words.argtypes = [ctypes.c_uint32, ctypes.c_int64, vp]
    L.hc_mt_words_soa.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, vp]
    L.hc_mt_words_pf.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, vp]
    L.hc_mt_words_reg.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, vp]
    L.hc_mt_pf_roundtrip.argtypes = [vp, vp, ctypes.c_int64, vp]
    L.hc_mt_words_wc.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, vp]
    L.hc_mt_wc_roundtrip.argtypes = [vp, vp, ctypes.c_int64, vp]
    L.hc_set_log_wc.argtypes = [ctypes.c_int]
    L.hc_absl_uniform.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64, vp]
    L.hc_cpp_shuffle.argtypes = [ctypes.c_uint32, ctypes.c_int32, vp]
    L.hc_np_ops.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64, vp, vp,
                            vp]
    L.hc_mt_roundtrip.argtypes = [vp, vp, ctypes.c_int64, vp]
    _lib = L
  return _lib


KEYS = ("child_action", "child_n", "child_w", "child_out", "nchild", "root_n",
        "root_w", "root_out", "best_action", "nodes")


def mcts_batch(game_string, acts, offs, bot_seeds, eval_seeds, max_children,
               uct_c=2.0, max_simulations=1000, n_rollouts=1, max_memory_mb=1000,
               solve=True, policy=0, puct=False):
  R = len(offs) - 1
  mc = max_children
  o = dict(child_action=np.zeros((R, mc), np.int32),
           child_n=np.zeros((R, mc), np.int32),
           child_w=np.zeros((R, mc), np.float64),
           child_out=np.zeros((R, mc), np.int8),
           nchild=np.zeros(R, np.int32), root_n=np.zeros(R, np.int32),
           root_w=np.zeros(R, np.float64), root_out=np.zeros(R, np.int8),
           best_action=np.zeros(R, np.int64), nodes=np.zeros(R, np.int32))
  # padding convention of the C-ABI
  o["child_action"][:] = -1
  o["child_out"][:] = 2
  acts = np.ascontiguousarray(acts, np.int64)
  offs = np.ascontiguousarray(offs, np.int64)
  bs = np.ascontiguousarray(bot_seeds, np.uint32)
  es = np.ascontiguousarray(eval_seeds, np.uint32)
  rc = lib().hc_mcts_batch(game_string.encode(), R, acts.ctypes.data,
                           offs.ctypes.data, uct_c, max_simulations, n_rollouts,
                           max_memory_mb, int(solve), policy | (256 if puct else 0),
                           bs.ctypes.data,
                           es.ctypes.data, mc, *[o[k].ctypes.data for k in KEYS])
  if rc:
    raise RuntimeError(lib().hc_last_error().decode())
  return o


def rollouts(game_string, history, seeds):
  a = np.ascontiguousarray(history, np.int64)
  s = np.ascontiguousarray(seeds, np.uint32)
  out = np.zeros((len(s), 2), np.float64)
  rc = lib().hc_rollouts(game_string.encode(), a.ctypes.data, len(a), len(s),
                         s.ctypes.data, out.ctypes.data)
  if rc:
    raise RuntimeError(lib().hc_last_error().decode())
  return out


def go_score(game_string, history):
  a = np.ascontiguousarray(history, np.int64)
  return float(lib().hc_go_score(game_string.encode(), a.ctypes.data, len(a)))


def mt_words(seed, n):
  out = np.zeros(n, np.uint32)
  lib().hc_mt_words(seed, n, out.ctypes.data)
  return out


def mt_words_soa(seed, stride, n):
  out = np.zeros(n, np.uint32)
  lib().hc_mt_words_soa(seed, stride, n, out.ctypes.data)
  return out


def mt_words_reg(seed, stride, n):
  out = np.zeros(n, np.uint32)
  lib().hc_mt_words_reg(seed, stride, n, out.ctypes.data)
  return out


def mt_words_pf(seed, stride, n):
  out = np.zeros(n, np.uint32)
  lib().hc_mt_words_pf(seed, stride, n, out.ctypes.data)
  return out


def set_log_wc(on):
  """Searches keep the go superko log's open 8-entry group in a side buffer
  (GoCtxT::wlog, as k_lsearch does)."""
  lib().hc_set_log_wc(1 if on else 0)


def mt_words_wc(seed, stride, n):
  out = np.zeros(n, np.uint32)
  lib().hc_mt_words_wc(seed, stride, n, out.ctypes.data)
  return out


def absl_uniform(seed, n, k):
  out = np.zeros(k, np.uint64)
  lib().hc_absl_uniform(seed, n, k, out.ctypes.data)
  return out


def absl_double(seed, k):
  out = np.zeros(k, np.float64)
  lib().hc_absl_double(ctypes.c_uint32(seed), ctypes.c_int64(k), out.ctypes.data_as(ctypes.c_void_p))
  return out


def np_choice_p(seed, n, k):
  out = np.zeros(k, np.int32)
  lib().hc_np_choice_p(ctypes.c_uint32(seed), ctypes.c_int32(n), ctypes.c_int64(k),
                       out.ctypes.data_as(ctypes.c_void_p))
  return out


def cpp_shuffle(seed, n):
  out = np.zeros(n, np.int32)
  lib().hc_cpp_shuffle(seed, n, out.ctypes.data)
  return out


def np_ops(seed, n, k):
  ch = np.zeros(k, np.uint32)
  perm = np.zeros(n, np.int32)
  nw = np.zeros(1, np.uint32)
  lib().hc_np_ops(seed, n, k, ch.ctypes.data, perm.ctypes.data, nw.ctypes.data)
  return ch, perm, int(nw[0])


def mt_roundtrip(key, pos, k):
  key = np.array(key, dtype=np.uint32).copy()
  p = np.array([pos], dtype=np.int32)
  out = np.zeros(k, np.uint32)
  lib().hc_mt_roundtrip(key.ctypes.data, p.ctypes.data, k, out.ctypes.data)
  return out, key, int(p[0])


def mt_pf_roundtrip(key, pos, k):
  key = np.array(key, dtype=np.uint32).copy()
  p = np.array([pos], dtype=np.int32)
  out = np.zeros(k, np.uint32)
  lib().hc_mt_pf_roundtrip(key.ctypes.data, p.ctypes.data, k, out.ctypes.data)
  return out, key, int(p[0])


def mt_wc_roundtrip(key, pos, k):
  key = np.array(key, dtype=np.uint32).copy()
  p = np.array([pos], dtype=np.int32)
  out = np.zeros(k, np.uint32)
  lib().hc_mt_wc_roundtrip(key.ctypes.data, p.ctypes.data, k, out.ctypes.data)
  return out, key, int(p[0])


# int cb(const float* obs, int32 obs_size, const uint8* legal, int32 A, int32 kind,
#        double* prior, double* value)
AZ_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.c_int32,
                         ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32, ctypes.c_int32,
                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double))


def az_batch(game_string, acts, offs, bot_seeds, max_children, eval_fn, puct=True,
             uct_c=2.0, max_simulations=100, max_memory_mb=1000, solve=True,
             dirichlet_alpha=0.0, dirichlet_epsilon=0.0, fused=False):
  """csrc/os_az.h stepped on the host; eval_fn(obs float32[obs_size], legal
  bool[A], kind) -> (prior [A], value).  fused: one kind-3 request per
  simulation (OS_AZ_REQUESTS_FUSED); `calls` in the result counts requests."""
  L = lib()
  vp = ctypes.c_void_p
  L.hc_az_batch.argtypes = [ctypes.c_char_p, ctypes.c_int64, vp, vp, ctypes.c_double,
                            ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                            ctypes.c_double, ctypes.c_double,
                            vp, AZ_CB, ctypes.c_int32] + [vp] * 10
  R = len(offs) - 1
  mc = max_children
  o = dict(child_action=np.zeros((R, mc), np.int32), child_n=np.zeros((R, mc), np.int32),
           child_w=np.zeros((R, mc), np.float64), child_out=np.zeros((R, mc), np.int8),
           nchild=np.zeros(R, np.int32), root_n=np.zeros(R, np.int32),
           root_w=np.zeros(R, np.float64), root_out=np.zeros(R, np.int8),
           best_action=np.zeros(R, np.int64), nodes=np.zeros(R, np.int32))
  o["child_action"][:] = -1
  o["child_out"][:] = 2
  calls = [0]

  def cb(obs, obs_size, legal, A, kind, prior_out, value_out):
    ob = np.ctypeslib.as_array(obs, shape=(obs_size,)).copy()
    lg = np.ctypeslib.as_array(legal, shape=(A,)).astype(bool)
    calls[0] += 1
    pr, v = eval_fn(ob, lg, int(kind))
    for a in range(A):
      prior_out[a] = float(pr[a])
    value_out[0] = float(v)
    return 0

  fn = AZ_CB(cb)
  acts = np.ascontiguousarray(acts, np.int64)
  offs = np.ascontiguousarray(offs, np.int64)
  bs = np.ascontiguousarray(bot_seeds, np.uint32)
  rc = L.hc_az_batch(game_string.encode(), R, acts.ctypes.data, offs.ctypes.data, uct_c,
                     max_simulations, max_memory_mb, int(solve), int(puct) | (2 if fused else 0),
                     float(dirichlet_alpha), float(dirichlet_epsilon), bs.ctypes.data,
                     fn, mc, *[o[k].ctypes.data for k in KEYS])
  if rc:
    raise RuntimeError(L.hc_last_error().decode())
  o["calls"] = calls[0]
  return o


def rollouts_go_logbloom(game_string, history, seeds):
  """go playouts with the bucketed superko log behind GoCtxT's Bloom filter."""
  a = np.ascontiguousarray(history, np.int64)
  s = np.ascontiguousarray(seeds, np.uint32)
  out = np.zeros((len(s), 2), np.float64)
  rc = lib().hc_rollouts_go_logbloom(game_string.encode(), a.ctypes.data, len(a), len(s),
                                     s.ctypes.data, out.ctypes.data)
  if rc:
    raise RuntimeError(lib().hc_last_error().decode())
  return out


def rollouts_go_link16(game_string, history, seeds):
  """go playouts with k_rollouts' context: 16-bit links behind the Bloom filter."""
  a = np.ascontiguousarray(history, np.int64)
  s = np.ascontiguousarray(seeds, np.uint32)
  out = np.zeros((len(s), 2), np.float64)
  rc = lib().hc_rollouts_go_link16(game_string.encode(), a.ctypes.data, len(a), len(s),
                                   s.ctypes.data, out.ctypes.data)
  if rc:
    raise RuntimeError(lib().hc_last_error().decode())
  return out


def b96_selftest(seed, n):
  """Mismatches of B96 against B128 over n random boards (hc_b96_selftest)."""
  return int(lib().hc_b96_selftest(seed, n))


def rollouts_go9(game_string, history, seeds):
  """go playouts as k_rollouts<Go9> plays them (three-word bitboards, <= 9 x 9)."""
  a = np.ascontiguousarray(history, np.int64)
  s = np.ascontiguousarray(seeds, np.uint32)
  out = np.zeros((len(s), 2), np.float64)
  rc = lib().hc_rollouts_go9(game_string.encode(), a.ctypes.data, len(a), len(s),
                             s.ctypes.data, out.ctypes.data)
  if rc:
    raise RuntimeError(lib().hc_last_error().decode())
  return out


def rollouts_go_bloom(game_string, history, seeds):
  """go playouts with the k_rollouts superko screen (GoCtxBloom)."""
  a = np.ascontiguousarray(history, np.int64)
  s = np.ascontiguousarray(seeds, np.uint32)
  out = np.zeros((len(s), 2), np.float64)
  rc = lib().hc_rollouts_go_bloom(game_string.encode(), a.ctypes.data, len(a), len(s),
                                  s.ctypes.data, out.ctypes.data)
  if rc:
    raise RuntimeError(lib().hc_last_error().decode())
  return out


def az_numpy(game_string, history, key, pos, eval_fn, max_children, uct_c=2.0,
             max_simulations=100, solve=False, puct=True, noise=None, eps=0.0):
  """One python/algorithms/mcts.py search with an external evaluator on the
  host (csrc/os_az.h az_step, numpy policy): the bot RandomState continues
  from (key, pos); returns (root outputs, key', pos').  noise: the caller's
  RandomState.dirichlet draw for the root (legal order) or None."""
  L = lib()
  vp = ctypes.c_void_p
  L.hc_az_numpy.argtypes = [ctypes.c_char_p, vp, ctypes.c_int64, ctypes.c_double,
                            ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp,
                            ctypes.c_double, AZ_CB, ctypes.c_int32] + [vp] * 9
  mc = max_children
  o = dict(child_action=np.full(mc, -1, np.int32), child_n=np.zeros(mc, np.int32),
           child_w=np.zeros(mc, np.float64), child_prior=np.zeros(mc, np.float64),
           child_out=np.full(mc, 2, np.int8), nchild=np.zeros(1, np.int32),
           root_n=np.zeros(1, np.int32), root_w=np.zeros(1, np.float64),
           best_action=np.zeros(1, np.int64))

  def cb(obs, obs_size, legal, A, kind, prior_out, value_out):
    ob = np.ctypeslib.as_array(obs, shape=(obs_size,)).copy()
    lg = np.ctypeslib.as_array(legal, shape=(A,)).copy()
    pr, v = eval_fn(ob, lg, int(kind))
    for a in range(A):
      prior_out[a] = float(pr[a])
    value_out[0] = float(v)
    return 0

  fn = AZ_CB(cb)
  h = np.ascontiguousarray(history, np.int64)
  k = np.array(key, np.uint32).copy()
  p = np.array([pos], np.int32)
  nz = None if noise is None else np.ascontiguousarray(noise, np.float64)
  rc = L.hc_az_numpy(game_string.encode(), h.ctypes.data, len(h), uct_c, max_simulations,
                     int(solve), int(puct), k.ctypes.data, p.ctypes.data,
                     None if nz is None else nz.ctypes.data, float(eps), fn, mc,
                     *[o[x].ctypes.data for x in ("child_action", "child_n", "child_w",
                                                  "child_prior", "child_out", "nchild",
                                                  "root_n", "root_w", "best_action")])
  if rc:
    raise RuntimeError(L.hc_last_error().decode())
  return o, k, int(p[0])
