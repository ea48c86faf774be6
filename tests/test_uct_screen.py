"""Error bound behind the wave kernel's f32-screened UCT argmax
(csrc/os_wave.h uct_argmax_screen).

The kernel computes A = w * rcp(n) + c * sqrt(logN * rcp(n)) in f32, with the
hardware's 1-ulp v_rcp_f32 / v_sqrt_f32, and trusts the f32 argmax only when no
other child is within 8E of it, E = (1 + |c| sqrt(logN)) 2^-20.  That is exact
iff |A - V| <= E for the f64 value V of mcts.cc:89-100.  Here every f32 step is
emulated with its worst-case error pushed both ways (rcp and sqrt off by one
ulp up and down, each product / sum rounded to f32) over the count ranges the
engine sees, and the deviation is checked against E.
"""
import numpy as np
import pytest

F = np.float32


def _ulp_nudge(x, k):
  """x moved by k ulps (f32)."""
  x = np.asarray(x, F)
  for _ in range(abs(k)):
    x = np.nextafter(x, F(np.inf) if k > 0 else F(-np.inf))
  return x


def _screen_values(n, w, log_n, c, rcp_ulp, sqrt_ulp, log_ulp=0):
  r = _ulp_nudge(F(1.0) / n.astype(F), rcp_ulp)
  q = (w.astype(F) * r).astype(F)
  t = (_ulp_nudge(F(log_n), log_ulp) * r).astype(F)
  s = _ulp_nudge(np.sqrt(t).astype(F), sqrt_ulp)
  return (q + (F(c) * s).astype(F)).astype(F)


@pytest.mark.parametrize("c", [2.0, 1.0, 0.5, 10.0])
@pytest.mark.parametrize("parent", [1, 2, 3, 7, 100, 1023, 1024, 2048, 65535, 1 << 20])
def test_f32_screen_within_bound(c, parent):
  rng = np.random.default_rng(parent)
  n = np.concatenate([np.arange(1, min(parent, 4096) + 1),
                      rng.integers(1, parent + 1, 4096)]).astype(np.int64)
  n = n[n <= parent]
  w = np.concatenate([n, -n, np.zeros_like(n), rng.integers(-n, n + 1)])
  n = np.tile(n, 4)
  log_n = np.log(np.float64(parent))
  v = w / n + c * np.sqrt(log_n / n)  # f64, as mcts.cc
  e = (1.0 + abs(c) * np.sqrt(max(log_n, 0.0))) * 2.0 ** -20
  for ru in (-1, 0, 1):
    for su in (-1, 0, 1):
      # log(N) as rounded from the f64 table (0), or from v_log_f32 * ln 2
      # (OS_SCREEN_LOG: within 4 ulp, see test_log_f32_within_4_ulp)
      for lu in ((-4, 0, 4) if parent > 1 else (0,)):  # log2(1) = 0 exactly
        a = _screen_values(n, w, log_n, c, ru, su, lu).astype(np.float64)
        assert np.max(np.abs(a - v)) <= e


def _log_f32_model(n, log2_ulp, prod_round=True):
  """v_log_f32 (log2 within 1 ulp) times ln 2 rounded to f32."""
  l2 = _ulp_nudge(np.log2(n.astype(np.float64)).astype(F), log2_ulp)
  return (l2 * F(float.fromhex("0x1.62e430p-1"))).astype(F)


@pytest.mark.gpu
def test_device_log2_f32_within_model():
  # v_log_f32 on the device (torch.log2 of f32 lowers to it for normal inputs)
  # is within 1 ulp of log2 and exact at 1; with the ln 2 product, within 4 ulp
  # of log(N) -- the input error test_f32_screen_within_bound allows.
  import torch
  n = torch.arange(1, 1 << 20, dtype=torch.float32, device="cuda")
  l2 = torch.log2(n).cpu().numpy()
  nn = np.arange(1, 1 << 20, dtype=np.int64)
  exact2 = np.log2(nn.astype(np.float64))
  assert l2[0] == 0.0
  ulp2 = np.spacing(np.maximum(exact2, 1.0).astype(F)).astype(np.float64)
  assert np.max(np.abs(l2.astype(np.float64) - exact2) / ulp2) <= 1.0
  got = (l2 * F(float.fromhex("0x1.62e430p-1"))).astype(np.float64)[1:]
  exact = np.log(nn[1:].astype(np.float64))
  assert np.max(np.abs(got - exact) / np.spacing(exact.astype(F)).astype(np.float64)) <= 4.0


def test_log_f32_within_4_ulp():
  # The screen's log(N) under OS_SCREEN_LOG: 1 ulp of v_log_f32, the f32 ln 2
  # constant and the product's rounding stay within 4 ulp of log(N).
  n = np.arange(2, 1 << 20, dtype=np.int64)
  exact = np.log(n.astype(np.float64))
  for u in (-1, 0, 1):
    got = _log_f32_model(n, u).astype(np.float64)
    ulp = np.spacing(exact.astype(F)).astype(np.float64)
    assert np.max(np.abs(got - exact) / ulp) <= 4.0


def test_identical_children_give_identical_f32_values():
  # The screen accepts near ties only between children with equal (n, w, out):
  # their f32 values are bitwise equal, so the first lane holding the max is
  # also the lowest index among the f64 maxima.
  n = np.array([5, 5, 5], np.int64)
  w = np.array([2, 2, 2], np.int64)
  a = _screen_values(n, w, np.log(40.0), 2.0, 0, 0)
  assert a[0] == a[1] == a[2]


def _f32_key(a):
  """csrc/os_wave.h f32_key: b ^ ((b >> 31) & 0x7FFFFFFF) on the int32 bits."""
  b = np.asarray(a, F).view(np.int32)
  return b ^ ((b >> 31) & np.int32(0x7FFFFFFF))


def test_f32_key_orders_like_floats_and_decodes():
  # The screen's integer-key wave maximum (OS_SCREEN_LOG) relies on the key
  # being strictly monotone in the float value (non-NaN, -0 below +0) and on
  # the same map decoding it (key_f32).
  rng = np.random.default_rng(7)
  vals = np.concatenate([
      rng.standard_normal(20000).astype(F) * F(100),
      np.array([-np.inf, np.inf, 0.0, -0.0, 1e-45, -1e-45, 3.4e38, -3.4e38, 1.0, -1.0], F),
      (rng.random(2000).astype(F) - F(0.5)) * F(1e-38)])
  keys = _f32_key(vals)
  order_f = np.argsort(vals, kind="stable")
  sv, sk = vals[order_f], keys[order_f]
  neq = sv[1:] != sv[:-1]  # equal floats: only -0 / +0 here, whose keys differ
  assert np.all((np.diff(sk.astype(np.int64)) > 0)[neq])           # strictly monotone
  assert _f32_key(F(-0.0)) < _f32_key(F(0.0))
  assert _f32_key(keys.view(F)).view(np.int32).tolist() == vals.view(np.int32).tolist()
