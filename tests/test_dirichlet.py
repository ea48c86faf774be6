"""Dirichlet root noise (mcts.cc:177-192): the product's host-drawn noise
(csrc/os_host.cpp DirichletNoise, C-ABI os_dirichlet_noise) against an
independent pure-Python restatement of what the reference's call compiles to:
libstdc++ 11 std::gamma_distribution<double> (bits/random.tcc:2335-2392,
Marsaglia-Tsang) over normal_distribution (random.tcc:1800-1835, polar
method with one cached value) and generate_canonical<double, 53> (two 32-bit
words, first low), on std::mt19937(seed) == numpy MT19937 legacy seeding.
The libm calls (log, sqrt, pow) are CPython's math module, i.e. the same
glibc the C++ code calls, so the comparison is bit-exact.

No reference test holds Dirichlet vectors: this pins the
product against libstdc++'s published algorithm, not against reference output.
"""
import ctypes
import math

import numpy as np
import pytest

from os_amd import _lib


class _Mt:
  """std::mt19937(seed) words (numpy MT19937 with legacy seeding)."""

  def __init__(self, seed):
    self.bg = np.random.MT19937(0)
    self.bg._legacy_seeding(seed)
    self.words = 0

  def __call__(self):
    self.words += 1
    return int(self.bg.random_raw())


def _canonical(g):
  s = float(g())
  s += float(g()) * 4294967296.0
  r = s / 18446744073709551616.0
  return math.nextafter(1.0, 0.0) if r >= 1.0 else r


class _Normal:
  def __init__(self):
    self.saved = None

  def __call__(self, g):
    if self.saved is not None:
      v, self.saved = self.saved, None
      return v
    while True:
      x = 2.0 * _canonical(g) - 1.0
      y = 2.0 * _canonical(g) - 1.0
      r2 = x * x + y * y
      if not (r2 > 1.0 or r2 == 0.0):
        break
    mult = math.sqrt(-2 * math.log(r2) / r2)
    self.saved = x * mult
    return y * mult


def _gamma(alpha, nd, g):
  malpha = alpha + 1.0 if alpha < 1.0 else alpha
  a1 = malpha - 1.0 / 3.0
  a2 = 1.0 / math.sqrt(9.0 * a1)
  while True:
    while True:
      n = nd(g)
      v = 1.0 + a2 * n
      if not v <= 0.0:
        break
    v = v * v * v
    u = _canonical(g)
    if not (u > 1.0 - 0.0331 * n * n * n * n and
            math.log(u) > 0.5 * n * n + a1 * (1.0 - v + math.log(v))):
      break
  if alpha == malpha:
    return a1 * v * 1.0
  while True:
    u = _canonical(g)
    if u != 0.0:
      break
  return math.pow(u, 1.0 / alpha) * a1 * v * 1.0


def py_dirichlet(seed, count, alpha):
  g = _Mt(seed)
  nd = _Normal()
  noise = [_gamma(alpha, nd, g) for _ in range(count)]
  total = 0.0
  for v in noise:
    total += v
  return [v / total for v in noise], g.words


@pytest.mark.parametrize("alpha", [0.03, 0.3, 1.0, 2.5])
@pytest.mark.parametrize("count", [1, 7, 82, 121, 362])  # 362: past the first 624 words
def test_noise_matches_libstdcxx_restatement(alpha, count):
  for seed in (0, 1, 42, 12345):
    want, words = py_dirichlet(seed, count, alpha)
    got = np.zeros(count, np.float64)
    w = _lib.lib.os_dirichlet_noise(seed, count, alpha, _lib.ptr(got))
    assert w == words, (seed, count, alpha)
    np.testing.assert_array_equal(got, np.array(want))
    assert abs(got.sum() - 1.0) < 1e-12


def test_bad_alpha_is_an_error():
  out = np.zeros(3, np.float64)
  assert _lib.lib.os_dirichlet_noise(1, 3, 0.0, _lib.ptr(out)) < 0
