"""Product RNG primitives (csrc/os_rng.h, host-compiled) against libstdc++
(through the oracle) and the container's numpy legacy RandomState."""
import numpy as np
import pytest

import hostcheck_lib as H
import oracle_lib as O


@pytest.mark.parametrize("seed", [0, 1, 42, 5489, 2**32 - 1])
def test_mt_stream_matches_std_mt19937(seed):
  # Crosses several lazy in-place twists.
  assert np.array_equal(H.mt_words(seed, 3000), O.mt19937(seed, 3000))


@pytest.mark.parametrize("seed", [0, 1, 42, 5489, 2**32 - 1])
@pytest.mark.parametrize("stride", [1, 3, 64])
def test_soa_stream_matches_std_mt19937(seed, stride):
  # k_rollouts' stream: the seeded block comes from running cursors (first
  # block's reads of words i, i+1, i+397), the twisted words from memory.
  assert np.array_equal(H.mt_words_soa(seed, stride, 2000), O.mt19937(seed, 2000))


@pytest.mark.parametrize("seed", [0, 1, 42, 5489, 2**32 - 1])
@pytest.mark.parametrize("stride", [1, 3, 64])
def test_register_block0_stream_matches_std_mt19937(seed, stride):
  # k_rollouts' stream: block 0 from seed cursors alone (no memory), block 1+
  # in memory after block 0 is written out from the seed.
  for n in (1, 227, 228, 623, 624, 625, 2600):
    assert np.array_equal(H.mt_words_reg(seed, stride, n), O.mt19937(seed, n)), n


@pytest.mark.parametrize("seed", [0, 1, 42, 5489, 2**32 - 1])
@pytest.mark.parametrize("stride", [1, 3, 64])
def test_read_ahead_stream_matches_std_mt19937(seed, stride):
  # k_lsearch's stream: loads of the next word's twist inputs issued after
  # each draw; four blocks cover every wrap (word 623 reads the new s[0]).
  assert np.array_equal(H.mt_words_pf(seed, stride, 2600), O.mt19937(seed, 2600))


@pytest.mark.parametrize("seed", [0, 1, 42, 5489, 2**32 - 1])
@pytest.mark.parametrize("stride", [1, 3, 64])
def test_write_combined_stream_matches_std_mt19937(seed, stride):
  # k_lsearch's stream with its stores in 16-word groups (MtStreamWc): every
  # word it reads back as rewritten lies in a stored group.
  assert np.array_equal(H.mt_words_wc(seed, stride, 2600), O.mt19937(seed, 2600))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 8, 48, 82, 121, 768])
def test_absl_uniform_matches_oracle(n):
  for seed in (3, 99):
    assert np.array_equal(H.absl_uniform(seed, n, 500), O.absl_uniform(seed, n, 500))


@pytest.mark.parametrize("n", list(range(1, 40)) + [48, 82, 121, 122])
def test_cpp_shuffle_matches_libstdcxx(n):
  for seed in (1, 17, 123456):
    assert np.array_equal(H.cpp_shuffle(seed, n), O.std_shuffle(seed, n))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 9, 16, 17, 82, 121])
def test_numpy_choice_and_shuffle(n):
  for seed in (0, 42, 77):
    rs = np.random.RandomState(seed)
    ch = [rs.choice(list(range(n))) for _ in range(50)]
    lst = list(range(n))
    rs.shuffle(lst)
    nxt = int(rs.randint(0, 2**32, dtype=np.uint64))
    hch, hperm, hnext = H.np_ops(seed, n, 50)
    assert list(hch) == ch
    assert list(hperm) == lst
    assert hnext == nxt


@pytest.mark.parametrize("k", [0, 1, 100, 623, 624, 625, 1500])
def test_numpy_state_roundtrip(k):
  rs = np.random.RandomState(9)
  rs.randint(0, 2**32, size=37, dtype=np.uint64)  # mid-block position
  st = rs.get_state()
  out, key, pos = H.mt_roundtrip(st[1], st[2], k)
  ref = rs.randint(0, 2**32, size=k, dtype=np.uint64).astype(np.uint32)
  assert np.array_equal(out, ref)
  st2 = rs.get_state()
  assert pos == st2[2]
  assert np.array_equal(key, st2[1])


@pytest.mark.parametrize("skip", [0, 37, 600, 624])
@pytest.mark.parametrize("k", [0, 1, 100, 587, 588, 624, 625, 1500])
def test_read_ahead_stream_numpy_roundtrip(skip, k):
  # k_lsearch's imported bot streams (pyspiel.MCTSBot on go above 11 x 11).
  rs = np.random.RandomState(11)
  rs.randint(0, 2**32, size=skip, dtype=np.uint64)
  st = rs.get_state()
  out, key, pos = H.mt_pf_roundtrip(st[1], st[2], k)
  ref = rs.randint(0, 2**32, size=k, dtype=np.uint64).astype(np.uint32)
  assert np.array_equal(out, ref)
  st2 = rs.get_state()
  assert pos == st2[2]
  assert np.array_equal(key, st2[1])


@pytest.mark.parametrize("skip", [0, 37, 600, 624])
@pytest.mark.parametrize("k", [0, 1, 15, 16, 17, 100, 587, 588, 624, 625, 1500])
def test_write_combined_stream_numpy_roundtrip(skip, k):
  # MtStreamWc continuing an imported (key, pos) state and exporting it back,
  # a partly filled 16-word group included.
  rs = np.random.RandomState(11)
  rs.randint(0, 2**32, size=skip, dtype=np.uint64)
  st = rs.get_state()
  out, key, pos = H.mt_wc_roundtrip(st[1], st[2], k)
  ref = rs.randint(0, 2**32, size=k, dtype=np.uint64).astype(np.uint32)
  assert np.array_equal(out, ref)
  st2 = rs.get_state()
  assert pos == st2[2]
  assert np.array_equal(key, st2[1])


def _py_absl_double(words):
  """abseil 20200225 GenerateRealFromBits<double, GeneratePositiveTag, true>
  over FastUniformBits<uint64> (first word high), restated in Python."""
  import struct
  out = []
  for i in range(0, len(words) - 1, 2):
    bits = (int(words[i]) << 32) | int(words[i + 1])
    if bits == 0:
      out.append(0.0)
      continue
    clz = 64 - bits.bit_length()
    bits = (bits << clz) & (2**64 - 1)
    val = ((1022 - clz) << 52) | ((bits >> 11) & (2**52 - 1))
    out.append(struct.unpack("<d", struct.pack("<Q", val))[0])
  return out


@pytest.mark.parametrize("seed", [0, 1, 42])
def test_absl_uniform_double_matches_restatement(seed):
  got = H.absl_double(seed, 2000)
  want = _py_absl_double(O.mt19937(seed, 4000))
  assert got.tolist() == want
  assert (got >= 0).all() and (got < 1).all()
  hist = np.histogram(got, bins=10, range=(0, 1))[0]
  assert hist.min() > 150  # uniform over [0, 1)


@pytest.mark.parametrize("n", [1, 2, 4, 6, 7])
def test_numpy_choice_with_p_matches_numpy(n):
  for seed in (0, 5, 42):
    rs = np.random.RandomState(seed)
    want = [int(rs.choice(n, p=[1.0 / n] * n)) for _ in range(300)]
    assert H.np_choice_p(seed, n, 300).tolist() == want
