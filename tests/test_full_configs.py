"""BASELINE configs C4 and C5 at full width on the GPU.

C4: hex(board_size=11) root-parallel MCTS, 8192 trees on one position through
the automatic layout and the PAGED arena, with the action-indexed device
reduction (k_root_scatter / k_root_reduce) that feeds the RCCL all-reduce
(os_amd/dist.py).  Sims are reduced so the oracle can check a 16-tree prefix
bit-exactly; the device sums must equal the sums of every tree's fetched
children.

C5: go(board_size=9) 2^20 random playouts (RandomRolloutEvaluator::Evaluate,
mcts.cc:42-71): device outcome counts (k_outcome_counts, the all-reduced
quantity) must equal the counts of the fetched returns, and 4096 seeds spread
over the batch must equal the oracle's playouts.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev(require_gpu):
  import torch
  return torch


def test_full_c4_paged_root_parallel(torch_dev):
  torch = torch_dev
  from os_amd import dist
  from os_amd import engine as E
  gs, T, sims = "hex(board_size=11)", 8192, 256  # >= 2 pages of 8192 nodes: pageable
  be = dist.HipBackend(gs, 0)
  eng = be.eng
  eng.set_arena_mode("paged")
  hist = np.zeros(0, np.int64)
  ids = np.arange(T, dtype=np.uint32)
  es = ids + np.uint32(dist.EVAL_SEED_OFFSET)
  kw = dict(uct_c=2.0, max_simulations=sims)
  be.root_sums(hist, ids, es, **kw)            # reserved run: sizes the page pool
  assert eng.arena_info()["paged"] == 0
  v, w = be.root_sums(hist, ids, es, **kw)     # the C4 production path
  info = eng.arena_info()
  assert info["paged"] == 1 and info["reruns"] == 0
  assert info["arena_bytes"] < info["reserved_bytes"]
  out = eng.fetch()
  A = eng.num_distinct_actions
  want = E.action_indexed_visits(out, A).sum(axis=0)
  assert np.array_equal(v.cpu().numpy(), want)
  wr = np.zeros(A)
  for r in range(T):  # the reduction's fixed order: per action, trees ascending
    nc = out["nchild"][r]
    wr[out["child_action"][r, :nc]] += out["child_w"][r, :nc]
  np.testing.assert_allclose(w.cpu().numpy(), wr, rtol=0, atol=1e-9)
  assert int(v.sum()) == int((out["root_n"] - 1).sum())
  assert (out["nchild"] == 121).all()
  sub = 16
  acts, offs = E.roots_from_histories([[]] * sub)
  ref = O.Game(gs).mcts_batch(acts, offs, ids[:sub], es[:sub], max_children=eng.max_children,
                              threads=8, **kw)
  for k in E.OUTPUT_KEYS:
    assert np.array_equal(out[k][:sub], ref[k]), k
  ref_last = O.Game(gs).mcts_batch(acts[:0], offs[:2], ids[-1:], es[-1:],
                                   max_children=eng.max_children, **kw)
  for k in E.OUTPUT_KEYS:
    assert np.array_equal(out[k][-1:], ref_last[k]), k


def test_full_c5_million_go_playouts(torch_dev):
  torch = torch_dev
  from os_amd import dist
  gs, N = "go(board_size=9)", 1 << 20
  be = dist.HipBackend(gs, 0)
  hist = np.zeros(0, np.int64)
  seeds = np.arange(N, dtype=np.uint32)
  be.prepare_playouts(hist, seeds)
  counts = be.run_playouts().cpu().numpy()   # device k_outcome_counts
  ret = be.eng.rollouts_fetch()
  assert ret.shape == (N, 2) and np.array_equal(ret[:, 1], -ret[:, 0])
  host = [int((ret[:, 0] > 0).sum()), int((ret[:, 0] < 0).sum()), int((ret[:, 0] == 0).sum())]
  assert counts.tolist() == host and sum(host) == N
  assert host[0] > 0 and host[1] > 0          # komi 7.5: both colours win some
  pick = np.arange(0, N, N // 4096, dtype=np.int64)[:4096]
  ref = O.Game(gs).rollouts(hist, seeds[pick])
  assert np.array_equal(ret[pick], ref)
  stats = be.eng.rollouts_stats()
  assert stats["moves"] > 100 * N             # random go9 games run > 100 plies


def test_c3_prefix_full_depth(torch_dev):
  """C3: breakthrough 8x8 roots from the config's own generator
  (seed 1000 + i, k ~ U[0,6] plies) at the full 2048 simulations; the first
  and last 32 of the 65536 roots, bit-exact against the oracle
  (mcts.cc:325-428)."""
  from os_amd import engine as E
  gs, R, sims = "breakthrough(rows=8,columns=8)", 65536, 2048
  acts, offs = E.make_roots(gs, R, seed_base=1000, max_plies=6)
  rows = np.r_[0:32, R - 32:R]
  hist = [acts[offs[r]:offs[r + 1]] for r in rows]
  sa, so = E.roots_from_histories(hist)
  bs = rows.astype(np.uint32)
  es = bs + np.uint32(1 << 20)
  eng = E.Engine(gs, device=0)
  kw = dict(uct_c=2.0, max_simulations=sims)
  got = eng.mcts_batch(sa, so, bs, es, **kw)
  ref = O.Game(gs).mcts_batch(sa, so, bs, es, max_children=eng.max_children, threads=8, **kw)
  for k in E.OUTPUT_KEYS:
    assert np.array_equal(got[k], ref[k]), k
  assert (got["root_n"] > 1).all()
