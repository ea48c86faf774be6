"""Paged search arena (include/os_mcts.h os_engine_set_arena_mode).

The reserved arena gives every root the worst case 1 + sims x max_children
nodes.  In paged mode, once a fetched run has shown how many nodes the
searches take, later batches of the same shape share one pool of pages; a
batch that still runs out of pages is rerun on the reserved arena inside the
fetch.  Either way the searches must be the oracle's, bit for bit.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def E(require_gpu):
  from os_amd import engine
  return engine


def _batch(E, gs, R, sims, plies, seed=1000):
  acts, offs = E.make_roots(gs, R, seed, plies)
  bs = np.arange(R, dtype=np.uint32) + np.uint32(seed)
  return acts, offs, bs, bs + np.uint32(1 << 20)


def _run(eng, batch, sims, **params):
  acts, offs, bs, es = batch
  eng.prepare(acts, offs, bs, es, uct_c=2.0, max_simulations=sims, **params)
  eng.run_async()
  return eng.fetch(), eng.arena_info()


def _check_oracle(E, gs, eng, out, batch, sims, roots=16, puct=False):
  acts, offs, bs, es = batch
  ref = O.Game(gs).mcts_batch(acts[:offs[roots]], offs[:roots + 1], bs[:roots], es[:roots],
                              uct_c=2.0, max_simulations=sims,
                              max_children=eng.max_children, threads=8, puct=puct)
  bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(out[k][:roots], ref[k])]
  assert not bad, bad


@pytest.mark.parametrize("gs,R,sims,plies", [("connect_four", 256, 400, 6),
                                             ("breakthrough", 128, 200, 4),
                                             ("hex(board_size=7)", 96, 300, 4)])
def test_paged_equals_reserved(E, gs, R, sims, plies):
  eng = E.Engine(gs)
  eng.set_arena_mode("paged")
  batch = _batch(E, gs, R, sims, plies)
  ref, info0 = _run(eng, batch, sims)       # no hint yet: reserved
  assert info0["paged"] == 0
  got, info = _run(eng, batch, sims)        # same shape: the pool
  assert info["paged"] == 1 and info["reruns"] == 0
  assert info["arena_bytes"] < info["reserved_bytes"]
  assert info["pages_used"] <= info["pool_pages_or_chunk_roots"]
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
  _check_oracle(E, gs, eng, got, batch, sims)
  # Tree export walks the pages and renumbers: the reserved arena's arrays.
  eng2 = E.Engine(gs)
  _run(eng2, batch, sims)
  for r in (0, R // 2, R - 1):
    a, b = eng.tree(r), eng2.tree(r)
    for k in a:
      np.testing.assert_array_equal(a[k], b[k], err_msg="root %d %s" % (r, k))


def test_pool_overflow_reruns_reserved(E):
  gs, R, sims = "connect_four", 128, 400
  eng = E.Engine(gs)
  eng.set_arena_mode("paged")
  # Player 0 wins at once in column 0: the solver proves these roots within a
  # few simulations, so the hint is about no pages beyond the roots' own.
  acts, offs = E.roots_from_histories([[0, 1, 0, 1, 0, 1]] * R)
  bs = np.arange(R, dtype=np.uint32)
  late = (acts, offs, bs, bs + np.uint32(1 << 20))
  _run(eng, late, sims)
  assert _run(eng, late, sims)[1]["paged"] == 1
  early = _batch(E, gs, R, sims, 0, seed=5000)  # opening roots: far bigger trees
  got, info = _run(eng, early, sims)
  assert info["reruns"] == 1 and info["overflowed_searches"] > 0
  assert info["paged"] == 0  # the rerun's reserved arena
  _check_oracle(E, gs, eng, got, early, sims)
  # The hint now covers the big trees: the next batch fits the pool.
  got2, info2 = _run(eng, early, sims)
  assert info2["paged"] == 1 and info2["reruns"] == 1
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got2[k], got[k], err_msg=k)


def test_reserved_is_default_and_small_batches_stay_reserved(E):
  eng = E.Engine("tic_tac_toe")
  batch = _batch(E, "tic_tac_toe", 128, 200, 2)
  _run(eng, batch, 200)
  assert _run(eng, batch, 200)[1]["paged"] == 0  # arena_mode defaults to reserved
  eng.set_arena_mode("paged")
  small = _batch(E, "tic_tac_toe", 16, 200, 2)
  _run(eng, small, 200)
  assert _run(eng, small, 200)[1]["paged"] == 0  # < 64 roots
  with pytest.raises(ValueError):
    eng.set_arena_mode("heap")


def test_root_sums_after_pool_overflow(E):
  """a paged root-parallel batch that runs out of pool pages is
  rerun on the reserved arena inside the fetch; the action-indexed sums that
  feed the all-reduce (dist.HipBackend.root_sums, C-ABI os_root_parallel) must
  then be those of the rerun, i.e. of the full searches."""
  from os_amd import dist
  gs, T, sims = "connect_four", 128, 400
  be = dist.HipBackend(gs, 0)
  be.eng.set_arena_mode("paged")
  ids = np.arange(T, dtype=np.uint32)
  es = ids + np.uint32(1 << 20)
  late = np.array([0, 1, 0, 1, 0, 1], np.int64)  # solved in a few sims: tiny hint
  be.root_sums(late, ids, es, uct_c=2.0, max_simulations=sims)
  be.root_sums(late, ids, es, uct_c=2.0, max_simulations=sims)
  assert be.eng.arena_info()["paged"] == 1
  v, w = be.root_sums(np.zeros(0, np.int64), ids, es, uct_c=2.0, max_simulations=sims)
  info = be.eng.arena_info()
  assert info["reruns"] == 1 and info["overflowed_searches"] > 0
  out = be.eng.fetch()
  want = E.action_indexed_visits(out, 7).sum(axis=0)
  assert np.array_equal(v.cpu().numpy(), want)
  assert int(want.sum()) == int((out["root_n"] - 1).sum())
  ref = O.Game(gs).mcts_batch(np.zeros(0, np.int64), np.array([0, 0]), ids[:1], es[:1],
                              uct_c=2.0, max_simulations=sims, max_children=7)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(out[k][:1], ref[k], err_msg=k)
  # The single-process C-ABI driver on a fresh engine: hint from the late
  # position only, then the opening overflows and is rerun there too.
  eng = E.Engine(gs)
  eng.set_arena_mode("paged")
  for _ in range(2):
    E.root_parallel([eng], late, T, uct_c=2.0, max_simulations=sims)
    eng.fetch()  # records the hint (os_root_parallel does not fetch)
  assert eng.arena_info()["paged"] == 1
  vis, rew, s = E.root_parallel([eng], np.zeros(0, np.int64), T, uct_c=2.0,
                                max_simulations=sims)
  assert eng.arena_info()["reruns"] == 1
  assert np.array_equal(vis, want) and s == int(out["root_n"].sum())
  np.testing.assert_array_equal(rew, w.cpu().numpy())


# The lane layouts' searches (os_mcts.h mcts_search, os_chance.h) take pages
# per lane: k_lsearch for go (narrow nodes at 9 x 9, wide above 11 x 11) and
# hex above 11 x 11, k_mcts for the rest (pig's chance search included), under
# UCT and PUCT.  sims is chosen so that two pages fit the worst case.
@pytest.mark.parametrize("gs,R,sims,plies,puct", [
    ("go(board_size=9)", 64, 256, 4, False),
    ("go(board_size=9)", 64, 256, 4, True),
    ("go(board_size=13)", 64, 256, 4, False),
    ("hex(board_size=13)", 64, 256, 4, False),
    ("connect_four", 128, 400, 6, False),
    ("pig", 64, 256, 0, False),
])
def test_lane_layout_paged_equals_reserved(E, gs, R, sims, plies, puct):
  from os_amd import _lib
  kw = dict(layout=_lib.LAYOUT_LANE,
            child_selection=_lib.SELECT_PUCT if puct else _lib.SELECT_UCT)
  eng = E.Engine(gs)
  eng.set_arena_mode("paged")
  batch = _batch(E, gs, R, sims, plies)
  ref, info0 = _run(eng, batch, sims, **kw)
  assert info0["paged"] == 0
  got, info = _run(eng, batch, sims, **kw)
  assert info["paged"] == 1 and info["reruns"] == 0
  assert info["arena_bytes"] < info["reserved_bytes"]
  assert info["pages_used"] <= info["pool_pages_or_chunk_roots"]
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
  _check_oracle(E, gs, eng, got, batch, sims, roots=8, puct=puct)
  eng2 = E.Engine(gs)
  _run(eng2, batch, sims, **kw)
  for r in (0, R - 1):
    a, b = eng.tree(r), eng2.tree(r)
    for k in a:
      np.testing.assert_array_equal(a[k], b[k], err_msg="root %d %s" % (r, k))


def test_lane_layout_pool_overflow_reruns_reserved(E):
  from os_amd import _lib
  gs, R, sims = "connect_four", 128, 400
  eng = E.Engine(gs)
  eng.set_arena_mode("paged")
  acts, offs = E.roots_from_histories([[0, 1, 0, 1, 0, 1]] * R)
  bs = np.arange(R, dtype=np.uint32)
  late = (acts, offs, bs, bs + np.uint32(1 << 20))
  _run(eng, late, sims, layout=_lib.LAYOUT_LANE)
  assert _run(eng, late, sims, layout=_lib.LAYOUT_LANE)[1]["paged"] == 1
  early = _batch(E, gs, R, sims, 0, seed=5000)
  got, info = _run(eng, early, sims, layout=_lib.LAYOUT_LANE)
  assert info["reruns"] == 1 and info["overflowed_searches"] > 0
  _check_oracle(E, gs, eng, got, early, sims)
