"""The search engine the gfx950 kernel runs (csrc/os_mcts.h), compiled for
the host, against the oracle: every output field bit-exact on seeded random
roots for all five games, both RNG policies, int and f64 rewards, solver on
and off, and the garbage-collection path."""
import numpy as np
import pytest

import hostcheck_lib as H
import oracle_lib as O
from os_amd import engine as E

CASES = [
    # game string, roots, sims, root plies
    ("tic_tac_toe", 24, 600, 4),
    ("connect_four", 24, 512, 8),
    ("breakthrough", 6, 256, 6),
    ("breakthrough(rows=6,columns=5)", 6, 256, 6),
    ("hex(board_size=5)", 8, 300, 6),
    ("hex", 3, 200, 4),
    ("go(board_size=7,komi=4.5)", 3, 120, 6),
    ("go(board_size=9)", 2, 96, 8),
]


def _roots(gs, R, plies, seed_base=1000):
  return E.make_roots(gs, R, seed_base, plies)


def _check(a, b):
  bad = [k for k in H.KEYS if not np.array_equal(a[k], b[k])]
  assert not bad, bad


@pytest.mark.parametrize("gs,R,sims,plies", CASES)
def test_cpp_policy_matches_oracle(gs, R, sims, plies):
  acts, offs = _roots(gs, R, plies)
  bs = np.arange(R, dtype=np.uint32) + 7
  es = bs + np.uint32(1 << 20)
  og = O.Game(gs)
  from os_amd import pyspiel
  maxc = pyspiel.load_game(gs)._info.max_children
  ref = og.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                      max_children=maxc)
  got = H.mcts_batch(gs, acts, offs, bs, es, maxc, uct_c=2.0, max_simulations=sims)
  _check(got, ref)


@pytest.mark.parametrize("gs", ["tic_tac_toe", "connect_four", "hex(board_size=5)",
                                "go(board_size=5,komi=0.5)"])
@pytest.mark.parametrize("n_rollouts,solve,uct_c", [(3, True, 1.4142135623730951),
                                                    (1, False, 2.0), (2, False, 0.5)])
def test_rollout_count_solver_and_uct_variants(gs, n_rollouts, solve, uct_c):
  from os_amd import pyspiel
  maxc = pyspiel.load_game(gs)._info.max_children
  acts, offs = _roots(gs, 8, 4)
  bs = np.arange(8, dtype=np.uint32) * 3 + 1
  es = bs + np.uint32(99)
  kw = dict(uct_c=uct_c, max_simulations=300, n_rollouts=n_rollouts, solve=solve)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=maxc, **kw)
  got = H.mcts_batch(gs, acts, offs, bs, es, maxc, **kw)
  _check(got, ref)


@pytest.mark.parametrize("gs,R,plies", [("go(board_size=5,komi=0.5)", 8, 4),
                                        ("go(board_size=7,komi=4.5)", 6, 6),
                                        ("go(board_size=9)", 4, 8)])
@pytest.mark.parametrize("n_rollouts", [1, 3])
def test_write_combined_go_log_matches_oracle(gs, R, plies, n_rollouts):
  """k_lsearch's superko log with its open 8-entry group in LDS
  (GoCtxT::wlog): lookups, inserts, group write-outs and the rewinds of
  several rollouts per leaf give the oracle's trees."""
  from os_amd import pyspiel
  maxc = pyspiel.load_game(gs)._info.max_children
  acts, offs = _roots(gs, R, plies)
  bs = np.arange(R, dtype=np.uint32) * 5 + 2
  es = bs + np.uint32(77)
  kw = dict(uct_c=2.0, max_simulations=160, n_rollouts=n_rollouts)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=maxc, **kw)
  H.set_log_wc(True)
  try:
    got = H.mcts_batch(gs, acts, offs, bs, es, maxc, **kw)
  finally:
    H.set_log_wc(False)
  _check(got, ref)


@pytest.mark.parametrize("gs,sims", [("go(board_size=9)", 700), ("hex", 2200)])
def test_garbage_collection_path(gs, sims):
  """max_memory_mb=1 -> max_nodes_ = 13108: GC fires (mcts.cc:402-424)."""
  from os_amd import pyspiel
  maxc = pyspiel.load_game(gs)._info.max_children
  acts, offs = np.zeros(0, np.int64), np.array([0, 0], np.int64)
  kw = dict(uct_c=2.0, max_simulations=sims, max_memory_mb=1)
  ref = O.Game(gs).mcts_batch(acts, offs, [5], [6], max_children=maxc, **kw)
  got = H.mcts_batch(gs, acts, offs, [5], [6], maxc, **kw)
  _check(got, ref)
  assert ref["nodes"][0] < 13108 + maxc  # GC did bring the tree down


@pytest.mark.parametrize("gs", ["tic_tac_toe", "connect_four", "hex(board_size=5)",
                                "go(board_size=5)"])
def test_numpy_policy_matches_oracle(gs):
  from os_amd import pyspiel
  maxc = pyspiel.load_game(gs)._info.max_children
  for seed in (0, 42, 1234):
    # One shared RandomState (mcts_test.py:41-54): oracle vs the Python host
    # loop running on the product State API with the real numpy.
    ref = O.Game(gs).mcts_numpy([], seed, uct_c=2.0, max_simulations=400)
    nc = ref["nchild"][0]
    assert sorted(zip(ref["child_action"][0][:nc].tolist(),
                      ref["child_n"][0][:nc].tolist(),
                      ref["child_w"][0][:nc].tolist())) == _python_host_search(
                          gs, seed, seed, 400)
    # Two separate RandomStates: the engine's numpy policy vs the host loop.
    got = H.mcts_batch(gs, np.zeros(0, np.int64), np.array([0, 0]), [seed],
                       [seed + 1], maxc, uct_c=2.0, max_simulations=400, policy=1)
    nc = got["nchild"][0]
    assert sorted(zip(got["child_action"][0][:nc].tolist(),
                      got["child_n"][0][:nc].tolist(),
                      got["child_w"][0][:nc].tolist())) == _python_host_search(
                          gs, seed, seed + 1, 400)


def _python_host_search(gs, bot_seed, eval_seed, sims):
  from os_amd import mcts, pyspiel
  game = pyspiel.load_game(gs)
  brs = np.random.RandomState(bot_seed)
  ers = brs if eval_seed == bot_seed else np.random.RandomState(eval_seed)
  bot = mcts.MCTSBot(game, 2.0, sims, mcts.RandomRolloutEvaluator(1, ers),
                     random_state=brs, backend="host")
  root = bot.mcts_search(game.new_initial_state())
  return sorted((c.action, c.explore_count, float(c.total_reward))
                for c in root.children)


@pytest.mark.parametrize("gs,plies", [("connect_four", 10), ("breakthrough", 20),
                                      ("hex", 30), ("go(board_size=9)", 40)])
def test_rollouts_match_oracle(gs, plies):
  acts, offs = _roots(gs, 1, plies, seed_base=77)
  seeds = np.arange(64, dtype=np.uint32) * 13 + 5
  ref = O.Game(gs).rollouts(acts, seeds)
  got = H.rollouts(gs, acts, seeds)
  assert np.array_equal(got, ref)


@pytest.mark.parametrize("gs", ["go(board_size=5,komi=0.5)", "go(board_size=7,komi=4.5)",
                                "go(board_size=9)", "go(board_size=11)"])
def test_go_playouts_match_oracle_many_seeds(gs):
  """GoT::apply's atari set (os_games.h, lazy chain floods) decides legality in
  every playout move: 1500 full random games per board from the empty board
  and from a mid-game position equal the oracle's go_board.cc restatement."""
  for plies in (0, 30):
    acts, offs = _roots(gs, 1, plies, seed_base=11)
    seeds = np.arange(1500, dtype=np.uint32) * 7 + 3
    ref = O.Game(gs).rollouts(acts, seeds)
    assert np.array_equal(H.rollouts(gs, acts, seeds), ref)
    # k_rollouts' Bloom-screened superko set gives the same playouts
    assert np.array_equal(H.rollouts_go_bloom(gs, acts, seeds), ref)
    assert np.array_equal(H.rollouts_go_logbloom(gs, acts, seeds), ref)
    assert np.array_equal(H.rollouts_go_link16(gs, acts, seeds), ref)
    if "board_size=11" not in gs:  # three-word bitboards (Go9) up to 9 x 9
      assert np.array_equal(H.rollouts_go9(gs, acts, seeds), ref)


@pytest.mark.parametrize("gs", ["go(board_size=9)", "go(board_size=7,komi=4.5)",
                                "go(board_size=11)"])
def test_go_tromp_taylor_score_matches_oracle(gs):
  """Go::score (regions by flood, the reference's early-abort DFS replayed
  only on regions bordering both colours) == the oracle's recursive DFS
  (go_board.cc:526-597) on every prefix of random games: mid-game boards have
  the large mixed regions where the abort quirk changes the count."""
  from os_amd import pyspiel
  og = O.Game(gs)
  game = pyspiel.load_game(gs)
  rng = np.random.RandomState(5)
  checked = 0
  for _ in range(12):
    st = game.new_initial_state()
    hist = []
    while not st.is_terminal():
      a = int(rng.choice(st.legal_actions()))
      st.apply_action(a)
      hist.append(a)
      if len(hist) % 3 == 0 or st.is_terminal():
        assert H.go_score(gs, hist) == og.go_score(hist), hist
        checked += 1
  assert checked > 300


# ChildSelectionPolicy::PUCT with the random-rollout evaluator's uniform prior
# (mcts.cc:102-111, mcts.py:135-142): both RNG policies, pig's chance search.
@pytest.mark.parametrize("gs", ["tic_tac_toe", "connect_four", "breakthrough(rows=5,columns=5)",
                                "hex(board_size=5)", "go(board_size=5,komi=0.5)",
                                "pig(horizon=30,winscore=10)"])
@pytest.mark.parametrize("uct_c,solve,nr", [(2.0, True, 1), (0.5, False, 2)])
def test_puct_matches_oracle(gs, uct_c, solve, nr):
  from os_amd import pyspiel
  maxc = pyspiel.load_game(gs)._info.max_children
  acts, offs = _roots(gs, 8, 4)
  bs = np.arange(8, dtype=np.uint32) * 5 + 2
  es = bs + np.uint32(1 << 20)
  kw = dict(uct_c=uct_c, max_simulations=300, n_rollouts=nr, solve=solve)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=maxc, puct=True, **kw)
  got = H.mcts_batch(gs, acts, offs, bs, es, maxc, puct=True, **kw)
  _check(got, ref)
  uct = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=maxc, **kw)
  assert not all(np.array_equal(uct[k], ref[k]) for k in H.KEYS)  # PUCT is not UCT


def test_b96_matches_b128_on_random_boards():
  """Go9's three-word bitboards (os_common.h B96) give B128's result for every
  operation GoT uses, on 200000 random boards of up to 96 cells (sparse to
  dense), shifts 1..31, every cell index."""
  assert H.b96_selftest(12345, 200000) == 0
