"""Self-play driver: two MCTSBots sharing one
RandomRolloutEvaluator play whole games (examples/mcts_example.cc PlayGame).

CPU tests pin the oracle's self-play against the oracle's own single-search
path (every move of a game == one MCTSearch from that position with the bot
and evaluator streams advanced by all earlier moves) and against the game
rules; GPU tests check the device driver bit-exact against the oracle:
actions, lengths, returns and per-move action-indexed root visit counts.
"""
import numpy as np
import pytest

import oracle_lib
from os_amd import engine as E

STARTS = {  # game -> list of start histories
    "tic_tac_toe": [[], [4], [0, 4], []],
    "connect_four": [[], [3, 3], [], [0, 1, 2]],
    "breakthrough(rows=6,columns=6)": [[], []],
    "hex(board_size=5)": [[], [12], []],
    "go(board_size=5,komi=0.5)": [[], [12]],
}
SIMS = {"tic_tac_toe": 60, "connect_four": 48, "breakthrough(rows=6,columns=6)": 24,
        "hex(board_size=5)": 32, "go(board_size=5,komi=0.5)": 24}


def _batch(game):
  hs = STARTS[game]
  acts, offs = E.roots_from_histories(hs)
  G = len(hs)
  bot = np.arange(2 * G, dtype=np.uint32).reshape(G, 2) * 7 + 3
  ev = np.arange(G, dtype=np.uint32) + 1000
  return acts, offs, bot, ev


@pytest.mark.parametrize("game", sorted(STARTS))
def test_oracle_selfplay_games_are_legal_and_scored(game):
  og = oracle_lib.Game(game)
  acts, offs, bot, ev = _batch(game)
  o = og.selfplay(acts, offs, bot, ev, og.max_game_length, max_simulations=SIMS[game])
  for g in range(len(offs) - 1):
    hist = list(acts[offs[g]:offs[g + 1]])
    n = int(o["length"][g])
    for m in range(n):
      info = og.state_info(hist)
      a = int(o["actions"][g, m])
      assert a in info["legal_actions"]
      v = o["visits"][g, m]
      assert v[a] > 0 and (v >= 0).all()
      assert set(np.nonzero(v)[0]) <= set(info["legal_actions"])
      hist.append(a)
    assert (o["actions"][g, n:] == -1).all()
    info = og.state_info(hist)
    assert info["is_terminal"]
    assert list(o["returns"][g]) == list(info["returns"])


def test_oracle_selfplay_first_move_is_one_search():
  # Move 0 of a game == MCTSBot(seed b0) + evaluator(seed e) searching the start.
  og = oracle_lib.Game("connect_four")
  acts, offs, bot, ev = _batch("connect_four")
  o = og.selfplay(acts, offs, bot, ev, 42, max_simulations=48)
  ref = og.mcts_batch(acts, offs, bot[:, 0].copy(), ev, max_simulations=48,
                      max_children=7)
  for g in range(len(offs) - 1):
    # player to move at the start picks bot 0 or 1
    p = len(acts[offs[g]:offs[g + 1]]) % 2
    if p == 0:
      assert o["actions"][g, 0] == ref["best_action"][g]
      v = np.zeros(7, np.int32)
      for k in range(ref["nchild"][g]):
        v[ref["child_action"][g, k]] = ref["child_n"][g, k]
      np.testing.assert_array_equal(o["visits"][g, 0], v)


@pytest.mark.gpu
@pytest.mark.parametrize("game", sorted(STARTS))
def test_gpu_selfplay_matches_oracle(require_gpu, game):
  og = oracle_lib.Game(game)
  acts, offs, bot, ev = _batch(game)
  L = og.max_game_length
  ref = og.selfplay(acts, offs, bot, ev, L, max_simulations=SIMS[game])
  eng = E.Engine(game)
  out = eng.selfplay(acts, offs, bot, ev, max_len=L, max_simulations=SIMS[game])
  for k in ("actions", "length", "returns", "visits"):
    np.testing.assert_array_equal(out[k], ref[k], err_msg=k)


@pytest.mark.gpu
def test_gpu_selfplay_many_games_no_visits(require_gpu):
  game = "connect_four"
  G = 96
  acts, offs = E.make_roots(game, G, seed_base=77, max_plies=4)
  bot = np.arange(2 * G, dtype=np.uint32).reshape(G, 2)
  ev = np.arange(G, dtype=np.uint32) + 5
  eng = E.Engine(game)
  out = eng.selfplay(acts, offs, bot, ev, max_len=42, record_visits=False,
                     max_simulations=32)
  ref = oracle_lib.Game(game).selfplay(acts, offs, bot, ev, 42, max_simulations=32,
                                       with_visits=False, threads=8)
  for k in ("actions", "length", "returns"):
    np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
  assert out["visits"] is None


@pytest.mark.gpu
@pytest.mark.parametrize("game", ["connect_four", "hex(board_size=5)",
                                  "go(board_size=5,komi=0.5)"])
def test_gpu_selfplay_observations_match_host_state(require_gpu, game):
  from os_amd import pyspiel
  acts, offs, bot, ev = _batch(game)
  eng = E.Engine(game)
  out = eng.selfplay(acts, offs, bot, ev, record_observations=True,
                     max_simulations=SIMS[game])
  g = pyspiel.load_game(game)
  obs = out["observations"]
  assert obs.shape[2:] == tuple(g.observation_tensor_shape())
  for gi in range(len(offs) - 1):
    st = g.new_initial_state()
    for a in acts[offs[gi]:offs[gi + 1]]:
      st.apply_action(int(a))
    n = int(out["length"][gi])
    for m in range(n):
      want = np.array(st.observation_tensor(st.current_player()), np.float32)
      np.testing.assert_array_equal(obs[gi, m].reshape(-1), want)
      st.apply_action(int(out["actions"][gi, m]))
    assert st.is_terminal()
    assert not obs[gi, n:].any()


@pytest.mark.gpu
def test_gpu_selfplay_errors(require_gpu):
  from os_amd import _lib
  eng = E.Engine("tic_tac_toe")
  acts, offs = E.roots_from_histories([[]])
  with pytest.raises(ValueError):
    eng.selfplay(acts, offs, [[1, 2]], [3], policy=_lib.POLICY_NUMPY, max_simulations=10)
  with pytest.raises(_lib.SpielError):
    eng.selfplay(acts, offs, [[1, 2]], [3], max_len=2, max_simulations=10)


# ---- AlphaZero's PlayGame move choice (alpha_zero.cc:64-118) -------------
AZ_CASES = [  # (game, temperature, drop, resign, puct)
    ("tic_tac_toe", 1.0, 4, False, False),
    ("connect_four", 0.5, 6, False, False),
    ("connect_four", 1.0, 10, True, False),
    ("hex(board_size=5)", 1.0, 8, True, True),
    ("breakthrough(rows=6,columns=6)", 0.7, 5, False, True),
    ("go(board_size=5,komi=0.5)", 1.0, 6, True, False),
]


def _az_kw(game, t, drop, resign, puct):
  return dict(uct_c=2.0, max_simulations=SIMS[game], puct=puct, temperature=t,
              temperature_drop=drop, resign=resign, cutoff_value=0.5, cutoff_probability=0.7)


def test_oracle_az_selfplay_without_sampling_is_plain_selfplay():
  """temperature <= 0 (or drop 0) and no resignation: the moves are BestChild,
  i.e. oref_selfplay's games; policies are normalised visit counts."""
  game = "connect_four"
  og = oracle_lib.Game(game)
  acts, offs, bot, ev = _batch(game)
  actor = np.arange(len(offs) - 1, dtype=np.uint32) + 77
  ref = og.selfplay(acts, offs, bot, ev, 42, max_simulations=SIMS[game])
  for t, drop in ((0.0, 10), (1.0, 0)):
    o = oracle_lib.selfplay_az(game, acts, offs, bot, ev, actor, 42, max_simulations=SIMS[game],
                               temperature=t, temperature_drop=drop)
    for k in ("actions", "length", "returns"):
      assert np.array_equal(o[k], ref[k]), (t, k)
    vis = ref["visits"].astype(np.float64)
    n = vis.sum(axis=2, keepdims=True)
    want = np.divide(vis, n, out=np.zeros_like(vis), where=n > 0)
    np.testing.assert_allclose(o["policy"], want, rtol=0, atol=1e-15)


@pytest.mark.parametrize("game,t,drop,resign,puct", AZ_CASES)
def test_oracle_az_selfplay_is_consistent(game, t, drop, resign, puct):
  og = oracle_lib.Game(game)
  acts, offs, bot, ev = _batch(game)
  G = len(offs) - 1
  actor = np.arange(G, dtype=np.uint32) * 13 + 5
  o = oracle_lib.selfplay_az(game, acts, offs, bot, ev, actor, og.max_game_length,
                             **_az_kw(game, t, drop, resign, puct))
  for g in range(G):
    hist = list(acts[offs[g]:offs[g + 1]])
    n = int(o["length"][g])
    for m in range(n):
      info = og.state_info(hist)
      a = int(o["actions"][g, m])
      assert a in info["legal_actions"] and o["policy"][g, m, a] > 0
      assert abs(o["policy"][g, m].sum() - 1) < 1e-12
      assert -1 <= o["root_value"][g, m] <= 1
      hist.append(a)
    info = og.state_info(hist)
    if not info["is_terminal"]:  # resigned: returns are the last root value
      v = o["root_value"][g, n - 1]
      assert resign and abs(v) > 0.5
      mover = og.state_info(hist[:-1])["current_player"]
      assert o["returns"][g, mover] == v and o["returns"][g, 1 - mover] == -v
    else:
      assert list(o["returns"][g]) == list(info["returns"])


@pytest.mark.gpu
@pytest.mark.parametrize("game,t,drop,resign,puct", AZ_CASES)
def test_gpu_az_selfplay_matches_oracle(require_gpu, game, t, drop, resign, puct):
  """k_wselfplay with AlphaZero's move choice: every action, length, return,
  policy target and root value bit-exact with the oracle's PlayGame."""
  from os_amd import _lib
  og = oracle_lib.Game(game)
  acts, offs, bot, ev = _batch(game)
  G = len(offs) - 1
  actor = np.arange(G, dtype=np.uint32) * 13 + 5
  kw = _az_kw(game, t, drop, resign, puct)
  ref = oracle_lib.selfplay_az(game, acts, offs, bot, ev, actor, og.max_game_length, **kw)
  eng = E.Engine(game)
  eng.selfplay_set_options(actor, temperature=t, temperature_drop=drop, resign=resign,
                           cutoff_value=kw["cutoff_value"],
                           cutoff_probability=kw["cutoff_probability"])
  got = eng.selfplay(acts, offs, bot, ev, og.max_game_length, record_visits=False,
                     record_policy=True, record_root_values=True, uct_c=2.0,
                     max_simulations=SIMS[game],
                     child_selection=_lib.SELECT_PUCT if puct else _lib.SELECT_UCT)
  for k in ("actions", "length", "returns", "policy", "root_value"):
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
