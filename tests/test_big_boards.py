"""Hex and go above 11 x 11 (up to 19 x 19): the drop-in `load_game("go")`
(default board_size 19, go.cc:45) and `hex(board_size=13)` load, and their host
State API (os_games.h HexT / GoT on B384 bitboards) follows the oracle move by
move on random games (basic_tests.cc RandomSimTest shape: legal actions,
current player, terminal, returns at every state; serialization round trips).
The GPU engine runs hex and go up to 19 x 19 (above 11 x 11: C++-policy
searches on the lane layout, k_lsearch over B384 bitboards with wide nodes,
parity in test_gpu_big_board_search_matches_oracle); the Python MCTSBot
(numpy policy) searches boards above 11 x 11 with its host loop, warning once,
and refuses backend='hip' there."""
import numpy as np
import pytest

import oracle_lib as O
import pyspiel
from open_spiel.python.algorithms import mcts

BIG = ["go", "go(board_size=13)", "go(board_size=12,komi=0.5)", "hex(board_size=13)",
       "hex(board_size=19)", "hex(board_size=12)",
       # handicap stones (go.cc:56-78, 211-225): white moves first, score -= h
       "go(handicap=2)", "go(handicap=5,komi=0.5)", "go(board_size=16,handicap=9)",
       "go(handicap=12)"]


def test_default_go_is_19x19():
  g = pyspiel.load_game("go")
  assert g.get_parameters()["board_size"] == 19
  assert g.num_distinct_actions() == 362 and g.max_game_length() == 722
  assert g.observation_tensor_shape() == [4, 19, 19]
  assert g.on_device() and not g.on_device(numpy_policy=True)
  g13 = pyspiel.load_game("go(board_size=13)")
  assert g13.on_device() and not g13.on_device(numpy_policy=True)
  h = pyspiel.load_game("hex(board_size=13)")
  assert h.on_device() and not h.on_device(numpy_policy=True)
  assert h.num_distinct_actions() == 169 and h.observation_tensor_shape() == [9, 13, 13]


@pytest.mark.parametrize("gs", BIG)
def test_random_games_match_oracle(gs):
  game = pyspiel.load_game(gs)
  og = O.Game(gs)
  rng = np.random.RandomState(17)
  for _ in range(2):
    st = game.new_initial_state()
    hist = []
    step = 0
    while True:
      ref = og.state_info(hist)
      assert st.is_terminal() == ref["is_terminal"]
      assert st.current_player() == ref["current_player"]
      assert list(st.returns()) == ref["returns"]
      if st.is_terminal():
        break
      legal = st.legal_actions()
      assert legal == ref["legal_actions"]
      assert legal == sorted(legal)
      mask = st.legal_actions_mask()
      assert [i for i, m in enumerate(mask) if m] == legal
      if step % 25 == 0:  # clone / serialization round trips
        assert str(st.clone()) == str(st)
        assert game.deserialize_state(st.serialize()).history() == st.history()
      a = int(rng.choice(legal))
      st.apply_action(a)
      hist.append(a)
      step += 1
    assert sum(st.returns()) == 0
    assert len(hist) <= game.max_game_length()


def test_big_go_action_strings():
  g = pyspiel.load_game("go")
  st = g.new_initial_state()
  assert st.action_to_string(0, 0) == "B a1"
  assert st.action_to_string(0, 18) == "B t1"       # no 'i' column (go_board.cc:478-506)
  assert st.action_to_string(1, 360) == "W t19"
  assert st.action_to_string(1, 361) == "W PASS"


def test_gpu_search_refuses_big_boards_and_auto_backend_uses_host_loop():
  g = pyspiel.load_game("go(board_size=13)")
  rs = np.random.RandomState(3)
  with pytest.raises(ValueError):
    mcts.MCTSBot(g, 2.0, 10, mcts.RandomRolloutEvaluator(1, rs), random_state=rs,
                 backend="hip")
  bot = mcts.MCTSBot(g, 2.0, 12, mcts.RandomRolloutEvaluator(1, rs), random_state=rs)
  with pytest.warns(RuntimeWarning, match="host CPU"):
    root = bot.mcts_search(g.new_initial_state())
  assert root.explore_count == 12 and len(root.children) == 170


@pytest.mark.gpu
@pytest.mark.parametrize("gs,R,sims,plies,kw", [
    ("go(board_size=13)", 70, 60, 10, {}),
    ("go(board_size=12,komi=0.5)", 66, 80, 4, dict(n_rollouts=2, solve=False)),
    ("go(board_size=15)", 66, 40, 20, {}),
    ("go", 66, 30, 8, {}),  # the default 19 x 19 (go.cc:45): 362 children, wide nodes
    ("go(board_size=19,komi=0.5)", 20, 300, 30, dict(n_rollouts=2)),
    ("go(handicap=4)", 40, 40, 0, {}),
    ("hex(board_size=13)", 66, 60, 10, {}),
    ("hex(board_size=19)", 40, 40, 20, dict(n_rollouts=2, solve=False)),
    ("hex(board_size=12)", 30, 80, 4, dict(child_selection=1)),
    ("go(board_size=13)", 40, 50, 6, dict(child_selection=1)),  # PUCT
])
def test_gpu_big_board_search_matches_oracle(require_gpu, gs, R, sims, plies, kw):
  from os_amd import engine as E
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 77, plies)
  bs = np.arange(R, dtype=np.uint32) * 5 + 1
  es = bs + np.uint32(1 << 20)
  kw = dict(dict(uct_c=2.0, max_simulations=sims), **kw)
  got = eng.mcts_batch(acts, offs, bs, es, **kw)
  okw = dict(kw)
  if okw.pop("child_selection", 0) == 1:
    okw["puct"] = True
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children, threads=8,
                              **okw)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


@pytest.mark.gpu
def test_gpu_cpp_bot_plays_go13_as_the_oracle(require_gpu):
  # pyspiel.MCTSBot (C++ semantics) on go 13 x 13: bot and evaluator streams
  # continue across moves through the device (k_lsearch import / export).
  # Two bots sharing one evaluator (mcts_example.cc PlayGame) = the oracle's
  # self-play games, compared on the first moves with every root's visits.
  g = pyspiel.load_game("go(board_size=13)")
  ev = pyspiel.RandomRolloutEvaluator(1, 7)
  bots = [pyspiel.MCTSBot(g, ev, 2.0, 40, 1000, True, s, False) for s in (3, 4)]
  st = g.new_initial_state()
  moves, visits = [], []
  for _ in range(6):
    root = bots[st.current_player()].mcts_search(st)
    v = np.zeros(g.num_distinct_actions(), np.int32)
    for c in root.children:
      v[c.action] = c.explore_count
    a = root.best_child().action
    moves.append(a)
    visits.append(v)
    st.apply_action(a)
  ref = O.Game("go(board_size=13)").selfplay(np.zeros(0, np.int64), np.array([0, 0]),
                                              [[3, 4]], [7], 6, uct_c=2.0,
                                              max_simulations=40, truncate=True)
  assert moves == list(ref["actions"][0])
  np.testing.assert_array_equal(np.array(visits), ref["visits"][0])


@pytest.mark.parametrize("h,stones", [(2, ["d4", "q16"]), (4, ["d4", "q16", "d16", "q4"]),
                                      (5, ["d4", "q16", "d16", "q4", "k10"]),
                                      (9, ["d4", "q16", "d16", "q4", "d10", "q10", "k4",
                                           "k16", "k10"]), (1, []), (10, [])])
def test_go_handicap_setup(h, stones):
  """go_test.cc:43-53 HandicapTest, every handicap count."""
  g = pyspiel.load_game("go(handicap=%d)" % h)
  st = g.new_initial_state()
  assert st.current_player() == (1 if h >= 2 else 0)
  assert st.history() == []
  cols = "abcdefghjklmnopqrst"
  black = {cols.index(x[0]) + 19 * (int(x[1:]) - 1) for x in stones}
  legal = set(st.legal_actions())
  assert not black & legal and len(legal) == 362 - len(black)
  assert g.get_parameters()["handicap"] == h
  ref = O.Game("go(handicap=%d)" % h).state_info([])
  assert sorted(legal) == ref["legal_actions"] and st.current_player() == ref["current_player"]


def test_go_handicap_off_the_board_is_an_error():
  with pytest.raises(RuntimeError):  # GoBoard::PlayMove's SPIEL_CHECK (go_board.cc:263)
    pyspiel.load_game("go(board_size=9,handicap=2)")
  pyspiel.load_game("go(board_size=9,handicap=1)")  # no stones: loads
