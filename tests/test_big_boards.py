"""Hex and go above 11 x 11 (up to 19 x 19): the drop-in `load_game("go")`
(default board_size 19, go.cc:45) and `hex(board_size=13)` load, and their host
State API (os_games.h HexT / GoT on B384 bitboards) follows the oracle move by
move on random games (basic_tests.cc RandomSimTest shape: legal actions,
current player, terminal, returns at every state; serialization round trips).
The GPU engine runs hex / go up to 11 x 11: the GPU search refuses larger
boards with ValueError at search time, and the Python MCTSBot's automatic
backend searches them with its host loop."""
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
  assert not g.on_device()
  h = pyspiel.load_game("hex(board_size=13)")
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
  cbot = pyspiel.MCTSBot(g, pyspiel.RandomRolloutEvaluator(1, 1), 2.0, 10, 100, True, 1,
                         False)
  with pytest.raises(ValueError):
    cbot.step(g.new_initial_state())


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
