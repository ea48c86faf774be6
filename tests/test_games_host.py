"""Product game state machines (csrc/os_games.h via the libos_mcts.so host
State API) against the playthrough goldens, the oracle on random
trajectories, and the invariants of the reference's tests/basic_tests.cc."""
import json
import os
import pickle

import numpy as np
import pytest

import oracle_lib as O
from os_amd import pyspiel

GOLD = os.path.join(os.path.dirname(__file__), "golden")
PLAYTHROUGHS = [("tic_tac_toe", "tic_tac_toe"), ("connect_four", "connect_four"),
                ("breakthrough", "breakthrough"), ("hex", "hex(board_size=5)"),
                ("go", "go(board_size=7,komi=4.5)"),
                # n-player pig with chance nodes (pig.cc:81-244)
                ("pig_3p", "pig(horizon=10,players=3,winscore=10)"),
                ("pig_4p", "pig(horizon=10,players=4,winscore=10)"),
                ("pig_5p", "pig(horizon=100,players=5,winscore=20)")]
GAMES = ["tic_tac_toe", "connect_four", "breakthrough",
         "breakthrough(rows=6,columns=5)", "breakthrough(rows=4,columns=3)",
         "hex(board_size=5)", "hex", "hex(board_size=2)", "go(board_size=9)",
         "go(board_size=7,komi=4.5)", "go(board_size=5)", "go(board_size=11)",
         "go(board_size=13)", "hex(board_size=13)"]  # B384 boards (host only)


def info(s):
  cp = s.current_player()
  la = s.legal_actions()
  return {"is_terminal": s.is_terminal(), "current_player": cp,
          "returns": s.returns(), "legal_actions": la,
          "string_legal_actions": [s.action_to_string(cp, a) for a in la],
          "observation_string": str(s)}


@pytest.mark.parametrize("short,gs", PLAYTHROUGHS)
def test_playthroughs(short, gs):
  with open(os.path.join(GOLD, "playthrough_%s.json" % short)) as f:
    d = json.load(f)
  game = pyspiel.load_game(gs)
  assert game.num_distinct_actions() == d["meta"]["num_distinct_actions"]
  assert game.max_game_length() == d["meta"]["max_game_length"]
  assert str(game) == d["meta"]["game_to_string"]
  if "observation_tensor_shape" in d["meta"]:
    assert game.observation_tensor_shape() == d["meta"]["observation_tensor_shape"]
  for st in d["states"]:
    s = game.new_initial_state()
    for a in st["history"]:
      s.apply_action(a)
    got = info(s)
    for k, v in got.items():
      if k in st:  # the pig playthroughs omit Returns() at chance nodes
        assert v == st[k], (short, st["history"], k)
    assert s.history() == st["history"]


@pytest.mark.parametrize("gs", GAMES)
def test_random_games_match_oracle(gs):
  """Every state along seeded random games equals the oracle's."""
  game = pyspiel.load_game(gs)
  og = O.Game(gs)
  rng = np.random.RandomState(hash(gs) & 0xFFFF)
  n_games = 6 if "go" in gs else 12
  for _ in range(n_games):
    s = game.new_initial_state()
    hist = []
    while True:
      ref = og.state_info(hist)
      got = info(s)
      for k in ("is_terminal", "current_player", "returns", "legal_actions",
                "string_legal_actions", "observation_string"):
        assert got[k] == ref[k], (gs, hist, k)
      if s.is_terminal() or not got["legal_actions"]:
        # hex(board_size=2): the reference's wrap filter leaves only vertical
        # adjacency, so a full board can be non-terminal with no legal move.
        break
      a = int(rng.choice(got["legal_actions"]))
      s.apply_action(a)
      hist.append(a)


@pytest.mark.parametrize("gs", [g for g in GAMES if g != "hex(board_size=2)"])
def test_basic_invariants(gs):
  """tests/basic_tests.cc RandomSimTest invariants."""
  game = pyspiel.load_game(gs)
  rng = np.random.RandomState(5)
  for _ in range(20):
    s = game.new_initial_state()
    steps = 0
    while not s.is_terminal():
      la = s.legal_actions()
      assert la == sorted(la) and len(la) > 0            # :110-118
      mask = s.legal_actions_mask()
      assert [i for i, m in enumerate(mask) if m] == la  # :120-140
      assert s.legal_actions(1 - s.current_player()) == []
      c = s.clone()                                      # :60-80
      assert str(c) == str(s) and c.history() == s.history()
      s.apply_action(int(rng.choice(la)))
      steps += 1
      assert steps <= game.max_game_length()             # :380
    r = s.returns()
    assert abs(sum(r)) < 1e-12 and s.current_player() == pyspiel.PlayerId.TERMINAL
    assert s.legal_actions() == []
    s2 = game.deserialize_state(s.serialize())           # :177-183
    assert str(s2) == str(s)
    s3 = pickle.loads(pickle.dumps(s))
    assert s3.history() == s.history()


def test_illegal_action_raises():
  s = pyspiel.load_game("connect_four").new_initial_state()
  for _ in range(6):
    s.apply_action(0)
  with pytest.raises(RuntimeError):
    s.apply_action(0)


def test_connect_four_fast_loss():
  """connect_four_test.cc FastLoss: 3 3 4 4 2 2 1 -> x wins horizontally."""
  s = pyspiel.load_game("connect_four").new_initial_state()
  for a in (3, 3, 4, 4, 2, 2, 1):
    s.apply_action(a)
  assert s.is_terminal() and s.returns() == [1.0, -1.0]


def test_unsupported_games_raise_value_error():
  with pytest.raises(ValueError):
    pyspiel.load_game("chess")
  with pytest.raises(ValueError):
    pyspiel.load_game("go(board_size=21)")  # go_board.h kMaxBoardSize = 19
  with pytest.raises(ValueError):
    pyspiel.load_game("hex(board_size=20)")  # beyond this engine's B384 boards
  with pytest.raises(RuntimeError):
    pyspiel.load_game("hex(bogus=1)")


def test_game_type_fields():
  gt = pyspiel.load_game("go(board_size=9)").get_type()
  assert gt.short_name == "go"
  assert gt.reward_model == pyspiel.GameType.RewardModel.TERMINAL
  assert gt.dynamics == pyspiel.GameType.Dynamics.SEQUENTIAL
