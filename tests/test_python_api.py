"""Drop-in Python surface: `pyspiel` / `open_spiel.python.algorithms.mcts`
behave like the reference modules (mcts_test.py analogues)."""
import json
import math
import os
import random

import numpy as np
import pytest

import pyspiel  # open_spiel-1_amd/pyspiel.py (drop-in)
from open_spiel.python.algorithms import evaluate_bots
from open_spiel.python.algorithms import mcts

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def probes():
  with open(os.path.join(GOLD, "reference_probes.json")) as f:
    return json.load(f)


def make_node(action, player=0, prior=1, **kwargs):
  node = mcts.SearchNode(action, player, prior)
  for k, v in kwargs.items():
    setattr(node, k, v)
  return node


@pytest.mark.parametrize("case", probes()["best_child_cases"]["cases"])
def test_best_child_ordering(case):
  kids = [make_node(**c) for c in case["children"]]
  random.shuffle(kids)
  root = make_node(-1, children=kids)
  assert root.best_child().action == case["choice"]


def test_throws_on_unsupported_game():
  with pytest.raises(ValueError):
    pyspiel.load_game("matrix_mp")


def test_host_backend_reproduces_reference_python_vector():
  case = probes()["python_mcts"][0]
  game = pyspiel.load_game(case["game"])
  rng = np.random.RandomState(case["seed"])
  bot = mcts.MCTSBot(game, case["uct_c"], case["max_simulations"],
                     mcts.RandomRolloutEvaluator(1, rng), random_state=rng,
                     backend="host")
  root = bot.mcts_search(game.new_initial_state())
  got = sorted([c.action, c.explore_count, c.total_reward] for c in root.children)
  assert got == [[a, n, float(w)] for a, n, w in case["children_sorted"]]


def test_can_play_tic_tac_toe_host():
  game = pyspiel.load_game("tic_tac_toe")
  ev = mcts.RandomRolloutEvaluator(n_rollouts=2, random_state=np.random.RandomState(1))
  bots = [mcts.MCTSBot(game, math.sqrt(2), 50, ev, backend="host",
                       random_state=np.random.RandomState(2)),
          mcts.MCTSBot(game, math.sqrt(2), 50, ev, backend="host",
                       random_state=np.random.RandomState(3))]
  v = evaluate_bots.evaluate_bots(game.new_initial_state(), bots, np.random)
  assert v[0] + v[1] == 0


def test_step_with_policy_is_one_hot():
  game = pyspiel.load_game("tic_tac_toe")
  rng = np.random.RandomState(0)
  bot = mcts.MCTSBot(game, 2.0, 100, mcts.RandomRolloutEvaluator(1, rng),
                     random_state=rng, backend="host")
  st = game.new_initial_state()
  policy, action = bot.step_with_policy(st)
  assert [a for a, _ in policy] == st.legal_actions()
  assert sum(p for _, p in policy) == 1.0 and dict(policy)[action] == 1.0


def test_hip_backend_rejects_custom_evaluators():
  class MyEval(mcts.Evaluator):
    pass
  game = pyspiel.load_game("tic_tac_toe")
  with pytest.raises(ValueError):
    mcts.MCTSBot(game, 2.0, 10, MyEval(), backend="hip")


def test_cpp_style_bot_validates_arguments():
  game = pyspiel.load_game("connect_four")
  ev = pyspiel.RandomRolloutEvaluator(1, 1)
  pyspiel.MCTSBot(game, ev, 2.0, 10, 100, True, 1, False,
                  pyspiel.ChildSelectionPolicy.PUCT)  # PUCT is bound (pyspiel.cc:512-524)
  with pytest.raises(ValueError):
    pyspiel.MCTSBot(game, ev, 2.0, 10, 100, True, 1, False, 7)
  with pytest.raises(ValueError):
    pyspiel.MCTSBot(game, object(), 2.0, 10, 100, True, 1, False)


def test_auto_backend_warns_before_a_host_search():
  """A search the GPU engine does not run is never silent under backend='auto'."""
  class MyEval(mcts.RandomRolloutEvaluator):
    pass
  game = pyspiel.load_game("tic_tac_toe")
  rng = np.random.RandomState(0)
  bot = mcts.MCTSBot(game, 2.0, 20, MyEval(1, rng), random_state=rng)
  with pytest.warns(RuntimeWarning, match="host CPU"):
    bot.mcts_search(game.new_initial_state())
  quiet = mcts.MCTSBot(game, 2.0, 20, MyEval(1, rng), random_state=rng, backend="host")
  import warnings
  with warnings.catch_warnings():
    warnings.simplefilter("error")
    quiet.mcts_search(game.new_initial_state())


def test_pig_buffers_hold_more_outcomes_than_distinct_actions():
  game = pyspiel.load_game("pig(diceoutcomes=10)")
  assert game.max_chance_outcomes() == 10
  st = game.new_initial_state()
  st.apply_action(0)  # roll
  outs = st.chance_outcomes()
  assert [a for a, _ in outs] == list(range(1, 11))
  assert st.legal_actions() == list(range(1, 11))
  assert pyspiel.load_game("pig(diceoutcomes=1)").max_chance_outcomes() == 1
