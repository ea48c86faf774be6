"""Pins the oracle (reference-faithful restatement) to the reference's own
fixtures: playthrough transition goldens, recorded MCTS outputs, the C++
standard's MT known answers, and the mcts_test solver known answers."""
import json
import math
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
PLAYTHROUGHS = [("tic_tac_toe", "tic_tac_toe"), ("connect_four", "connect_four"),
                ("breakthrough", "breakthrough"), ("hex", "hex(board_size=5)"),
                ("go", "go(board_size=7,komi=4.5)"),
                ("pig_3p", "pig(players=3,horizon=10,winscore=10)"),
                ("pig_4p", "pig(players=4,horizon=10,winscore=10)"),
                ("pig_5p", "pig(players=5,horizon=100,winscore=20)")]
FIELDS = ("is_terminal", "current_player", "returns", "legal_actions",
          "string_legal_actions", "observation_string", "is_chance_node")


def probes():
  with open(os.path.join(GOLD, "reference_probes.json")) as f:
    return json.load(f)


@pytest.mark.parametrize("short,gs", PLAYTHROUGHS)
def test_oracle_replays_playthroughs(short, gs):
  with open(os.path.join(GOLD, "playthrough_%s.json" % short)) as f:
    d = json.load(f)
  g = O.Game(gs)
  assert g.num_distinct_actions == d["meta"]["num_distinct_actions"]
  assert g.max_game_length == d["meta"]["max_game_length"]
  for st in d["states"]:
    info = g.state_info(st["history"])
    for k in FIELDS:
      if k in st:  # chance states record no Returns()
        assert info[k] == st[k], (short, st["history"], k)
    if st.get("chance_outcomes"):  # printed with 12 significant digits
      got = [[a, float("%.12g" % p)] for a, p in info["chance_outcomes"]]
      assert got == st["chance_outcomes"], (short, st["history"])


def test_mt_known_answers():
  ka = probes()["known_answers"]
  assert O.mt19937(5489, 10000)[-1] == ka["mt19937_default_seed_5489_word_10000"]
  assert O.mt19937_64(5489, 10000)[-1] == ka["mt19937_64_default_seed_5489_word_10000"]


def test_mt_matches_numpy_legacy_seeding():
  # randint over the full 32-bit range returns raw MT19937 words, so the
  # streams of RandomState(seed) and std::mt19937(seed) must coincide.
  for seed in (0, 1, 42, 2**31 + 7):
    words = np.random.RandomState(seed).randint(0, 2**32, size=2000,
                                                dtype=np.uint64)
    assert np.array_equal(words.astype(np.uint32), O.mt19937(seed, 2000))


def test_absl_uniform_power_of_two_uses_low_bits_of_second_word():
  raw = O.mt19937(7, 20)
  got = O.absl_uniform(7, 8, 10)
  for i in range(10):
    assert got[i] == (int(raw[2 * i + 1]) & 7)


def test_absl_uniform_lemire_64():
  raw = O.mt19937(11, 40)
  for n in (3, 7, 67, 121):
    got = O.absl_uniform(11, n, 20)
    for i in range(20):
      bits = (int(raw[2 * i]) << 32) | int(raw[2 * i + 1])
      assert got[i] == (bits * n) >> 64  # rejection prob ~n/2^64: never here


@pytest.mark.parametrize("case", probes()["cpp_mcts"], ids=lambda c: c["name"])
def test_oracle_cpp_mcts_matches_recorded_reference(case):
  g = O.Game(case["game"])
  acts, offs = np.array(case["history"], np.int64), np.array([0, len(case["history"])])
  o = g.mcts_batch(acts, offs, [case["bot_seed"]], [case["eval_seed"]],
                   uct_c=case["uct_c"], max_simulations=case["max_simulations"],
                   n_rollouts=case["n_rollouts"], solve=case["solve"],
                   max_memory_mb=case["max_memory_mb"])
  nc = o["nchild"][0]
  kids = [[int(a), int(n)] for a, n in zip(o["child_action"][0][:nc],
                                           o["child_n"][0][:nc])]
  if "children_in_order" in case:
    assert kids == case["children_in_order"]
  if "children_subset" in case:
    for pair in case["children_subset"]:
      assert pair in kids
  if "root_n" in case:
    assert o["root_n"][0] == case["root_n"]
  assert o["root_w"][0] == case["root_w"]


@pytest.mark.parametrize("case", probes()["python_mcts"], ids=lambda c: c["name"])
def test_oracle_python_mcts_matches_recorded_reference(case):
  g = O.Game(case["game"])
  o = g.mcts_numpy(case["history"], case["seed"], uct_c=case["uct_c"],
                   max_simulations=case["max_simulations"],
                   n_rollouts=case["n_rollouts"], solve=case["solve"])
  nc = o["nchild"][0]
  kids = sorted([int(a), int(n), float(w)] for a, n, w in zip(
      o["child_action"][0][:nc], o["child_n"][0][:nc], o["child_w"][0][:nc]))
  assert kids == [[a, n, float(w)] for a, n, w in case["children_sorted"]]


def _ttt_actions(g, labels):
  hist = []
  for lab in labels:
    info = g.state_info(hist)
    idx = info["string_legal_actions"].index(lab)
    hist.append(info["legal_actions"][idx])
  return hist


@pytest.mark.parametrize("case", probes()["solver_cases"]["cases"],
                         ids=lambda c: c["name"])
def test_oracle_solver_known_answers(case):
  g = O.Game("tic_tac_toe")
  hist = _ttt_actions(g, case["actions"])
  assert g.state_info(hist)["observation_string"] == case["board"]
  # C++ path (mcts_test.cc): evaluator(20, 42), bot seed 42, 10 MB.
  o = g.mcts_batch(np.array(hist, np.int64), np.array([0, len(hist)]), [42], [42],
                   uct_c=math.sqrt(2), max_simulations=10000, n_rollouts=20,
                   max_memory_mb=10, solve=True)
  _check_solver(g, hist, o, case)
  # Python path (mcts_test.py): one RandomState(42).
  o = g.mcts_numpy(hist, 42, uct_c=math.sqrt(2), max_simulations=10000,
                   n_rollouts=20, solve=True)
  _check_solver(g, hist, o, case)


def _check_solver(g, hist, o, case):
  assert o["root_out"][0] == case["root_outcome"]
  nc = o["nchild"][0]
  outs = o["child_out"][0][:nc]
  if "children_outcome_le" in case:
    assert all(v <= case["children_outcome_le"] for v in outs)
  if "children_outcome_eq" in case:
    assert all(v == case["children_outcome_eq"] for v in outs)
  if "best_in" in case:
    info = g.state_info(hist)
    lab = info["string_legal_actions"][info["legal_actions"].index(
        int(o["best_action"][0]))]
    assert lab in case["best_in"]
  if "best_outcome" in case:
    k = list(o["child_action"][0][:nc]).index(o["best_action"][0])
    assert outs[k] == case["best_outcome"]
