"""examples/mcts_example.cc as a CLI (os_amd/mcts_example.py), the verbose
report of MCTSBot::Step (mcts.cc:226-245) and the reference's own GC test
(mcts_test.cc:143-157) replayed on the device.

CPU: flag parsing, the UniformRandomBot draw (absl::uniform_int_distribution
<int> over std::mt19937, restated here from the oracle's raw MT words),
random-vs-random games including pig's chance nodes.
GPU: mcts-vs-mcts games equal the oracle's EvaluateBots with the same seeds,
the verbose report's tables equal the oracle's tree, GC replay bit-exact.
"""
import io
import math
import re

import numpy as np
import pytest

import oracle_lib as O
from os_amd import mcts_example as X
from os_amd import pyspiel


def _run(argv):
  err = io.StringIO()
  res = X.Example(X.parse_args(argv), err=err).run()
  return res, err.getvalue()


def test_absl_style_flags():
  a = X.parse_args(["--game=connect_four", "--player1", "random", "--nosolve",
                    "--verbose", "--quiet=false", "--seed=9", "x(0,0)"])
  assert a.game == "connect_four" and a.player1 == "random" and a.player2 == "random"
  assert a.solve is False and a.verbose is True and a.quiet is False and a.seed == 9
  assert a.initial_actions == ["x(0,0)"]
  d = X.parse_args([])  # mcts_example.cc:32-44 defaults
  assert (d.game, d.player1, d.player2, d.uct_c, d.rollout_count, d.max_simulations,
          d.num_games, d.max_memory_mb, d.solve, d.seed, d.verbose, d.quiet) == (
              "tic_tac_toe", "mcts", "random", 2.0, 10, 10000, 1, 1000, True, 0, False,
              False)


def _lemire32(words, n):
  """absl uniform_int_distribution<int>(0, n-1) on a word iterator."""
  r = n - 1
  w = next(words)
  if r & n == 0:
    return w & r
  p = w * n
  if p % (1 << 32) < n:
    thr = ((1 << 32) - n) % n
    while p % (1 << 32) < thr:
      p = next(words) * n
  return p >> 32


@pytest.mark.parametrize("seed", [1, 42, 2**31 + 5])
def test_uniform_random_bot_draws(seed):
  words = iter(int(w) for w in O.mt19937(seed, 4000))
  bot = X.UniformRandomBot(0, seed)
  for n in (1, 2, 3, 5, 7, 9, 48, 121, 1000003):
    want = _lemire32(words, n)
    assert X.absl_uniform_int(bot._rng, n) == want


def test_random_vs_random_games_replay():
  res, log = _run(["--game=tic_tac_toe", "--player1=random", "--player2=random",
                   "--seed=5", "--num_games=4", "--quiet"])
  game = pyspiel.load_game("tic_tac_toe")
  for returns, history in res["games"]:
    st = game.new_initial_state()
    for s in history:
      st.apply_action(st.string_to_action(s))
    assert st.is_terminal() and list(st.returns()) == returns
  assert log.startswith("game: tic_tac_toe\n")
  assert "Number of games played: 4\n" in log
  assert sum(res["overall_wins"]) == sum(1 for r, _ in res["games"] if max(r) > 0)


def test_random_game_with_chance_nodes_and_forced_opening():
  res, log = _run(["--game=pig", "--player1=random", "--player2=random", "--seed=3",
                   "--quiet", "roll"])
  (returns, history), = res["games"]
  assert history[0] == "roll"
  assert sorted(returns) == [-1.0, 1.0]
  # the forced action is not sampled; the next entry is a chance outcome
  assert history[1].startswith("chance outcome ") or history[1] in ("roll", "stop")


def test_bad_player_type():
  with pytest.raises(pyspiel.SpielError):
    _run(["--player1=minimax"])


# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("gs,sims,rollouts", [("tic_tac_toe", 300, 3),
                                              ("connect_four", 200, 1),
                                              ("pig(winscore=12)", 150, 1)])
def test_mcts_vs_mcts_equals_oracle_evaluate_bots(require_gpu, gs, sims, rollouts):
  """Both bots MCTSBot(seed) sharing RandomRolloutEvaluator(rollout_count,
  seed) and chance sampled from mt19937(seed): the oracle's EvaluateBots
  (evaluate_bots.cc:24-61) with the same seeds plays the same game."""
  seed = 77
  res, _ = _run(["--game=" + gs, "--player1=mcts", "--player2=mcts", "--quiet",
                 "--seed=%d" % seed, "--max_simulations=%d" % sims,
                 "--rollout_count=%d" % rollouts])
  (returns, history), = res["games"]
  ref_hist, ref_ret = O.evaluate_mcts_bots(gs, [seed, seed], rollouts, seed, seed,
                                           uct_c=2.0, max_simulations=sims,
                                           max_memory_mb=1000)
  game = pyspiel.load_game(gs)
  st = game.new_initial_state()
  names = []
  for a in ref_hist:
    names.append(st.action_to_string(st.current_player(), a))
    st.apply_action(a)
  assert history == names
  assert returns == ref_ret


@pytest.mark.gpu
def test_verbose_report_matches_oracle_tree(require_gpu, capsys):
  """MCTSBot::Step's verbose report (mcts.cc:226-245): the root line and the
  children table (CompareFinal order) agree with the oracle's search."""
  game = pyspiel.load_game("connect_four")
  bot = pyspiel.MCTSBot(game, pyspiel.RandomRolloutEvaluator(1, 11), 2.0, 500, 1000, True,
                        5, True)
  st = game.new_initial_state()
  best = bot.step(st)
  err = capsys.readouterr().err
  lines = err.split("\n")
  assert lines[0].startswith("Finished 500 sims in ") and "sims/s, tree size: " in lines[0]
  ref = O.Game("connect_four").mcts_batch(np.zeros(0, np.int64), np.array([0, 0]), [5], [11],
                                          uct_c=2.0, max_simulations=500)
  assert " nodes / 0 mb." in lines[0] and ("%d nodes" % ref["nodes"][0]) in lines[0]
  assert lines[1] == "Root:"
  assert lines[2].startswith("  none: player: 0, prior: 1.000, value: ")
  assert "sims:   500, outcome: none,   7 children" in lines[2]
  assert lines[3] == "Children:"
  rows = lines[4:11]
  nc = int(ref["nchild"][0])
  kids = sorted(zip(ref["child_n"][0][:nc], ref["child_w"][0][:nc], ref["child_action"][0][:nc]),
                key=lambda t: (t[0], t[1]), reverse=True)
  # best-first (ties between equal (n, w) may list in either order)
  want = ["%6s: player: 0, prior: 0.143, value: %6.3f, sims: %5d"
          % (st.action_to_string(0, int(a)), w / n, n) for n, w, a in kids]
  assert sorted(r[:len(want[0])] for r in rows) == sorted(want)
  def stats(line):
    return re.search(r"value: *([-0-9.]+), sims: *([0-9]+)", line).groups()
  assert [stats(r) for r in rows] == [stats(w) for w in want]
  assert best == ref["best_action"][0]
  assert "Children of chosen:" in err


@pytest.mark.gpu
def test_reference_garbage_collect_case_on_device(require_gpu):
  """MCTSTest_GarbageCollect (mcts_test.cc:143-157): tic_tac_toe, 1,000,000
  sims, max_memory_mb 1, RandomRolloutEvaluator(1, 42), seed 42: the root is
  solved (or every simulation ran), with GC firing on the way, bit-exact
  against the oracle."""
  from os_amd import engine as E
  eng = E.Engine("tic_tac_toe")
  acts, offs = np.zeros(0, np.int64), np.array([0, 0], np.int64)
  kw = dict(uct_c=2.0, max_simulations=1000000, max_memory_mb=1, n_rollouts=1, solve=True)
  got = eng.mcts_batch(acts, offs, [42], [42], **kw)
  st = eng.stats()
  assert got["root_out"][0] != 2 or got["root_n"][0] == 1000000
  assert st["gc_runs"] > 0
  ref = O.Game("tic_tac_toe").mcts_batch(acts, offs, [42], [42],
                                         max_children=eng.max_children, **kw)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
  if got["root_out"][0] != 2:
    assert got["root_out"][0] == 0  # proven: tic_tac_toe is a draw
  assert math.isfinite(got["root_w"][0])
