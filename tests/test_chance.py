"""Chance nodes: pig (pig.cc) on the product, against
the oracle, which the reference's own pig playthroughs pin (test_oracle.py)
and the unmodified reference mcts.py pins on the numpy path
(test_python_goldens.py, python_mcts_pig*.json).

  * CPU: the product's host State API (pig, 2..5 players) equals the oracle's on
    random games; the search engine compiled for the host (csrc/os_chance.h)
    equals the oracle's MCTSBot / numpy bot; product rollouts equal the
    oracle's RandomRolloutEvaluator.
  * GPU: the same through the lane-layout and wave-layout search kernels, the
    rollout kernel, self-play with chance outcomes and the Python MCTSBot
    drop-ins.
"""
import numpy as np
import pytest

import hostcheck_lib as H
import oracle_lib as O
from os_amd import engine as E
from os_amd import pyspiel

PIGS = ["pig", "pig(horizon=30,winscore=8)", "pig(diceoutcomes=4,winscore=25)",
        # more than two players (pig.cc:94-111 returns, round-robin turns)
        "pig(horizon=30,players=3,winscore=20)", "pig(horizon=40,players=4,winscore=12)",
        "pig(diceoutcomes=4,horizon=50,players=5,winscore=10)"]
NP = {"pig(horizon=30,players=3,winscore=20)": 3, "pig(horizon=40,players=4,winscore=12)": 4,
      "pig(diceoutcomes=4,horizon=50,players=5,winscore=10)": 5}


def _random_games(gs, n, seed):
  rs = np.random.RandomState(seed)
  g = pyspiel.load_game(gs)
  for _ in range(n):
    st = g.new_initial_state()
    hist = []
    while not st.is_terminal() and len(hist) < 400:
      yield hist, st
      a = int(rs.choice(st.legal_actions()))
      st.apply_action(a)
      hist.append(a)
    yield hist, st


@pytest.mark.parametrize("gs", PIGS)
def test_host_state_matches_oracle(gs):
  og = O.Game(gs)
  for hist, st in _random_games(gs, 6, 3):
    ref = og.state_info(hist)
    assert st.is_terminal() == ref["is_terminal"]
    assert st.current_player() == ref["current_player"]
    assert st.legal_actions() == ref["legal_actions"]
    assert st.returns() == ref["returns"]
    assert st.is_chance_node() == ref["is_chance_node"]
    assert str(st) == ref["observation_string"]
    assert [st.action_to_string(a) for a in st.legal_actions()] == \
        ref["string_legal_actions"]
    if st.is_chance_node():
      assert [list(x) for x in st.chance_outcomes()] == ref["chance_outcomes"]
    else:
      assert st.chance_outcomes() == []


def test_observation_tensor_bins():
  g = pyspiel.load_game("pig(winscore=10)")
  assert g.observation_tensor_shape() == [3, 11]
  st = g.new_initial_state()
  for a in (0, 6, 1, 0, 3, 1):  # p0 rolls 6 (+7), stops; p1 rolls 3 (+4), stops
    st.apply_action(a)
  t = np.array(st.observation_tensor()).reshape(3, 11)
  assert t.sum(axis=1).tolist() == [1, 1, 1]
  assert [int(np.argmax(r)) for r in t] == [0, 7, 4]


def _roots(gs, R, plies=12, seed=1000):
  return E.make_roots(gs, R, seed, plies)


def test_make_roots_are_decision_nodes():
  acts, offs = _roots("pig", 64)
  g = pyspiel.load_game("pig")
  for r in range(64):
    st = g.new_initial_state()
    for a in acts[offs[r]:offs[r + 1]]:
      st.apply_action(int(a))
    assert not st.is_chance_node() and not st.is_terminal()


@pytest.mark.parametrize("gs", PIGS)
@pytest.mark.parametrize("n_rollouts,solve", [(1, True), (2, True), (1, False)])
def test_engine_cpp_policy_matches_oracle(gs, n_rollouts, solve):
  R = 8
  acts, offs = _roots(gs, R)
  bs = np.arange(R, dtype=np.uint32) * 5 + 3
  es = bs + np.uint32(1 << 20)
  kw = dict(uct_c=2.0, max_simulations=300, n_rollouts=n_rollouts, solve=solve)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=6, **kw)
  got = H.mcts_batch(gs, acts, offs, bs, es, 6, **kw)
  bad = [k for k in H.KEYS if not np.array_equal(got[k], ref[k])]
  assert not bad, bad


@pytest.mark.parametrize("gs", PIGS)
def test_engine_rollouts_match_oracle(gs):
  if gs in NP:
    pytest.skip("rollout batches return two players' values")
  seeds = np.arange(200, dtype=np.uint32)
  for hist in ([], [0], [0, 3], [1, 0, 4]):
    np.testing.assert_array_equal(H.rollouts(gs, hist, seeds),
                                  O.Game(gs).rollouts(hist, seeds))


def test_solver_proves_short_games():
  # pig(horizon=2): two decisions end the game, every leaf is a draw, so each
  # chance node's children share one outcome and the root is proven a draw.
  gs = "pig(horizon=2)"
  acts, offs = E.roots_from_histories([[], [0, 6]])
  bs = np.array([1, 2], np.uint32)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, bs + 9, max_simulations=2000, max_children=6)
  got = H.mcts_batch(gs, acts, offs, bs, bs + 9, 6, max_simulations=2000)
  for k in H.KEYS:
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
  assert (ref["root_out"] == 0).all()  # proven through chance nodes


@pytest.mark.parametrize("gs", sorted(NP))
def test_n_player_api(gs):
  n = NP[gs]
  g = pyspiel.load_game(gs)
  assert g.num_players() == n and g.get_parameters()["players"] == n
  assert g.observation_tensor_shape()[0] == 1 + n
  for hist, st in _random_games(gs, 3, 11):
    r = st.returns()
    assert len(r) == n
    if st.is_terminal():
      assert abs(sum(r)) < 1e-12
      if max(r) > 0:
        assert sorted(r)[:-1] == [-1.0 / (n - 1)] * (n - 1)
    else:
      assert st.current_player() in list(range(n)) + [pyspiel.PlayerId.CHANCE]
      assert len(st.observation_tensor(n - 1)) == (1 + n) * (g.get_parameters()["winscore"] + 1)


def test_chance_node_api():
  g = pyspiel.load_game("pig")
  assert g.get_type().chance_mode == pyspiel.GameType.ChanceMode.EXPLICIT_STOCHASTIC
  assert g.max_chance_outcomes() == 6
  st = g.new_initial_state()
  st.apply_action(0)
  assert st.is_chance_node() and st.current_player() == pyspiel.PlayerId.CHANCE
  assert not st.is_player_node()
  assert st.action_to_string(pyspiel.PlayerId.CHANCE, 3) == "chance outcome 3"


# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("gs", PIGS)
@pytest.mark.parametrize("policy", ["cpp", "numpy"])
@pytest.mark.parametrize("block", [0, 64])
def test_gpu_search_matches_oracle(require_gpu, gs, policy, block):
  # The lane layout (k_mcts; AUTO picks the wave layout for pig).
  # block 64: full wave64 workgroups, searches in lanes 32-63 too
  from os_amd import _lib
  R = 64 if block == 0 else 96
  acts, offs = _roots(gs, R)
  bs = np.arange(R, dtype=np.uint32) * 5 + 3
  es = bs + np.uint32(1 << 20)
  eng = E.Engine(gs)
  if policy == "cpp":
    ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_simulations=300, max_children=6)
    got = eng.mcts_batch(acts, offs, bs, es, max_simulations=300, block_size=block,
                         layout=_lib.LAYOUT_LANE)
  else:
    ref = H.mcts_batch(gs, acts, offs, bs, es, 6, max_simulations=300,
                       policy=_lib.POLICY_NUMPY)
    got = eng.mcts_batch(acts, offs, bs, es, max_simulations=300, block_size=block,
                         policy=_lib.POLICY_NUMPY, layout=_lib.LAYOUT_LANE)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k][:, :got[k].shape[1]] if ref[k].ndim == 2
                                  else ref[k], err_msg=k)


@pytest.mark.gpu
def test_gpu_rollouts_match_oracle(require_gpu):
  eng = E.Engine("pig")
  seeds = np.arange(4096, dtype=np.uint32)
  got = eng.rollouts([0, 4], seeds)
  np.testing.assert_array_equal(got, O.Game("pig").rollouts([0, 4], seeds))


@pytest.mark.gpu
@pytest.mark.parametrize("gs", PIGS)
@pytest.mark.parametrize("policy", ["cpp", "numpy"])
def test_gpu_wave_layout_matches_oracle(require_gpu, gs, policy):
  """One wave per search (k_wsearch_chance, wave-uniform mcts_search_chance)."""
  from os_amd import _lib
  R = 40
  acts, offs = _roots(gs, R)
  bs = np.arange(R, dtype=np.uint32) * 7 + 2
  es = bs + np.uint32(1 << 20)
  eng = E.Engine(gs)
  kw = dict(max_simulations=250, layout=_lib.LAYOUT_WAVE)
  if policy == "cpp":
    ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_simulations=250, max_children=6)
    got = eng.mcts_batch(acts, offs, bs, es, **kw)
  else:
    ref = H.mcts_batch(gs, acts, offs, bs, es, 6, max_simulations=250,
                       policy=_lib.POLICY_NUMPY)
    got = eng.mcts_batch(acts, offs, bs, es, policy=_lib.POLICY_NUMPY, **kw)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k][:, :got[k].shape[1]] if ref[k].ndim == 2
                                  else ref[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("gs,sims,nr", [("pig(winscore=20)", 120, 1),
                                        ("pig(horizon=30,winscore=8)", 200, 2)])
def test_gpu_selfplay_with_chance_nodes_matches_oracle(require_gpu, gs, sims, nr):
  """k_wselfplay_chance: mcts_example.cc PlayGame with chance outcomes drawn
  by the game's rng (actor seed) -- every game equals the oracle's EvaluateBots
  (evaluate_bots.cc:24-61) with bots (b0, b1), evaluator seed e and chance rng
  seed = the actor seed."""
  G = 6
  acts, offs = E.roots_from_histories([[]] * G)
  bot = np.array([[3 * g + 1, 3 * g + 2] for g in range(G)], np.uint32)
  ev = np.arange(G, dtype=np.uint32) + 100
  actor = np.arange(G, dtype=np.uint32) * 11 + 5
  eng = E.Engine(gs)
  L = 600
  eng.selfplay_set_options(actor_seeds=actor)
  out = eng.selfplay(acts, offs, bot, ev, max_len=L, max_simulations=sims, n_rollouts=nr,
                     record_visits=True)
  for g in range(G):
    hist, ret = O.evaluate_mcts_bots(gs, [int(bot[g, 0]), int(bot[g, 1])], nr, int(ev[g]),
                                     int(actor[g]), uct_c=2.0, max_simulations=sims,
                                     max_memory_mb=1000)
    n = int(out["length"][g])
    assert list(out["actions"][g, :n]) == hist, g
    assert list(out["returns"][g]) == ret, g
    # visit targets on decision moves only
    st = pyspiel.load_game(gs).new_initial_state()
    for m, a in enumerate(hist):
      row = out["visits"][g, m]
      assert (row.sum() == 0) == st.is_chance_node()
      st.apply_action(a)


@pytest.mark.gpu
def test_gpu_selfplay_with_chance_nodes_needs_actor_seeds(require_gpu):
  eng = E.Engine("pig")
  acts, offs = E.roots_from_histories([[]])
  with pytest.raises(Exception):
    eng.selfplay(acts, offs, [[1, 2]], [3], max_len=400, max_simulations=10)


@pytest.mark.gpu
def test_gpu_cpp_bot_plays_pig(require_gpu):
  """pyspiel.MCTSBot steps at decision nodes; chance outcomes are sampled by
  the driver (evaluate_bots.cc:32-37 style)."""
  g = pyspiel.load_game("pig(winscore=20)")
  ev = pyspiel.RandomRolloutEvaluator(1, 5)
  bots = [pyspiel.MCTSBot(g, ev, 2.0, 200, 1000, True, s, False) for s in (1, 2)]
  rs = np.random.RandomState(0)
  st = g.new_initial_state()
  while not st.is_terminal():
    if st.is_chance_node():
      acts, probs = zip(*st.chance_outcomes())
      st.apply_action(int(rs.choice(acts, p=probs)))
    else:
      st.apply_action(bots[st.current_player()].step(st))
  assert st.returns() in ([1.0, -1.0], [-1.0, 1.0])


def test_sample_action_follows_absl_uniform_double():
  """os_sample_action = SampleAction(outcomes, absl::Uniform(rng, 0.0, 1.0))
  (spiel.cc:337-366) on a caller-held std::mt19937, as EvaluateBots samples
  chance nodes (evaluate_bots.cc:32-37)."""
  import ctypes
  from os_amd import _lib
  zs = H.absl_double(42, 300)
  key, pos = pyspiel._mt_key(42)
  pos_a = np.array([pos], np.int32)
  rs = np.random.RandomState(9)
  for i in range(300):
    n = int(rs.randint(1, 7))
    p = rs.dirichlet([1.0] * n)
    p[-1] = 1.0 - p[:-1].sum() if n > 1 else 1.0
    k = _lib.lib.os_sample_action(p.ctypes.data, n, key.ctypes.data, pos_a.ctypes.data)
    acc, want = 0.0, None
    for j in range(n):
      if acc <= zs[i] < acc + p[j]:
        want = j
        break
      acc += p[j]
    assert k == (want if want is not None else -1), i


@pytest.mark.gpu
def test_gpu_three_player_pig_as_mcts_test(require_gpu):
  """mcts_test.cc:73-84 MCTSTest_CanPlayThreePlayerStochasticGames on the
  drop-in: three pyspiel.MCTSBot(uct_c 2, 1000 sims, max_memory_mb 5, solve,
  seed 42) sharing RandomRolloutEvaluator(20, 42), pyspiel.evaluate_bots(...,
  42).  The whole game (every chance draw and every bot move) equals the
  oracle's EvaluateBots, and the returns sum to 0 as the reference asserts."""
  gs = "pig(players=3,winscore=20,horizon=30)"
  g = pyspiel.load_game(gs)
  ev = pyspiel.RandomRolloutEvaluator(20, 42)
  bots = [pyspiel.MCTSBot(g, ev, 2.0, 1000, 5, True, 42, False) for _ in range(3)]
  st = g.new_initial_state()
  ret = pyspiel.evaluate_bots(st, bots, 42)
  assert abs(sum(ret)) < 1e-12
  hist, ref = O.evaluate_mcts_bots(gs, [42, 42, 42], 20, 42, 42, uct_c=2.0,
                                   max_simulations=1000, max_memory_mb=5, num_players=3)
  assert st.history() == hist
  assert ret == ref
