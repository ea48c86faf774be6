"""The reference's Python AlphaZero bot through the drop-in (VERDICT r04
missing #2 / #3): `mcts.MCTSBot` built exactly as alpha_zero.py:181-192
`_init_bot` builds it -- PUCT (`SearchNode.puct_value`), Dirichlet root noise
`(policy_epsilon, policy_alpha)`, solve=False -- over an `AlphaZeroEvaluator`
(alpha_zero/evaluator.py) wrapping a deterministic model
(tests/az_toy_model.py), plays a few moves; every search must equal the
UNMODIFIED reference mcts.py + evaluator.py run on the same model and seed
(tests/golden/python_az_bot.json, tools/gen_az_python_goldens.py): the
root's children in tree order (action, visits, reward, prior, outcome), the
root counts, best_child, and the bot's RandomState after each search --
position, key, and the cached gaussian of its Dirichlet draws.

On the GPU the search runs in the external-evaluator kernel with the numpy
policy (RandomState.shuffle expansions, no single-child stop), the noise drawn
by the bot's own RandomState.dirichlet at the root's expansion
(mcts.py:314-316) and mixed on the device.  On the CPU the drop-in's host
loop (backend="host") is held to the same fixture.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from az_toy_model import ToyModel

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "python_az_bot.json")


def _cases():
  with open(GOLD) as f:
    return json.load(f)["cases"]


def _init_bot(mcts, config, game, evaluator_, evaluation, backend):
  # alpha_zero.py:181-192
  noise = None if evaluation else (config["policy_epsilon"], config["policy_alpha"])
  return mcts.MCTSBot(game, config["uct_c"], config["max_simulations"], evaluator_,
                      solve=False, dirichlet_noise=noise,
                      child_selection_fn=mcts.SearchNode.puct_value, verbose=False,
                      backend=backend)


def _rs_state(rs):
  st = rs.get_state()
  return {"pos": int(st[2]),
          "key_sha256": hashlib.sha256(np.asarray(st[1], np.uint32).tobytes()).hexdigest(),
          "has_gauss": int(st[3]), "gauss": float(st[4])}


def _play(case, backend):
  import pyspiel
  from open_spiel.python.algorithms import mcts
  from open_spiel.python.algorithms.alpha_zero import evaluator as evl
  game = pyspiel.load_game(case["game"])
  model = ToyModel(int(np.prod(game.observation_tensor_shape())), game.num_distinct_actions(),
                   dtype=case.get("model_dtype", "float64"))
  bot = _init_bot(mcts, case["config"], game, evl.AlphaZeroEvaluator(game, model),
                  case["evaluation"], backend)
  bot._random_state.seed(case["seed"])
  state = game.new_initial_state()
  for want in case["searches"]:
    assert state.history() == want["history"]
    root = bot.mcts_search(state)
    out = lambda o: None if o is None else [float(x) for x in o]
    got = [[int(c.action), int(c.explore_count), float(c.total_reward), float(c.prior),
            out(c.outcome)] for c in root.children]
    assert got == want["children"], (case["game"], case["seed"], len(state.history()))
    assert int(root.explore_count) == want["root"]["explore_count"]
    assert float(root.total_reward) == want["root"]["total_reward"]
    assert out(root.outcome) == want["root"]["outcome"]
    best = root.best_child()
    assert int(best.action) == want["best_action"]
    assert _rs_state(bot._random_state) == want["rng_after"]
    state.apply_action(best.action)
  return bot


CASE_IDS = ["%s-%d-%s" % (c["game"].split("(")[0], c["seed"], c.get("model_dtype", "float64"))
            for c in _cases()]
F64 = [c for c in _cases() if c.get("model_dtype", "float64") == "float64"]
F64_IDS = [i for i, c in zip(CASE_IDS, _cases()) if c in F64]
F32 = [c for c in _cases() if c.get("model_dtype") == "float32"]
F32_IDS = [i for i, c in zip(CASE_IDS, _cases()) if c in F32]


@pytest.mark.parametrize("case", _cases(), ids=CASE_IDS)
def test_host_loop_equals_reference_az_bot(case):
  bot = _play(case, "host")
  assert not bot._use_gpu()


def test_az_bot_device_eligibility_and_auto_routing():
  import pyspiel
  from open_spiel.python.algorithms import mcts
  from open_spiel.python.algorithms.alpha_zero import evaluator as evl
  game = pyspiel.load_game("connect_four")
  ev = evl.AlphaZeroEvaluator(game, ToyModel(126, 7))
  cfg = {"uct_c": 2.0, "max_simulations": 50, "policy_epsilon": 0.25, "policy_alpha": 1.0}
  bot = _init_bot(mcts, cfg, game, ev, False, "auto")
  assert bot._gpu_eligible() and bot._external_eligible() and not bot._rollout_eligible()
  # one search over an external evaluator: "auto" keeps the host loop (faster
  # than a device round trip per simulation, profiles/r06/az_step_latency.md);
  # "hip" runs it on the device
  assert not bot._use_gpu()
  assert _init_bot(mcts, cfg, game, ev, False, "hip")._use_gpu()
  # a chance game, or a custom selection function, stays on the host
  pig = pyspiel.load_game("pig")
  with pytest.raises(ValueError):
    evl.AlphaZeroEvaluator(pig, ToyModel(1, 1))
  other = mcts.MCTSBot(game, 2.0, 10, ev, child_selection_fn=lambda c, n, u: 0.0)
  assert not other._gpu_eligible()


@pytest.mark.gpu
@pytest.mark.parametrize("case", F64, ids=F64_IDS)
def test_gpu_equals_reference_az_bot(require_gpu, case):
  bot = _play(case, "hip")
  assert bot._use_gpu() and bot._external_eligible()


@pytest.mark.parametrize("case", F32, ids=F32_IDS)
def test_float32_model_under_auto_equals_reference(case):
  """A float32 model (the reference's TensorFlow one returns float32): the
  host loop that backend="auto" runs computes in the model's dtype, as the
  reference mcts.py does under NumPy 2, so the searches equal the
  reference's float32 fixtures."""
  with pytest.warns(RuntimeWarning, match="host loop"):
    bot = _play(case, "auto")
  assert not bot._use_gpu()


@pytest.mark.gpu
def test_float32_model_is_refused_on_hip_without_touching_the_stream(require_gpu):
  import pyspiel
  from open_spiel.python.algorithms import mcts
  from open_spiel.python.algorithms.alpha_zero import evaluator as evl
  case = F32[0]
  game = pyspiel.load_game(case["game"])
  model = ToyModel(int(np.prod(game.observation_tensor_shape())), game.num_distinct_actions(),
                   dtype=np.float32)
  bot = _init_bot(mcts, case["config"], game, evl.AlphaZeroEvaluator(game, model),
                  case["evaluation"], "hip")
  bot._random_state.seed(case["seed"])
  before = _rs_state(bot._random_state)
  with pytest.raises(mcts.Float32ModelError):
    bot.step(game.new_initial_state())
  assert _rs_state(bot._random_state) == before  # the noise draw was undone


@pytest.mark.gpu
def test_gpu_az_bot_step_matches_search(require_gpu):
  """step() takes the engine's best action without the tree export; it must
  play the move mcts_search's best_child names, and leave the RandomState
  where the search does."""
  import pyspiel
  from open_spiel.python.algorithms import mcts
  from open_spiel.python.algorithms.alpha_zero import evaluator as evl
  case = [c for c in _cases() if c["game"] == "connect_four"][0]
  game = pyspiel.load_game(case["game"])
  ev = evl.AlphaZeroEvaluator(game, ToyModel(126, 7))
  bot = _init_bot(mcts, case["config"], game, ev, case["evaluation"], "hip")
  bot._random_state.seed(case["seed"])
  state = game.new_initial_state()
  for want in case["searches"]:
    a = bot.step(state)
    assert a == want["best_action"]
    assert _rs_state(bot._random_state) == want["rng_after"]
    state.apply_action(a)


@pytest.mark.parametrize("case", F64, ids=F64_IDS)
def test_host_compiled_az_kernel_equals_reference_az_bot(case):
  """The device search's own code (csrc/os_az.h az_step with the numpy
  policy), compiled for the host (tests/hostcheck), against the same
  fixtures: the bot's RandomState draws the root noise where mcts.py:314-316
  does, the engine continues the stream for the expansions' shuffles."""
  import pyspiel
  import hostcheck_lib as hc
  game = pyspiel.load_game(case["game"])
  A = game.num_distinct_actions()
  model = ToyModel(int(np.prod(game.observation_tensor_shape())), A)

  def ev(obs, legal, kind):
    v, p = model.inference(obs[None].astype(np.float64), legal[None].astype(np.int64))
    return p[0], v[0, 0]

  cfg = case["config"]
  rs = np.random.RandomState()
  rs.seed(case["seed"])
  state = game.new_initial_state()
  mc = max(A, 1)
  for want in case["searches"]:
    noise = None
    if not case["evaluation"] and cfg["max_simulations"] >= 2:
      n = len(state.legal_actions())
      noise = np.zeros(mc)
      noise[:n] = rs.dirichlet([cfg["policy_alpha"]] * n)
    st = rs.get_state()
    o, key, pos = hc.az_numpy(case["game"], state.history(), st[1], st[2], ev, mc,
                              uct_c=cfg["uct_c"], max_simulations=cfg["max_simulations"],
                              solve=False, puct=True, noise=noise,
                              eps=cfg["policy_epsilon"] if noise is not None else 0.0)
    nc = int(o["nchild"][0])
    got = [[int(o["child_action"][k]), int(o["child_n"][k]), float(o["child_w"][k]),
            float(o["child_prior"][k])] for k in range(nc)]
    assert got == [c[:4] for c in want["children"]], (case["game"], case["seed"])
    assert int(o["root_n"][0]) == want["root"]["explore_count"]
    assert float(o["root_w"][0]) == want["root"]["total_reward"]
    assert int(o["best_action"][0]) == want["best_action"]
    rs.set_state(("MT19937", key, pos, st[3], st[4]))
    assert _rs_state(rs) == want["rng_after"]
    state.apply_action(want["best_action"])
