"""External-evaluator MCTS / PUCT (csrc/os_az.h).

A deterministic toy "network" f(ObservationTensor, legal mask) with exactly
representable arithmetic stands in for VPNetEvaluator.  The oracle MCTSBot
(reference-faithful restatement of mcts.cc with an Evaluator whose Prior /
Evaluate call f on the state's observation) is compared bit-exact with:
  * the product state machine stepped on the host (tests/hostcheck, CPU), and
  * the GPU kernel stepped by os_amd.az.ExternalEvaluatorSearch (gpu).
Both UCT and PUCT child selection are covered, on all five games (go's
positional-superko set travels in the continuation), and Dirichlet root noise
(mcts.cc:177-192, :265-273) with alpha below and above 1 (the two branches of
libstdc++'s gamma sampler).
"""
import numpy as np
import pytest

import hostcheck_lib as hc
import oracle_lib
from os_amd import engine as E
from os_amd import pyspiel

CASES = {
    "tic_tac_toe": ([[], [4], [0, 4, 8]], 80),
    "connect_four": ([[], [3], [3, 3, 2]], 60),
    "breakthrough(rows=6,columns=6)": ([[], [86]], 40),
    "hex(board_size=5)": ([[], [12]], 48),
    "go(board_size=5)": ([[], [12], [6, 12, 7]], 48),
}
# (alpha, epsilon): the AlphaZero defaults (alpha_zero.py: 1 / 0.25) and a
# sub-1 alpha (pow(u, 1 / alpha) branch of gamma_distribution).
NOISE = [(1.0, 0.25), (0.3, 0.25)]


def toy_eval(obs, legal, kind=0):
  """Deterministic prior / value from (observation, legal); exact doubles."""
  o = np.asarray(obs, np.float64).reshape(-1)
  w = (np.arange(o.size) % 7 + 1).astype(np.float64)
  s = float((o * w).sum())                  # integer-valued
  value = ((s % 11.0) - 5.0) / 8.0          # exact
  acts = np.nonzero(legal)[0]
  raw = 1.0 + ((acts * 3 + s) % 5.0)        # integers 1..5
  prior = np.zeros(len(legal), np.float64)
  prior[acts] = raw / raw.sum()
  return prior, value


def _oracle_eval_fn(game_string):
  g = pyspiel.load_game(game_string)
  A = g.num_distinct_actions()

  def fn(history, kind):
    st = g.new_initial_state()
    for a in history:
      st.apply_action(a)
    legal = np.zeros(A, bool)
    legal[st.legal_actions()] = True
    return toy_eval(np.array(st.observation_tensor(st.current_player()), np.float32),
                    legal, kind)
  return fn


def _roots(game):
  hs, sims = CASES[game]
  acts, offs = E.roots_from_histories(hs)
  seeds = np.arange(len(hs), dtype=np.uint32) * 11 + 5
  return acts, offs, seeds, sims


@pytest.mark.parametrize("puct", [True, False])
@pytest.mark.parametrize("game", sorted(CASES))
def test_host_state_machine_matches_oracle(game, puct):
  acts, offs, seeds, sims = _roots(game)
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), puct=puct, uct_c=1.5,
                         max_simulations=sims, max_children=A)
  sep = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=puct, uct_c=1.5,
                    max_simulations=sims)
  fused = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=puct, uct_c=1.5,
                      max_simulations=sims, fused=True)
  for got in (sep, fused):
    for k in E.OUTPUT_KEYS:
      np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
  # one evaluator round per simulation instead of two (terminal leaves ask none)
  assert fused["calls"] <= int(ref["root_n"].sum())
  assert fused["calls"] < sep["calls"]


@pytest.mark.parametrize("game,sims", [("connect_four", 6000),
                                       ("breakthrough(rows=6,columns=6)", 2600)])
def test_host_fused_requests_under_gc(game, sims):
  # max_memory_mb=1 (13108 nodes): GC (mcts.cc:402-424) prunes expanded nodes
  # and their re-expansion takes the parked priors again, not a new request.
  acts, offs = E.roots_from_histories([[]])
  seeds = np.array([3], np.uint32)
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  kw = dict(puct=True, uct_c=1.5, max_simulations=sims, max_memory_mb=1)
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=A, **kw)
  sep = hc.az_batch(game, acts, offs, seeds, A, toy_eval, **kw)
  got = hc.az_batch(game, acts, offs, seeds, A, toy_eval, fused=True, **kw)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(sep[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
  big = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=A,
                         **dict(kw, max_memory_mb=1000))
  assert int(ref["nodes"][0]) < int(big["nodes"][0])  # GC ran (nodes_ shrank)


@pytest.mark.parametrize("noise", NOISE)
@pytest.mark.parametrize("game", sorted(CASES))
def test_host_state_machine_dirichlet_matches_oracle(game, noise):
  acts, offs, seeds, sims = _roots(game)
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  alpha, eps = noise
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), puct=True, uct_c=1.5,
                         max_simulations=sims, max_children=A, dirichlet_alpha=alpha,
                         dirichlet_epsilon=eps)
  for fused in (False, True):
    got = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=True, uct_c=1.5,
                      max_simulations=sims, dirichlet_alpha=alpha, dirichlet_epsilon=eps,
                      fused=fused)
    for k in E.OUTPUT_KEYS:
      np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_dirichlet_noise_changes_the_search():
  game = "connect_four"
  acts, offs, seeds, sims = _roots(game)
  a = hc.az_batch(game, acts, offs, seeds, 7, toy_eval, max_simulations=sims)
  b = hc.az_batch(game, acts, offs, seeds, 7, toy_eval, max_simulations=sims,
                  dirichlet_alpha=0.3, dirichlet_epsilon=0.25)
  assert not all(np.array_equal(a[k], b[k]) for k in ("child_action", "child_n"))


def test_puct_changes_the_search():
  game = "connect_four"
  acts, offs, seeds, sims = _roots(game)
  A = 7
  a = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=True, max_simulations=sims)
  b = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=False, max_simulations=sims)
  assert not np.array_equal(a["child_n"], b["child_n"])


def _gpu_toy_evaluator(A):
  import torch

  def evaluator(obs, legal, kind):
    ob = obs.cpu().numpy().reshape(obs.shape[0], -1)
    lg = legal.cpu().numpy()
    kd = kind.cpu().numpy()
    pr = np.zeros((ob.shape[0], A), np.float64)
    v = np.zeros(ob.shape[0], np.float64)
    for i in range(ob.shape[0]):
      if kd[i]:
        pr[i], v[i] = toy_eval(ob[i], lg[i], int(kd[i]))
    return torch.from_numpy(pr).to(obs.device), torch.from_numpy(v).to(obs.device)
  return evaluator


def _torch_toy_evaluator(A):
  """toy_eval in torch f64 on the device (integer-valued sums, one exact
  division: the same doubles as the numpy version) -- capturable in a HIP
  graph."""
  import torch

  def evaluator(obs, legal, kind):
    o = obs.reshape(obs.shape[0], -1).double()
    w = (torch.arange(o.shape[1], device=o.device) % 7 + 1).double()
    s = (o * w).sum(1)
    value = (torch.remainder(s, 11.0) - 5.0) / 8.0
    a = torch.arange(A, device=o.device).double()
    raw = (1.0 + torch.remainder(a[None, :] * 3 + s[:, None], 5.0)) * legal.double()
    prior = raw / raw.sum(1, keepdim=True).clamp_min(1.0)
    return prior, value
  return evaluator


@pytest.mark.gpu
@pytest.mark.parametrize("game", ["connect_four", "hex(board_size=5)", "go(board_size=5)"])
def test_gpu_graph_replayed_rounds_match_oracle(require_gpu, game):
  from os_amd.az import ExternalEvaluatorSearch
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  R, sims = 80, 20
  acts, offs = E.make_roots(game, R, seed_base=5, max_plies=4)
  seeds = np.arange(R, dtype=np.uint32) + 9
  kw = dict(puct=True, uct_c=1.25, max_simulations=sims, dirichlet_alpha=1.0,
            dirichlet_epsilon=0.25)
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=A, **kw)
  search = ExternalEvaluatorSearch(game)
  for graph in (False, True):
    got = search.run(acts, offs, seeds, _torch_toy_evaluator(A), graph=graph, graph_batch=4,
                     **kw)
    mc = search.eng.max_children
    for k in E.OUTPUT_KEYS:
      r = ref[k][:, :mc] if ref[k].ndim == 2 else ref[k]
      np.testing.assert_array_equal(got[k], r, err_msg="%s graph=%s" % (k, graph))


def _check_gpu(game, puct, alpha=0.0, eps=0.0, requests="fused", layout="auto"):
  from os_amd.az import ExternalEvaluatorSearch
  acts, offs, seeds, sims = _roots(game)
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), puct=puct, uct_c=1.5,
                         max_simulations=sims, max_children=A, dirichlet_alpha=alpha,
                         dirichlet_epsilon=eps)
  search = ExternalEvaluatorSearch(game)
  got = search.run(acts, offs, seeds, _gpu_toy_evaluator(A), puct=puct, uct_c=1.5,
                   max_simulations=sims, dirichlet_alpha=alpha, dirichlet_epsilon=eps,
                   requests=requests, layout=layout)
  mc = search.eng.max_children
  for k in E.OUTPUT_KEYS:
    r = ref[k][:, :mc] if ref[k].ndim == 2 else ref[k]
    np.testing.assert_array_equal(got[k], r, err_msg=k)
  assert search.requests > 0


# Both kernels: k_waz_step (one wave per search, the default) and k_az_step
# (one lane per search).
@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["wave", "lane"])
@pytest.mark.parametrize("requests", ["fused", "separate"])
@pytest.mark.parametrize("puct", [True, False])
@pytest.mark.parametrize("game", sorted(CASES))
def test_gpu_external_evaluator_matches_oracle(require_gpu, game, puct, requests, layout):
  _check_gpu(game, puct, requests=requests, layout=layout)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["wave", "lane"])
@pytest.mark.parametrize("requests", ["separate", "fused"])
def test_gpu_external_evaluator_many_roots(require_gpu, requests, layout):
  # 160 searches: several waves, every lane of a wave64 (the small cases
  # above run <= 3 roots, all in lanes 0-2).
  from os_amd.az import ExternalEvaluatorSearch
  game = "connect_four"
  R, sims = 160, 24
  acts, offs = E.make_roots(game, R, seed_base=77, max_plies=6)
  seeds = np.arange(R, dtype=np.uint32) * 3 + 1
  og = oracle_lib.Game(game)
  kw = dict(puct=True, uct_c=1.25, max_simulations=sims, dirichlet_alpha=1.0,
            dirichlet_epsilon=0.25)
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=7, **kw)
  got = ExternalEvaluatorSearch(game).run(acts, offs, seeds, _gpu_toy_evaluator(7),
                                          requests=requests, layout=layout, **kw)
  bad = sorted({int(r) for k in E.OUTPUT_KEYS
                for r in np.nonzero((got[k] != ref[k]).reshape(R, -1).any(axis=1))[0]})
  assert not bad, "roots differing from the oracle: %s" % bad


@pytest.mark.gpu
def test_gpu_fused_requests_halve_the_rounds(require_gpu):
  from os_amd.az import ExternalEvaluatorSearch
  acts, offs, seeds, sims = _roots("connect_four")
  ev = _gpu_toy_evaluator(7)
  search = ExternalEvaluatorSearch("connect_four")
  a = search.run(acts, offs, seeds, ev, max_simulations=sims, requests="separate")
  sep = (search.steps, search.requests)
  b = search.run(acts, offs, seeds, ev, max_simulations=sims, requests="fused")
  assert search.steps <= sims + 2 < sep[0]
  assert search.requests < sep[1]
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("noise", NOISE)
@pytest.mark.parametrize("game", sorted(CASES))
def test_gpu_external_evaluator_dirichlet_matches_oracle(require_gpu, game, noise):
  _check_gpu(game, True, *noise)
  _check_gpu(game, True, *noise, requests="separate")


@pytest.mark.gpu
@pytest.mark.parametrize("game,sims", [("connect_four", 6000)])
def test_gpu_gc_budget_runs_the_lane_kernel(require_gpu, game, sims):
  """A node budget GC can reach: `auto` takes k_az_step (GC, mcts.cc:402-424),
  `wave` is refused."""
  from os_amd.az import ExternalEvaluatorSearch
  acts, offs = E.roots_from_histories([[]])
  seeds = np.array([3], np.uint32)
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  kw = dict(puct=True, uct_c=1.5, max_simulations=sims, max_memory_mb=1)
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=A, **kw)
  search = ExternalEvaluatorSearch(game)
  got = search.run(acts, offs, seeds, _torch_toy_evaluator(A), **kw)
  for k in E.OUTPUT_KEYS:
    r = ref[k][:, :search.eng.max_children] if ref[k].ndim == 2 else ref[k]
    np.testing.assert_array_equal(got[k], r, err_msg=k)
  with pytest.raises(ValueError):
    search.run(acts, offs, seeds, _torch_toy_evaluator(A), layout="wave", **kw)


@pytest.mark.gpu
def test_gpu_dirichlet_with_gc_budget_is_refused(require_gpu):
  from os_amd.az import ExternalEvaluatorSearch
  search = ExternalEvaluatorSearch("tic_tac_toe")
  acts, offs = E.roots_from_histories([[]])
  with pytest.raises(ValueError):
    search.run(acts, offs, [1], lambda *a: None, max_simulations=100000, max_memory_mb=1,
               dirichlet_alpha=0.3, dirichlet_epsilon=0.25)


# AlphaZero's actor (alpha_zero.cc:64-135): PUCT bots with Dirichlet noise
# and the external evaluator, rng_ continued across each game's searches,
# pow(count, 1/T) policy sampled before temperature_drop, resignation.
ACTOR = [("tic_tac_toe", 30, 1.0, 3, False, (1.0, 0.25)),
         ("connect_four", 24, 1.0, 6, True, (1.0, 0.25)),
         ("hex(board_size=5)", 20, 0.5, 4, True, (0.3, 0.25)),
         ("go(board_size=5)", 16, 1.0, 5, False, (0.0, 0.0))]


@pytest.mark.gpu
@pytest.mark.parametrize("game,sims,t,drop,resign,noise", ACTOR)
def test_gpu_alphazero_actor_matches_oracle(require_gpu, game, sims, t, drop, resign, noise):
  from os_amd.az import AlphaZeroActor
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  hs = [[], [], [1], []]
  acts, offs = E.roots_from_histories(hs)
  G = len(hs)
  bots = np.arange(2 * G, dtype=np.uint32).reshape(G, 2) * 5 + 1
  actor = np.arange(G, dtype=np.uint32) + 100
  kw = dict(uct_c=1.5, max_simulations=sims, temperature=t, temperature_drop=drop,
            resign=resign, cutoff_value=0.3, cutoff_probability=0.6,
            dirichlet_alpha=noise[0], dirichlet_epsilon=noise[1])
  ref = og.az_actor(acts, offs, bots, actor, _oracle_eval_fn(game), og.max_game_length, **kw)
  got = AlphaZeroActor(game).play(acts, offs, bots, actor, _gpu_toy_evaluator(A),
                                  og.max_game_length,
                                  requests="separate" if resign else "fused", **kw)
  for k in ("actions", "length", "returns", "policy", "root_value"):
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


class _IntoToyEvaluator:
  """The torch toy evaluator through the in-place protocol (evaluate_into)."""

  def __init__(self, A):
    self.f = _torch_toy_evaluator(A)

  def evaluate_into(self, obs, legal, kind, prior, value):
    pr, v = self.f(obs, legal.bool(), kind)
    prior.copy_(pr)
    value.copy_(v)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["wave", "lane"])
def test_gpu_evaluate_into_protocol_matches_oracle(require_gpu, layout):
  from os_amd.az import ExternalEvaluatorSearch
  game = "connect_four"
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  R, sims = 96, 24
  acts, offs = E.make_roots(game, R, seed_base=11, max_plies=4)
  seeds = np.arange(R, dtype=np.uint32) + 3
  kw = dict(puct=True, uct_c=1.25, max_simulations=sims, dirichlet_alpha=1.0,
            dirichlet_epsilon=0.25)
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=A, **kw)
  search = ExternalEvaluatorSearch(game)
  for graph in (False, True):
    got = search.run(acts, offs, seeds, _IntoToyEvaluator(A), graph=graph, graph_batch=4,
                     layout=layout, **kw)
    mc = search.eng.max_children
    for k in E.OUTPUT_KEYS:
      r = ref[k][:, :mc] if ref[k].ndim == 2 else ref[k]
      np.testing.assert_array_equal(got[k], r, err_msg="%s graph=%s" % (k, graph))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_gpu_heads_kernel_matches_torch(require_gpu, dtype):
  """os_az_heads_async against the reference heads (alpha_zero/model.py:278-282,
  304) in torch f64: illegal logits -1e32, softmax, tanh.  Tolerance 1e-13
  relative (device exp / tanh vs torch's, f64)."""
  import torch
  from os_amd.az import heads_into
  g = torch.Generator().manual_seed(1)
  N, A = 1000, 82
  logits = (torch.randn(N, A + 1, generator=g) * 4).to("cuda", getattr(torch, dtype))
  legal = (torch.rand(N, A, generator=g) < 0.4).to(torch.uint8)
  legal[3] = 0  # a row without a legal action: uniform, as the reference's softmax
  legal[4] = 1
  legal = legal.cuda()
  prior = torch.full((N, A), -7.0, dtype=torch.float64, device="cuda")
  value = torch.full((N,), -7.0, dtype=torch.float64, device="cuda")
  heads_into(logits, legal, prior, value)
  lg = logits.double()
  ref_p = torch.softmax(lg[:, :A].masked_fill(legal == 0, -1e32), dim=-1)
  ref_v = torch.tanh(lg[:, A])
  torch.testing.assert_close(prior, ref_p, rtol=1e-13, atol=1e-300)
  torch.testing.assert_close(value, ref_v, rtol=1e-13, atol=1e-300)
  some = legal.any(1, keepdim=True)
  assert torch.all(prior[(legal == 0) & some] == 0)  # exp(-1e32 - max) underflows to 0
  np.testing.assert_allclose(prior[3].cpu().numpy(), np.full(A, 1.0 / A), rtol=1e-15)
  # The reference model's heads run in float32 (alpha_zero/model.py:278-282,
  # 304): the f64 kernel agrees with a float32 softmax / tanh to float32
  # rounding (a few ulp of f32), not bitwise.
  f32_p = torch.softmax(logits.float()[:, :A].masked_fill(legal == 0, -1e32), dim=-1)
  f32_v = torch.tanh(logits.float()[:, A])
  torch.testing.assert_close(prior, f32_p.double(), rtol=4e-6, atol=1e-7)
  torch.testing.assert_close(value, f32_v.double(), rtol=4e-6, atol=1e-7)


@pytest.mark.gpu
def test_gpu_heads_into_rejects_bad_tensors(require_gpu):
  """heads_into checks what the kernel assumes: [N, A] contiguous legal /
  prior, [N] value, all on the logits' GPU."""
  import torch
  from os_amd.az import heads_into
  N, A = 8, 7
  logits = torch.zeros(N, A + 1, device="cuda")
  legal = torch.ones(N, A, dtype=torch.uint8, device="cuda")
  prior = torch.zeros(N, A, dtype=torch.float64, device="cuda")
  value = torch.zeros(N, dtype=torch.float64, device="cuda")
  heads_into(logits, legal, prior, value)
  bad = [(logits, legal[:, :A - 1], prior, value),
         (logits, legal, prior, value[:N - 1]),
         (logits, legal, torch.zeros(A, N, dtype=torch.float64, device="cuda").t(), value),
         (logits, legal.cpu(), prior, value)]
  for args in bad:
    with pytest.raises(ValueError):
      heads_into(*args)


def test_heads_abi_rejects_bad_shapes():
  from os_amd import _lib
  L = _lib.lib
  assert L.os_az_heads_async(None, 0, 0, 7, 8, None, None, None, None) == 0  # empty: no launch
  assert L.os_az_heads_async(None, 0, 4, 7, 7, None, None, None, None) != 0  # ld < A + 1
  assert L.os_az_heads_async(None, 2, 4, 7, 8, None, None, None, None) != 0  # dtype
  assert L.os_az_heads_async(None, 0, 4, 7, 8, None, None, None, None) != 0  # null buffers


@pytest.mark.gpu
@pytest.mark.parametrize("game", ["connect_four", "go(board_size=5)"])
def test_gpu_staged_batch_matches_oracle(require_gpu, game):
  """os_az_stage (host half, run on a worker thread while the previous batch
  searches) + os_az_prepare_staged == os_az_prepare: the bench's overlapped
  az step."""
  from concurrent.futures import ThreadPoolExecutor
  from os_amd.az import ExternalEvaluatorSearch
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  R, sims = 96, 24
  acts, offs = E.make_roots(game, R, seed_base=11, max_plies=4)
  seeds = np.arange(R, dtype=np.uint32) * 5 + 2
  kw = dict(puct=True, uct_c=1.25, max_simulations=sims, dirichlet_alpha=1.0,
            dirichlet_epsilon=0.25)
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), max_children=A, **kw)
  search = ExternalEvaluatorSearch(game)
  ev = _gpu_toy_evaluator(A)
  search.stage(acts, offs, seeds, **kw)
  pool = ThreadPoolExecutor(max_workers=1)
  futs = []
  for _ in range(2):  # the second batch was staged while the first ran
    got = search.run(acts, offs, seeds, ev, staged=True,
                     after_prepare=lambda: futs.append(pool.submit(search.stage, acts, offs,
                                                                   seeds, **kw)), **kw)
    futs.pop().result()
    mc = search.eng.max_children
    for k in E.OUTPUT_KEYS:
      r = ref[k][:, :mc] if ref[k].ndim == 2 else ref[k]
      np.testing.assert_array_equal(got[k], r, err_msg=k)
  pool.shutdown()
  with pytest.raises(RuntimeError):  # a staged batch is consumed once
    search.run(acts, offs, seeds, ev, staged=True, **kw)
    search.run(acts, offs, seeds, ev, staged=True, **kw)
  # run(staged=True) must describe the staged batch: its own arguments are
  # not used, so a mismatch is an error, not a silently different search
  search.stage(acts, offs, seeds, **kw)
  with pytest.raises(ValueError):
    search.run(acts, offs, seeds, ev, staged=True, **dict(kw, max_simulations=sims + 1))


def _bf16_round(x):
  """float32 -> bfloat16 value (round to nearest even), as float64."""
  u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
  r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
  return r.astype(np.uint32).view(np.float32).astype(np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("obs_size,hidden,A", [(126, 256, 7), (27, 64, 9), (83, 128, 15)])
def test_gpu_mlp_heads_kernel_matches_exact_reference(require_gpu, obs_size, hidden, A):
  """os_az_mlp_heads_async (both products on the matrix cores) against a
  numpy restatement on integer-valued data: every f32 partial sum is an exact
  integer, so the products are order-independent and the bf16 roundings
  deterministic; the heads then agree to the device exp's rounding."""
  import torch
  from os_amd.az import MlpNetwork
  rs = np.random.RandomState(obs_size + hidden)
  N = 1000
  obs = (rs.rand(N, obs_size) < 0.3).astype(np.float32)
  w1 = rs.randint(-2, 3, size=(obs_size, hidden)).astype(np.float32)
  wo = rs.randint(-2, 3, size=(hidden, A + 1)).astype(np.float32) / 64.0  # exact in bf16
  legal = (rs.rand(N, A) < 0.6).astype(np.uint8)
  legal[0] = 0
  net = MlpNetwork(torch.from_numpy(w1).cuda(), torch.from_numpy(wo).cuda())
  prior = torch.full((N, A), -7.0, dtype=torch.float64, device="cuda")
  value = torch.full((N,), -7.0, dtype=torch.float64, device="cuda")
  net.heads_into(torch.from_numpy(obs).cuda(), torch.from_numpy(legal).cuda(), prior, value)
  h = np.maximum(obs.astype(np.float64) @ w1.astype(np.float64), 0.0)   # exact
  h = _bf16_round(h)
  logits = _bf16_round(h @ wo.astype(np.float64))
  masked = np.where(legal == 1, logits[:, :A], -1e32)
  m = masked.max(axis=1, keepdims=True)
  e = np.exp(masked - m)
  ref_p = e / e.sum(axis=1, keepdims=True)
  ref_v = np.tanh(logits[:, A])
  np.testing.assert_allclose(prior.cpu().numpy(), ref_p, rtol=1e-13, atol=1e-300)
  np.testing.assert_allclose(value.cpu().numpy(), ref_v, rtol=1e-13, atol=1e-15)


@pytest.mark.gpu
def test_gpu_mlp_heads_kernel_matches_torch_network(require_gpu):
  """The bench's random bf16 network: the fused kernel against the same
  network in torch (bf16 GEMMs), to bf16 rounding."""
  import torch
  from os_amd.az import MlpNetwork, heads_into
  g = torch.Generator().manual_seed(3)
  N, O, H, A = 4096, 126, 256, 7
  w1 = (torch.randn(O, H, generator=g) / O ** 0.5).to("cuda", torch.bfloat16)
  wpv = (torch.randn(H, A + 1, generator=g) / H ** 0.5).to("cuda", torch.bfloat16)
  obs = (torch.rand(N, O, generator=g) < 0.3).float().cuda()
  legal = (torch.rand(N, A, generator=g) < 0.7).to(torch.uint8).cuda()
  p1 = torch.zeros(N, A, dtype=torch.float64, device="cuda")
  v1 = torch.zeros(N, dtype=torch.float64, device="cuda")
  MlpNetwork(w1, wpv).heads_into(obs, legal, p1, v1)
  p2 = torch.zeros_like(p1)
  v2 = torch.zeros_like(v1)
  heads_into(torch.relu(obs.to(torch.bfloat16) @ w1) @ wpv, legal, p2, v2)
  torch.testing.assert_close(p1, p2, rtol=0.05, atol=0.02)
  torch.testing.assert_close(v1, v2, rtol=0.05, atol=0.02)
