"""External-evaluator MCTS / PUCT (csrc/os_az.h).

A deterministic toy "network" f(ObservationTensor, legal mask) with exactly
representable arithmetic stands in for VPNetEvaluator.  The oracle MCTSBot
(reference-faithful restatement of mcts.cc with an Evaluator whose Prior /
Evaluate call f on the state's observation) is compared bit-exact with:
  * the product state machine stepped on the host (tests/hostcheck, CPU), and
  * the GPU kernel stepped by os_amd.az.ExternalEvaluatorSearch (gpu).
Both UCT and PUCT child selection are covered.
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
}


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
  got = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=puct, uct_c=1.5,
                    max_simulations=sims)
  for k in E.OUTPUT_KEYS:
    np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_puct_changes_the_search():
  game = "connect_four"
  acts, offs, seeds, sims = _roots(game)
  A = 7
  a = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=True, max_simulations=sims)
  b = hc.az_batch(game, acts, offs, seeds, A, toy_eval, puct=False, max_simulations=sims)
  assert not np.array_equal(a["child_n"], b["child_n"])


@pytest.mark.gpu
@pytest.mark.parametrize("puct", [True, False])
@pytest.mark.parametrize("game", sorted(CASES))
def test_gpu_external_evaluator_matches_oracle(require_gpu, game, puct):
  import torch
  from os_amd.az import ExternalEvaluatorSearch
  acts, offs, seeds, sims = _roots(game)
  og = oracle_lib.Game(game)
  A = og.num_distinct_actions
  ref = og.mcts_external(acts, offs, seeds, _oracle_eval_fn(game), puct=puct, uct_c=1.5,
                         max_simulations=sims, max_children=A)

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

  search = ExternalEvaluatorSearch(game)
  got = search.run(acts, offs, seeds, evaluator, puct=puct, uct_c=1.5,
                   max_simulations=sims)
  mc = search.eng.max_children
  for k in E.OUTPUT_KEYS:
    r = ref[k][:, :mc] if ref[k].ndim == 2 else ref[k]
    np.testing.assert_array_equal(got[k], r, err_msg=k)
  assert search.requests > 0


@pytest.mark.gpu
def test_gpu_external_evaluator_rejects_go(require_gpu):
  from os_amd.az import ExternalEvaluatorSearch
  search = ExternalEvaluatorSearch("go(board_size=5)")
  acts, offs = E.roots_from_histories([[]])
  with pytest.raises(ValueError):
    search.run(acts, offs, [1], lambda *a: None, max_simulations=4)
