"""Edge cases of the search boundary, against the oracle (mcts.cc's behaviour
on them): empty batches, zero simulations, roots with one legal action (the
C++ bot's early stop, mcts.cc:398-401) mixed with ordinary roots in a ragged
batch across a wave boundary, on both kernel layouts; terminal roots, which a
bot is never asked to move from (mcts.py's step and mcts.cc's BestChild fail
on them), are refused at the boundary; rollouts from a terminal state."""
import numpy as np
import pytest

import oracle_lib as O

TTT_WON = [0, 3, 1, 4, 2]                  # x has the top row: terminal
TTT_ONE_LEGAL = [6, 0, 5, 4, 3, 2, 8, 7]   # one empty cell, not terminal


@pytest.fixture(scope="module")
def E(require_gpu):
  from os_amd import engine
  return engine


def _cmp(E, got, ref):
  bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(got[k], ref[k])]
  assert not bad, bad


def _batch(histories):
  offs = np.zeros(len(histories) + 1, np.int64)
  for i, h in enumerate(histories):
    offs[i + 1] = offs[i] + len(h)
  acts = np.array([a for h in histories for a in h], np.int64)
  return acts, offs


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["wave", "lane"])
def test_gpu_empty_batch(E, layout):
  from os_amd import _lib
  eng = E.Engine("connect_four")
  lay = _lib.LAYOUT_WAVE if layout == "wave" else _lib.LAYOUT_LANE
  got = eng.mcts_batch(np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.uint32),
                       np.zeros(0, np.uint32), max_simulations=64, layout=lay)
  for k in E.OUTPUT_KEYS:
    assert len(got[k]) == 0, k
  out = eng.rollouts([], np.zeros(0, np.uint32))
  assert out.shape == (0, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["wave", "lane"])
@pytest.mark.parametrize("sims", [0, 1, 2, 300])
def test_gpu_one_legal_and_ordinary_roots(E, layout, sims):
  """One-legal-action roots (the C++ policy's early stop once the root has
  its single child), the initial state and ordinary roots in one ragged batch of 68
  roots (across the 64-lane wave boundary of the lane layout)."""
  from os_amd import _lib
  gs = "tic_tac_toe"
  eng = E.Engine(gs)
  acts0, offs0 = E.make_roots(gs, 64, 1000, 4)
  hist = [list(acts0[offs0[i]:offs0[i + 1]]) for i in range(64)]
  hist += [TTT_ONE_LEGAL, [], TTT_ONE_LEGAL, [4]]
  acts, offs = _batch(hist)
  R = len(hist)
  bs = np.arange(R, dtype=np.uint32) * 7 + 3
  es = bs + np.uint32(1 << 20)
  lay = _lib.LAYOUT_WAVE if layout == "wave" else _lib.LAYOUT_LANE
  got = eng.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims, layout=lay)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                              max_children=eng.max_children)
  _cmp(E, got, ref)
  # A one-legal root is expanded on its second visit and the search stops
  # there, its single child chosen (mcts.cc:398-401).
  assert got["root_n"][64] == min(sims, 2)
  assert got["nchild"][64] == (1 if sims >= 2 else 0)


@pytest.mark.gpu
def test_gpu_terminal_root_is_refused(E):
  eng = E.Engine("tic_tac_toe")
  acts, offs = _batch([[4], TTT_WON])
  with pytest.raises(RuntimeError, match="terminal"):
    eng.mcts_batch(acts, offs, np.array([1, 2], np.uint32), np.array([3, 4], np.uint32),
                   max_simulations=16)


@pytest.mark.gpu
def test_gpu_terminal_rollouts(E):
  """RandomRolloutEvaluator on a terminal state returns its returns without
  drawing (mcts.cc:46-55)."""
  eng = E.Engine("tic_tac_toe")
  seeds = np.arange(5, dtype=np.uint32)
  got = eng.rollouts(TTT_WON, seeds)
  ref = O.Game("tic_tac_toe").rollouts(TTT_WON, seeds)
  assert np.array_equal(got, ref)
  assert np.all(got[:, 0] == 1.0)


@pytest.mark.gpu
def test_gpu_empty_selfplay_and_external_evaluator_batches(E):
  """Zero games of self-play and zero external-evaluator searches: empty
  outputs, no launch errors."""
  import torch
  from os_amd.az import ExternalEvaluatorSearch
  eng = E.Engine("connect_four")
  out = eng.selfplay(np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros((0, 2), np.uint32),
                     np.zeros(0, np.uint32), max_simulations=16)
  assert len(out["length"]) == 0 and out["actions"].shape[0] == 0
  search = ExternalEvaluatorSearch("connect_four")
  A = search.num_actions

  def evaluator(obs, legal, kind):
    n = obs.shape[0]
    return (torch.full((n, A), 1.0 / A, dtype=torch.float64, device=obs.device),
            torch.zeros(n, dtype=torch.float64, device=obs.device))

  got = search.run(np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.uint32),
                   evaluator, max_simulations=8)
  for k in E.OUTPUT_KEYS:
    assert len(got[k]) == 0, k
