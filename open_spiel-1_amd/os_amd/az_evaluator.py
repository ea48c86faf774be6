"""AlphaZeroEvaluator drop-in (python/algorithms/alpha_zero/evaluator.py) with
the batched protocol the device search drives.

The reference evaluator answers `evaluate(state)` / `prior(state)` one state at
a time through its model's `inference(obs, mask)` on a singleton batch,
memoised in an LRU cache keyed by the observation and mask bytes
(evaluator.py:28-83).  The model's `inference` takes a batch, so the same
network answers a whole round of device requests at once: `evaluate_batch`
hands it every pending request of an external-evaluator step
(os_amd/az.py) with the arrays `_inference` would have built -- observation
rows as float64 (ObservationTensor, flat), legal masks as int64 -- and returns
action-indexed priors and player-0 values.  The evaluator is a pure function
of (observation, mask) (the cache relies on that too), so the device search
fuses each leaf's Evaluate and Prior into one request
(os_az_set_requests OS_AZ_REQUESTS_FUSED).  Results equal the per-state calls
for a model whose outputs do not depend on the batch they are computed in.
"""
import collections

import numpy as np

from . import pyspiel
from .mcts import Evaluator, Float32ModelError


class LRUCache(object):
  """Least-recently-used cache (python/utils/lru_cache.py:38-93)."""

  CacheInfo = collections.namedtuple("CacheInfo", ["hits", "misses", "size", "max_size"])

  def __init__(self, max_size):
    self._max_size = max_size
    self._data = collections.OrderedDict()
    self._hits = 0
    self._misses = 0

  def clear(self):
    self._data.clear()
    self._hits = self._misses = 0

  def make(self, key, fn):
    if key in self._data:
      val = self._data.pop(key)
      self._hits += 1
    else:
      self._misses += 1
      val = fn()
      if len(self._data) >= self._max_size:
        self._data.popitem(last=False)
    self._data[key] = val
    return val

  def info(self):
    return LRUCache.CacheInfo(self._hits, self._misses, len(self._data), self._max_size)


class AlphaZeroEvaluator(Evaluator):
  """An AlphaZero MCTS evaluator over a model with `inference(obs, mask)`
  returning (value [N, 1], policy [N, A]) (evaluator.py:28-83)."""

  # evaluate / prior are one cached inference: a fused device request
  pure_function = True

  def __init__(self, game, model, cache_size=2 ** 16):
    if game.num_players() != 2:
      raise ValueError("Game must be for two players.")
    gt = game.get_type()
    if gt.reward_model != pyspiel.GameType.RewardModel.TERMINAL:
      raise ValueError("Game must have terminal rewards.")
    if gt.dynamics != pyspiel.GameType.Dynamics.SEQUENTIAL:
      raise ValueError("Game must have sequential turns.")
    if gt.chance_mode != pyspiel.GameType.ChanceMode.DETERMINISTIC:
      raise ValueError("Game must be deterministic.")
    self._model = model
    self._cache = LRUCache(cache_size)

  def cache_info(self):
    return self._cache.info()

  def clear_cache(self):
    self._cache.clear()

  def _inference(self, state):
    obs = np.expand_dims(state.observation_tensor(), 0)
    mask = np.expand_dims(state.legal_actions_mask(), 0)
    key = obs.tobytes() + mask.tobytes()
    value, policy = self._cache.make(key, lambda: self._model.inference(obs, mask))
    return value[0, 0], policy[0]

  def evaluate(self, state):
    value, _ = self._inference(state)
    return np.array([value, -value])

  def prior(self, state):
    _, policy = self._inference(state)
    return [(action, policy[action]) for action in state.legal_actions()]

  def evaluate_batch(self, obs, legal, kind):
    """One round of device requests (os_amd/az.py protocol): obs float32
    [N, C, H, W], legal bool [N, A], kind int32 [N] (0 = idle) on the GPU;
    returns (prior float64 [N, A] action-indexed, value float64 [N], player 0).

    Every live row goes through the LRU cache under the key `_inference`
    builds (ObservationTensor as float64 bytes + legal mask as int64 bytes),
    and the misses go to the model as one batch.  A device request is a fused
    Evaluate + Prior, so cache_info() counts one lookup per request where the
    reference's host loop counts two per expanded node (its evaluate, then
    its prior on the second visit).

    The device search accumulates values and scores children in float64.
    The reference's mcts.py inherits the model's dtype instead (NumPy 2 keeps
    float32 in `total_reward += value` and in PUCTValue), so a model with
    float32 outputs is refused here (Float32ModelError) rather than searched
    with different arithmetic.  MCTSBot(backend="auto") runs a lone search
    over this evaluator in the host loop anyway (faster, os_amd/mcts.py
    _use_gpu), whose arithmetic is the reference's for either dtype."""
    import torch
    n, a = legal.shape
    prior = np.zeros((n, a), np.float64)
    value = np.zeros(n, np.float64)
    live = np.nonzero(kind.cpu().numpy())[0]
    if len(live):
      # the arrays _inference builds: ObservationTensor as float64 rows (the
      # tensor's values are exact in float32), legal_actions_mask as int64
      o = obs.reshape(n, -1)[live].to(torch.float64).cpu().numpy()
      m = legal[live].to(torch.int64).cpu().numpy()
      keys = [o[i].tobytes() + m[i].tobytes() for i in range(len(live))]
      got = [None] * len(live)
      miss = []
      for i, k in enumerate(keys):
        if k in self._cache._data:
          got[i] = self._cache.make(k, None)
        else:
          miss.append(i)
      if miss:
        v, p = self._model.inference(o[miss], m[miss])
        v, p = np.asarray(v), np.asarray(p)
        if v.dtype != np.float64 or p.dtype != np.float64:
          raise Float32ModelError(
              "the model returns %s values / %s policies: the device search computes in "
              "float64, the reference mcts.py in the model's dtype" % (v.dtype, p.dtype))
        for j, i in enumerate(miss):
          row = (v[j:j + 1], p[j:j + 1])
          got[i] = self._cache.make(keys[i], lambda row=row: row)
      for i, r in enumerate(live):
        value[r] = got[i][0].reshape(-1)[0]
        prior[r] = got[i][1].reshape(-1)
    dev = obs.device
    return torch.from_numpy(prior).to(dev), torch.from_numpy(value).to(dev)

