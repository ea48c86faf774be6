"""A deterministic stand-in for the AlphaZero network (alpha_zero/model.py
`inference(obs, mask) -> (value [N, 1], policy [N, A])`), used to pin the
Python AlphaZero bot wiring (alpha_zero.py:185-192) against the reference.

Test infrastructure only.  Every output row is a function of its own input
row alone and is computed with exact integer arithmetic plus one correctly
rounded division per element, so a batch of N rows gives bit-for-bit the
same rows as N singleton batches (the reference evaluator's calls) on any
host: no BLAS summation order, no transcendental functions.
"""
import numpy as np


class ToyModel(object):

  def __init__(self, obs_size, num_actions, seed=12345, dtype=np.float64):
    # dtype: the outputs' dtype.  float32 stands in for the reference's
    # TensorFlow model (alpha_zero/model.py:339-344 returns float32 arrays),
    # whose dtype mcts.py then carries into its sums under NumPy 2.
    self.dtype = np.dtype(dtype)
    rs = np.random.RandomState(seed)
    # integer weights: obs values are 0 / 1, so every dot product is an exact
    # small integer whatever the summation order
    self.w = rs.randint(-4, 5, size=(obs_size, num_actions + 1)).astype(np.int64)
    self.A = num_actions

  def inference(self, obs, mask):
    o = np.rint(np.asarray(obs, np.float64)).astype(np.int64).reshape(len(obs), -1)
    m = np.asarray(mask).astype(np.int64).reshape(len(obs), self.A)
    z = o @ self.w                                  # exact integers
    num = (np.mod(z[:, :self.A], 7) + 1) * m        # 1..7 on legal actions, 0 elsewhere
    den = num.sum(axis=1, keepdims=True)
    den[den == 0] = 1
    policy = num.astype(np.float64) / den.astype(np.float64)
    value = (np.mod(z[:, self.A:], 21) - 10).astype(np.float64) / 10.0
    return value.astype(self.dtype), policy.astype(self.dtype)
