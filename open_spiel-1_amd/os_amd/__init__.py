"""os_amd — MI355X-native batched MCTS engine with OpenSpiel's bot API.

Submodules:
  engine   Engine (batched GPU searches / rollouts), make_roots
  pyspiel  load_game / Game / State / MCTSBot / RandomRolloutEvaluator
           (the `pyspiel` surface the Python bot path uses)
  mcts     Evaluator / RandomRolloutEvaluator / SearchNode / MCTSBot
           (open_spiel/python/algorithms/mcts.py drop-in)
  dist     multi-GPU sharding (torch.distributed / RCCL)
"""
from . import _lib  # noqa: F401  (fails loudly if libos_mcts.so is missing)
from .engine import Engine, make_roots  # noqa: F401
