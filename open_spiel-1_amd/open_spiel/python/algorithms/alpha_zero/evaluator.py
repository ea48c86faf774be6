"""open_spiel.python.algorithms.alpha_zero.evaluator drop-in (see os_amd.az_evaluator)."""
from os_amd.az_evaluator import AlphaZeroEvaluator, LRUCache  # noqa: F401
