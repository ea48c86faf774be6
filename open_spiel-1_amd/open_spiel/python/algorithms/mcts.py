"""open_spiel.python.algorithms.mcts drop-in (see os_amd.mcts)."""
from os_amd.mcts import (Evaluator, Float32ModelError, MCTSBot, RandomRolloutEvaluator,  # noqa: F401
                         SearchNode)
