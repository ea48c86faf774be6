"""Drop-in `pyspiel` module: `import pyspiel` with open_spiel-1_amd/ on
sys.path gives the GPU-backed subset implemented by os_amd.pyspiel."""
from os_amd.pyspiel import *  # noqa: F401,F403
from os_amd.pyspiel import (Bot, ChildSelectionPolicy, Evaluator, Game,  # noqa: F401
                            GameType, INVALID_ACTION, MCTSBot, PlayerId,
                            RandomRolloutEvaluator, SpielError, State,
                            TensorLayout, load_game)
