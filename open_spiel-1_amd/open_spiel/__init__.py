"""Namespace shim so `from open_spiel.python.algorithms import mcts` resolves to
the MI355X-backed drop-in (os_amd.mcts)."""
