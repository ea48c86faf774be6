"""Bot-vs-bot game loop (python/algorithms/evaluate_bots.py:24-49 semantics)."""
from os_amd import pyspiel


def evaluate_bots(state, bots, rng):
  """Plays `bots` against each other from `state`; returns the returns."""
  for bot in bots:
    bot.restart_at(state)
  while not state.is_terminal():
    if state.is_chance_node():
      outcomes, probs = zip(*state.chance_outcomes())
      action = rng.choice(outcomes, p=probs)
      for bot in bots:
        bot.inform_action(state, pyspiel.PlayerId.CHANCE, action)
      state.apply_action(action)
      continue
    mover = state.current_player()
    action = bots[mover].step(state)
    for i, bot in enumerate(bots):
      if i != mover:
        bot.inform_action(state, mover, action)
    state.apply_action(action)
  return state.returns()
