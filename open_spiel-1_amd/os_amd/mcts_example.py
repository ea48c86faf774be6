"""Bot-vs-bot games with the GPU MCTSBot: examples/mcts_example.cc as a CLI.

  python -m os_amd.mcts_example --game=connect_four --player1=mcts \\
      --player2=mcts --max_simulations=1000 --rollout_count=1 --seed=7 [ACTION ...]

Flags, defaults and printed lines follow mcts_example.cc:32-44, 77-190:
- `mcts` players are pyspiel.MCTSBot (MCTSearch in the gfx950 kernel), all
  seeded Seed() and sharing ONE RandomRolloutEvaluator(rollout_count, Seed())
  (:51-66, :152-158), their rng_ persisting across moves and games;
- `random` players are UniformRandomBot(player, Seed()) (spiel_bots.cc:31-60):
  absl::uniform_int_distribution<int>(0, n - 1) over std::mt19937;
- chance nodes are sampled by SampleAction with the example's own
  std::mt19937(Seed()) (:103-109, spiel.cc:337-366);
- positional arguments are forced opening actions, by ActionToString (:68-96).
Seed() is --seed, or the current time in microseconds when it is 0 (:46-49).
Everything goes to stderr, as in the reference.
"""
import argparse
import sys
import time

import numpy as np

from . import _lib
from . import pyspiel


def _bool(v):
  v = v.lower()
  if v in ("1", "true", "t", "yes", "y"):
    return True
  if v in ("0", "false", "f", "no", "n"):
    return False
  raise argparse.ArgumentTypeError("expected a boolean, got %r" % v)


def parse_args(argv):
  """absl-style flags (mcts_example.cc:32-44): --flag=value, --flag value,
  and --flag / --noflag for booleans."""
  ap = argparse.ArgumentParser(prog="mcts_example", description=__doc__.split("\n")[0])
  ap.add_argument("--game", default="tic_tac_toe")
  ap.add_argument("--player1", default="mcts")
  ap.add_argument("--player2", default="random")
  ap.add_argument("--uct_c", type=float, default=2.0)
  ap.add_argument("--rollout_count", type=int, default=10)
  ap.add_argument("--max_simulations", type=int, default=10000)
  ap.add_argument("--num_games", type=int, default=1)
  ap.add_argument("--max_memory_mb", type=int, default=1000)
  ap.add_argument("--seed", type=int, default=0)
  bools = (("solve", True), ("verbose", False), ("quiet", False))
  for name, default in bools:
    ap.add_argument("--" + name, dest=name, action="store_true", default=default)
    ap.add_argument("--no" + name, dest=name, action="store_false")
  ap.add_argument("initial_actions", nargs="*")
  # absl booleans take a value only as --flag=value (never as a separate word)
  names = {"--" + n for n, _ in bools}
  norm = []
  for arg in argv:
    flag, eq, val = arg.partition("=")
    if eq and flag in names:
      arg = flag if _bool(val) else "--no" + flag[2:]
    norm.append(arg)
  return ap.parse_args(norm)


class _Mt19937:
  """std::mt19937(seed): numpy's legacy MT19937 is the same engine (same
  init_genrand seeding and word stream)."""

  def __init__(self, seed):
    self.rs = np.random.RandomState(seed & 0xFFFFFFFF)

  def word(self):
    # a full-range uint32 draw is one raw word in numpy's legacy generator
    return int(self.rs.randint(0, 2 ** 32, dtype=np.uint32))

  def state(self):
    st = self.rs.get_state()
    return np.array(st[1], np.uint32), np.array([st[2]], np.int32)

  def set_state(self, key, pos):
    self.rs.set_state(("MT19937", key, int(pos[0]), 0, 0.0))


def absl_uniform_int(rng, n):
  """absl::uniform_int_distribution<int>(0, n - 1)(rng) over a 32-bit URBG
  (absl 20200225 Generate: a mask for power-of-two ranges, else Lemire's
  multiply-shift with rejection; SURVEY §8c O3(ii), pinned by the
  negotiation playthrough)."""
  r = n - 1
  bits = rng.word()
  if r & n == 0:
    return bits & r
  prod = bits * n
  if prod & 0xFFFFFFFF < n:
    threshold = ((1 << 32) - n) % n
    while prod & 0xFFFFFFFF < threshold:
      prod = rng.word() * n
  return prod >> 32


class UniformRandomBot(pyspiel.Bot):
  """MakeUniformRandomBot(player, seed) (spiel_bots.cc:31-60, :167-169)."""

  def __init__(self, player_id, seed):
    pyspiel.Bot.__init__(self)
    self._player = player_id
    self._rng = _Mt19937(seed)

  def step(self, state):
    legal = state.legal_actions(self._player)
    return legal[absl_uniform_int(self._rng, len(legal))]


def sample_action(outcomes, rng):
  """SampleAction(outcomes, rng).first (spiel.cc:337-366) on the example's rng."""
  probs = np.array([p for _, p in outcomes], np.float64)
  key, pos = rng.state()
  k = _lib.lib.os_sample_action(probs.ctypes.data, len(outcomes), key.ctypes.data,
                                pos.ctypes.data)
  if k < 0:
    _lib.check(int(k))
  rng.set_state(key, pos)
  return outcomes[k][0]


def _fmt(x):
  return "%g" % x


class Example:
  def __init__(self, args, err=sys.stderr):
    self.args, self.err = args, err

  def seed(self):
    """Seed() (mcts_example.cc:46-49)."""
    if self.args.seed != 0:
      return self.args.seed
    return int(time.time() * 1e6) & 0xFFFFFFFF

  def init_bot(self, kind, game, player, evaluator):
    """InitBot (mcts_example.cc:51-66)."""
    if kind == "random":
      return UniformRandomBot(player, self.seed())
    if kind == "mcts":
      a = self.args
      return pyspiel.MCTSBot(game, evaluator, a.uct_c, a.max_simulations, a.max_memory_mb,
                             a.solve, self.seed(), a.verbose)
    raise pyspiel.SpielError("Bad player type. Known types: mcts, random")

  def play_game(self, game, bots, rng, initial_actions):
    """PlayGame (mcts_example.cc:77-135): (returns, history of action strings)."""
    quiet, err = self.args.quiet, self.err
    state = game.new_initial_state()
    history = []
    for action_str in initial_actions:
      action = next((a for a in state.legal_actions()
                     if state.action_to_string(state.current_player(), a) == action_str),
                    None)
      if action is None:
        raise pyspiel.SpielError("Invalid action: " + action_str)
      history.append(action_str)
      state.apply_action(action)
      if not quiet:
        err.write("Forced action%s\nNext state:\n%s\n" % (action_str, state))
    while not state.is_terminal():
      player = state.current_player()
      if not quiet:
        err.write("player turn: %d\n" % player)
      if state.is_chance_node():
        action = sample_action(state.chance_outcomes(), rng)
        if not quiet:
          err.write("Sampled action: %s\n" % state.action_to_string(player, action))
      else:
        action = bots[player].step(state)
        if not quiet:
          err.write("Chose action: %s\n" % state.action_to_string(player, action))
      for p, b in enumerate(bots):
        if p != player:
          b.inform_action(state, player, action)
      history.append(state.action_to_string(player, action))
      state.apply_action(action)
      if not quiet:
        err.write("State: \n%s\n" % state)
    returns = state.returns()
    err.write("Returns: %s Game actions: %s\n" % (",".join(_fmt(r) for r in returns),
                                                  " ".join(history)))
    return returns, history

  def run(self):
    """main (mcts_example.cc:138-190); returns the summary as a dict."""
    a, err = self.args, self.err
    rng = _Mt19937(self.seed())
    err.write("game: %s\n" % a.game)
    game = pyspiel.load_game(a.game)
    if game.num_players() > 2:
      raise pyspiel.SpielError("mcts_example assumes 2-player games")
    evaluator = pyspiel.RandomRolloutEvaluator(a.rollout_count, self.seed())
    bots = [self.init_bot(a.player1, game, 0, evaluator),
            self.init_bot(a.player2, game, 1, evaluator)]
    histories = {}
    overall_returns, overall_wins = [0.0, 0.0], [0, 0]
    games = []
    for _ in range(a.num_games):
      returns, history = self.play_game(game, bots, rng, a.initial_actions)
      games.append((list(returns), history))
      key = " ".join(history)
      histories[key] = histories.get(key, 0) + 1
      for i, v in enumerate(returns):
        overall_returns[i] += v
        if v > 0:
          overall_wins[i] += 1
    err.write("Number of games played: %d\n" % a.num_games)
    err.write("Number of distinct games played: %d\n" % len(histories))
    err.write("Overall wins: %s\n" % ",".join(str(w) for w in overall_wins))
    err.write("Overall returns: %s\n" % ",".join(_fmt(r) for r in overall_returns))
    err.flush()
    return {"games": games, "overall_wins": overall_wins,
            "overall_returns": overall_returns, "distinct": len(histories)}


def main(argv=None):
  Example(parse_args(sys.argv[1:] if argv is None else argv)).run()
  return 0


if __name__ == "__main__":
  sys.exit(main())
