"""`pyspiel`-compatible surface for the five target games.

Mirrors the subset of open_spiel/python/pybind11/pyspiel.cc the Python MCTS
bot path uses (load_game :675-684, State :292-360, Game :362-390, GameType
:215-284, PlayerId :277-281, Bot :487-497, RandomRolloutEvaluator / MCTSBot
:499-524).  Game rules run in libos_mcts.so (the same state machines the
gfx950 kernel runs); `MCTSBot.step` / `.mcts_search` run on the GPU.

Errors follow the reference: SpielFatalError conditions raise RuntimeError
(`SpielError`), unsupported games raise ValueError.
"""
import ctypes
import enum

import numpy as np

from . import _lib
from ._lib import check, get_string, lib

SpielError = _lib.SpielError
INVALID_ACTION = -1


class PlayerId(enum.IntEnum):
  """spiel.h:40-49."""
  INVALID = -3
  TERMINAL = -4
  CHANCE = -1
  SIMULTANEOUS = -2


class TensorLayout(enum.IntEnum):
  HWC = 0
  CHW = 1


class GameType:
  """spiel.h:61-143 (read-only record)."""

  class Dynamics(enum.IntEnum):
    SIMULTANEOUS = 0
    SEQUENTIAL = 1

  class ChanceMode(enum.IntEnum):
    DETERMINISTIC = 0
    EXPLICIT_STOCHASTIC = 1
    SAMPLED_STOCHASTIC = 2

  class Information(enum.IntEnum):
    ONE_SHOT = 0
    PERFECT_INFORMATION = 1
    IMPERFECT_INFORMATION = 2

  class Utility(enum.IntEnum):
    ZERO_SUM = 0
    CONSTANT_SUM = 1
    GENERAL_SUM = 2
    IDENTICAL = 3

  class RewardModel(enum.IntEnum):
    REWARDS = 0
    TERMINAL = 1

  def __init__(self, short_name, long_name, dynamics, chance_mode, information,
               utility, reward_model, max_num_players, min_num_players,
               provides_information_state_string, provides_information_state_tensor,
               provides_observation_string, provides_observation_tensor,
               parameter_specification):
    """Keyword names and order of the pybind constructor (pyspiel.cc:218-229),
    so Python-defined games (python/games/tic_tac_toe.py:293-307) build theirs."""
    self.short_name = short_name
    self.long_name = long_name
    self.dynamics = dynamics
    self.chance_mode = chance_mode
    self.information = information
    self.utility = utility
    self.reward_model = reward_model
    self.max_num_players = max_num_players
    self.min_num_players = min_num_players
    self.provides_information_state_string = provides_information_state_string
    self.provides_information_state_tensor = provides_information_state_tensor
    self.provides_observation_string = provides_observation_string
    self.provides_observation_tensor = provides_observation_tensor
    self.parameter_specification = dict(parameter_specification)
    self.default_loadable = True

  def __repr__(self):
    return "<GameType '%s'>" % self.short_name


def _two_player_type(short_name, long_name, params, info_string=True):
  return GameType(short_name, long_name, GameType.Dynamics.SEQUENTIAL,
                  GameType.ChanceMode.DETERMINISTIC,
                  GameType.Information.PERFECT_INFORMATION,
                  GameType.Utility.ZERO_SUM, GameType.RewardModel.TERMINAL, 2, 2,
                  info_string, False, True, True, params)


_TYPES = {
    0: _two_player_type("tic_tac_toe", "Tic Tac Toe", {}),
    1: _two_player_type("connect_four", "Connect Four", {}),
    2: _two_player_type("breakthrough", "Breakthrough", {"rows": 8, "columns": 8},
                        info_string=False),
    3: _two_player_type("hex", "Hex", {"board_size": 11}),
    4: _two_player_type("go", "Go", {"komi": 7.5, "board_size": 19, "handicap": 0}),
    # pig.cc:42-62 (2..10 players)
    5: GameType("pig", "Pig", GameType.Dynamics.SEQUENTIAL,
                GameType.ChanceMode.EXPLICIT_STOCHASTIC,
                GameType.Information.PERFECT_INFORMATION, GameType.Utility.ZERO_SUM,
                GameType.RewardModel.TERMINAL, 10, 2, False, False, True, True,
                {"players": 2, "horizon": 1000, "winscore": 100, "diceoutcomes": 6}),
}
_PIG = 5


def _game_string(name, params):
  if not params:
    return name
  return "%s(%s)" % (name, ",".join("%s=%s" % (k, params[k]) for k in sorted(params)))


class Game:
  """Game (spiel.h:601-750) backed by libos_mcts.so."""

  def __init__(self, game_string):
    h = ctypes.c_void_p()
    check(lib.os_game_load(game_string.encode(), ctypes.byref(h)))
    self._h = h
    self._info = _lib.GameInfo()
    check(lib.os_game_get_info(h, ctypes.byref(self._info)))
    self._string = get_string(lib.os_game_to_string, h)
    self.game_string = game_string

  def __del__(self):
    if getattr(self, "_h", None) and self._h.value:
      lib.os_game_free(self._h)

  def new_initial_state(self):
    return State(self)

  def num_distinct_actions(self):
    return self._info.num_distinct_actions

  def policy_tensor_shape(self):
    return [self._info.num_distinct_actions]

  def max_chance_outcomes(self):
    # pig.h:88: diceoutcomes (the largest chance branching); 0 for the others
    return self._pig_dice() if self._info.kind == _PIG else 0

  def num_players(self):
    return self._info.num_players

  def min_utility(self):
    return self._info.min_utility

  def max_utility(self):
    return self._info.max_utility

  def utility_sum(self):
    return self._info.utility_sum

  def max_game_length(self):
    return self._info.max_game_length

  def observation_tensor_shape(self):
    shape = np.zeros(3, np.int32)
    lib.os_game_observation_shape(self._h, shape.ctypes.data)
    if self._info.kind == _PIG:  # pig.cc:119-122: [1 + players, winscore + 1]
      return [int(shape[0]), int(shape[2])]
    return [int(x) for x in shape]

  def observation_tensor_size(self):
    return int(lib.os_game_observation_shape(self._h, None))

  def observation_tensor_layout(self):
    return TensorLayout.CHW

  def get_type(self):
    return _TYPES[self._info.kind]

  # hex / go sides the device engine runs: every search up to 11 x 11 (B128
  # bitboards); up to 19 x 19 (every board the games load) with C++-policy
  # searches (k_lsearch over B384 bitboards).
  DEVICE_MAX_SIDE = 11
  DEVICE_MAX_SIDE_CPP = 19

  def on_device(self, numpy_policy=False):
    """Whether the GPU engine can search this game (else: host State API);
    numpy_policy: for the Python MCTSBot's RandomState streams."""
    k, n = self._info.kind, self._info.rows
    if k in (3, 4):
      return n <= (Game.DEVICE_MAX_SIDE if numpy_policy else Game.DEVICE_MAX_SIDE_CPP)
    return True

  def get_parameters(self):
    k = self._info.kind
    if k == 2:
      return {"columns": self._info.cols, "rows": self._info.rows}
    if k == 3:
      return {"board_size": self._info.rows}
    if k == 4:
      return {"board_size": self._info.rows, "handicap": self._info.handicap,
              "komi": self._info.komi}
    if k == _PIG:
      return {"diceoutcomes": self._pig_dice(), "horizon": self._info.max_game_length,
              "players": self._info.num_players, "winscore": self._info.cols - 1}
    return {}

  def _pig_dice(self):
    st = self.new_initial_state()
    st.apply_action(0)
    return len(st.chance_outcomes())

  def deserialize_state(self, s):
    """Inverse of State.serialize() (history form, spiel.cc:375-420)."""
    st = self.new_initial_state()
    for line in s.split("\n"):
      if line:
        st.apply_action(int(line))
    return st

  def __str__(self):
    return self._string

  def __eq__(self, other):
    return isinstance(other, Game) and str(self) == str(other)

  def __hash__(self):
    return hash(self._string)

  def __reduce__(self):
    return (load_game, (self.game_string,))


def load_game(name, params=None):
  """pyspiel.load_game(name[, params]) (pyspiel.cc:675-684)."""
  return Game(_game_string(name, params) if params else name)


class State:
  """State (spiel.h:173-592) backed by libos_mcts.so host state machines."""

  __slots__ = ("_game", "_h")

  def __init__(self, game, handle=None):
    self._game = game
    if handle is None:
      handle = ctypes.c_void_p()
      check(lib.os_state_new(game._h, ctypes.byref(handle)))
    self._h = handle

  def __del__(self):
    h = getattr(self, "_h", None)
    if h is not None and h.value:
      lib.os_state_free(h)

  def clone(self):
    h = ctypes.c_void_p()
    check(lib.os_state_clone(self._h, ctypes.byref(h)))
    return State(self._game, h)

  def __deepcopy__(self, memo):
    return self.clone()

  def __copy__(self):
    return self.clone()

  def child(self, action):
    c = self.clone()
    c.apply_action(action)
    return c

  def current_player(self):
    return int(lib.os_state_current_player(self._h))

  def is_terminal(self):
    return bool(lib.os_state_is_terminal(self._h))

  def is_chance_node(self):
    return bool(lib.os_state_is_chance_node(self._h))

  def is_simultaneous_node(self):
    return False

  def is_player_node(self):
    return self.current_player() >= 0

  def apply_action(self, action):
    check(lib.os_state_apply(self._h, int(action)))

  def legal_actions(self, player=None):
    if player is not None and player != self.current_player():
      return []
    cap = max(self._game._info.num_distinct_actions, self._game._info.max_children)
    buf = np.zeros(cap, np.int64)
    n = lib.os_state_legal_actions(self._h, buf.ctypes.data, cap)
    if n > cap:  # chance outcomes can outnumber the distinct actions (pig)
      buf = np.zeros(n, np.int64)
      n = lib.os_state_legal_actions(self._h, buf.ctypes.data, n)
    return [int(a) for a in buf[:n]]

  def legal_actions_mask(self, player=None):
    mask = [0] * self._game.num_distinct_actions()
    for a in self.legal_actions(player):
      mask[a] = 1
    return mask

  def action_to_string(self, arg0, arg1=None):
    if arg1 is None:
      player, action = self.current_player(), arg0
    else:
      player, action = arg0, arg1
    return get_string(lib.os_state_action_to_string, self._h, int(player),
                      int(action))

  def string_to_action(self, arg0, arg1=None):
    if arg1 is None:
      player, s = self.current_player(), arg0
    else:
      player, s = arg0, arg1
    for a in self.legal_actions():
      if self.action_to_string(player, a) == s:
        return a
    raise SpielError("Illegal move: %s" % s)

  def returns(self):
    r = np.zeros(self._game._info.num_players, np.float64)
    lib.os_state_returns(self._h, r.ctypes.data)
    return [float(x) for x in r]

  def rewards(self):
    return self.returns() if self.is_terminal() else [0.0] * self.num_players()

  def player_return(self, player):
    return self.returns()[player]

  def player_reward(self, player):
    return self.rewards()[player]

  def history(self):
    buf = np.zeros(512, np.int64)
    n = lib.os_state_history(self._h, buf.ctypes.data, 512)
    if n > 512:
      buf = np.zeros(n, np.int64)
      lib.os_state_history(self._h, buf.ctypes.data, n)
    return [int(a) for a in buf[:n]]

  def history_str(self):
    return " ".join(str(a) for a in self.history())

  def information_state_string(self, player=None):
    return self.history_str()

  def observation_string(self, player=None):
    return str(self)

  def observation_tensor(self, player=None):
    """State.observation_tensor([player]) (pyspiel.cc:292-360): flat list of
    floats in ObservationTensorShape (CHW) order."""
    p = self.current_player() if player is None else int(player)
    if p < 0:
      p = 0  # terminal: the reference's default player argument is 0 there
    n = self._game.observation_tensor_size()
    out = np.zeros(n, np.float32)
    rc = lib.os_state_observation_tensor(self._h, p, out.ctypes.data, n)
    if rc < 0:
      check(int(rc))
    return [float(x) for x in out]

  def chance_outcomes(self):
    """ChanceOutcomes() (spiel.h:322-327): [(action, probability)] in outcome
    order; [] at a decision node."""
    cap = max(self._game._info.num_distinct_actions, self._game._info.max_children)
    acts = np.zeros(cap, np.int64)
    probs = np.zeros(cap, np.float64)
    n = lib.os_state_chance_outcomes(self._h, acts.ctypes.data, probs.ctypes.data, cap)
    if n > cap:
      acts = np.zeros(n, np.int64)
      probs = np.zeros(n, np.float64)
      n = lib.os_state_chance_outcomes(self._h, acts.ctypes.data, probs.ctypes.data, n)
    return [(int(acts[i]), float(probs[i])) for i in range(n)]

  def num_distinct_actions(self):
    return self._game.num_distinct_actions()

  def num_players(self):
    return self._game.num_players()

  def get_game(self):
    return self._game

  def get_type(self):
    return self._game.get_type()

  def serialize(self):
    h = self.history()
    return "".join("%d\n" % a for a in h)

  def __str__(self):
    return get_string(lib.os_state_to_string, self._h)

  def __reduce__(self):
    return (_restore_state, (self._game.game_string, self.history()))


def _restore_state(game_string, history):
  st = load_game(game_string).new_initial_state()
  for a in history:
    st.apply_action(a)
  return st


class Bot:
  """pyspiel.Bot (spiel_bots.h; pybind trampoline pyspiel.cc:82-178)."""

  def __init__(self):
    pass

  def step(self, state):
    raise NotImplementedError

  def step_with_policy(self, state):
    a = self.step(state)
    return [(a, 1.0)], a

  def restart(self):
    pass

  def restart_at(self, state):
    pass

  def inform_action(self, state, player_id, action):
    pass

  def provides_force_action(self):
    return False

  def force_action(self, state, action):
    raise SpielError("force_action not implemented")

  def provides_policy(self):
    return False

  def get_policy(self, state):
    raise SpielError("get_policy not implemented")


class ChildSelectionPolicy(enum.IntEnum):
  UCT = 0
  PUCT = 1


def _mt_key(seed):
  """std::mt19937(seed) state as (key[624], pos=624) (== numpy legacy)."""
  st = np.random.RandomState(seed & 0xFFFFFFFF).get_state()
  return np.array(st[1], dtype=np.uint32), int(st[2])


class Evaluator:
  """pyspiel.Evaluator (no Python trampoline in the reference either)."""


class RandomRolloutEvaluator(Evaluator):
  """RandomRolloutEvaluator(n_rollouts, seed) (mcts.h:92-106).

  Holds its std::mt19937 stream; a bot using it advances the stream on the GPU
  and writes it back, so an evaluator shared by several bots interleaves its
  random numbers in call order exactly as in the reference (mcts_test.cc:39).
  """

  def __init__(self, n_rollouts, seed):
    self.n_rollouts = int(n_rollouts)
    self._state = _mt_key(seed)


def evaluate_bots(state, bots, seed):
  """pyspiel.evaluate_bots(state, bots, seed) (pyspiel.cc:724; EvaluateBots,
  evaluate_bots.cc:24-61): plays to the end from `state`, chance nodes sampled
  by SampleAction with a std::mt19937(seed) (absl::Uniform(rng, 0.0, 1.0),
  os_sample_action); every other bot is informed of each move.  Returns
  state.returns()."""
  key, pos = _mt_key(seed)
  pos_a = np.array([pos], np.int32)
  if state.history():
    for b in bots:
      b.restart_at(state)
  else:
    for b in bots:
      b.restart()
  while not state.is_terminal():
    if state.is_chance_node():
      outs = state.chance_outcomes()
      probs = np.array([p for _, p in outs], np.float64)
      k = lib.os_sample_action(probs.ctypes.data, len(outs), key.ctypes.data,
                               pos_a.ctypes.data)
      if k < 0:
        check(int(k))
      action = outs[k][0]
      for b in bots:
        b.inform_action(state, PlayerId.CHANCE, action)
    else:
      mover = state.current_player()
      action = bots[mover].step(state)
      for p, b in enumerate(bots):
        if p != mover:
          b.inform_action(state, mover, action)
    state.apply_action(action)
  return state.returns()


_ENGINES = {}


def _engine_for(game):
  from .engine import Engine
  key = str(game)
  eng = _ENGINES.get(key)
  if eng is None:
    eng = Engine(game.game_string, device=0)
    _ENGINES[key] = eng
  return eng


_AZ_SEARCHES = {}


def _az_search_for(game):
  """The external-evaluator search (os_amd/az.py) a Python MCTSBot with a
  batched evaluator runs on, one per game."""
  from .az import ExternalEvaluatorSearch
  key = str(game)
  s = _AZ_SEARCHES.get(key)
  if s is None:
    s = ExternalEvaluatorSearch(game.game_string, device=0)
    _AZ_SEARCHES[key] = s
  return s


class MCTSBot(Bot):
  """pyspiel.MCTSBot (mcts.h:139-208; pyspiel.cc:512-524) on the GPU.

  Every `step` / `mcts_search` runs MCTSBot::MCTSearch (mcts.cc:325-428) in
  the gfx950 kernel, continuing this bot's and its evaluator's MT19937
  streams, so a sequence of calls is bit-exact with the C++ bot.
  """

  def __init__(self, game, evaluator, uct_c, max_simulations, max_memory_mb,
               solve, seed, verbose,
               child_selection_policy=ChildSelectionPolicy.UCT):
    Bot.__init__(self)
    if not isinstance(evaluator, RandomRolloutEvaluator):
      raise ValueError("the GPU MCTSBot supports RandomRolloutEvaluator only "
                       "(pyspiel.Evaluator has no Python trampoline either)")
    if child_selection_policy not in (ChildSelectionPolicy.UCT, ChildSelectionPolicy.PUCT):
      raise ValueError("unknown child_selection_policy")
    gt = game.get_type()
    if gt.reward_model != GameType.RewardModel.TERMINAL:
      raise SpielError("Game must have terminal rewards.")
    if gt.dynamics != GameType.Dynamics.SEQUENTIAL:
      raise SpielError("Game must have sequential turns.")
    self._game = game
    self._evaluator = evaluator
    self.uct_c = float(uct_c)
    self.max_simulations = int(max_simulations)
    self.max_memory_mb = int(max_memory_mb)
    self.solve = bool(solve)
    self.verbose = bool(verbose)
    self._state = _mt_key(seed)
    self._select = (_lib.SELECT_PUCT if child_selection_policy == ChildSelectionPolicy.PUCT
                    else _lib.SELECT_UCT)

  def _run(self, state):
    eng = _engine_for(self._game)
    o, self._state, self._evaluator._state = eng.mcts_stateful(
        state.history(), self._state, self._evaluator._state,
        uct_c=self.uct_c, max_simulations=self.max_simulations,
        n_rollouts=self._evaluator.n_rollouts, max_memory_mb=self.max_memory_mb,
        solve=self.solve, policy=_lib.POLICY_CPP, child_selection=self._select)
    return o, eng

  def mcts_search(self, state):
    """MCTSearch (mcts.cc:325-428): the root of the search tree (its nodes are
    built from the device arena as they are read)."""
    from .mcts import tree_to_search_nodes
    _, eng = self._run(state)
    return tree_to_search_nodes(eng.tree(0), state, self._game, root_action=-1)

  def step(self, state):
    """MCTSBot::Step (mcts.cc:219-248): BestChild's action, taken from the
    engine (no tree is exported unless `verbose`)."""
    import time
    t0 = time.time()
    o, eng = self._run(state)
    if o["nchild"][0] <= 0:
      raise SpielError("MCTSBot: root has no children")
    best = int(o["best_action"][0])
    if self.verbose:
      self._print_verbose(state, eng, o, time.time() - t0, best)
    return best

  _SEARCH_NODE_BYTES = 80  # sizeof(SearchNode) in the reference build

  def _print_verbose(self, state, eng, o, seconds, best):
    """The report MCTSBot::Step writes to stderr when verbose (mcts.cc:226-245;
    SearchNode::ToString / ChildrenStr :143-175)."""
    import sys
    from .mcts import tree_to_search_nodes
    root = tree_to_search_nodes(eng.tree(0), state, self._game, root_action=-1)
    nodes = int(o["nodes"][0])
    n = root.explore_count
    err = sys.stderr
    err.write("Finished %d sims in %.3f secs, %.1f sims/s, tree size: %d nodes / %d mb.\n"
              % (n, seconds, n / max(seconds, 1e-12), nodes,
                 nodes * self._SEARCH_NODE_BYTES // (1 << 20)))
    err.write("Root:\n%s\n" % _node_string(root, state))
    err.write("Children:\n%s\n" % _children_string(root, state))
    chosen = next(c for c in root.children if c.action == best)
    if chosen.children:
      err.write("Children of chosen:\n%s\n" % _children_string(chosen, state.child(best)))
    err.flush()

  def step_with_policy(self, state):
    a = self.step(state)
    return [(a, 1.0)], a


def _node_string(node, state):
  """SearchNode::ToString(state) (mcts.cc:162-175): `state` is the node's
  parent position, whose ActionToString names the node's action."""
  name = ("none" if node.action is None or node.action == -1
          else state.action_to_string(node.player, node.action))
  value = node.total_reward / node.explore_count if node.explore_count else 0.0
  if node.outcome is None:
    outcome = "none"
  else:
    outcome = "%4.1f" % node.outcome[0 if node.player == PlayerId.CHANCE else node.player]
  return ("%6s: player: %d, prior: %5.3f, value: %6.3f, sims: %5d, outcome: %s, "
          "%3d children" % (name, node.player, node.prior, value, node.explore_count,
                            outcome, len(node.children)))


def _children_string(node, state):
  """SearchNode::ChildrenStr (mcts.cc:143-160): children best-first by
  CompareFinal (outcome, explore_count, total_reward), one line each."""
  def key(c):
    proven = 0.0 if c.outcome is None else c.outcome[0 if c.player == PlayerId.CHANCE
                                                     else c.player]
    return (proven, c.explore_count, c.total_reward)
  ordered = sorted(node.children, key=key, reverse=True)
  return "".join(_node_string(c, state) + "\n" for c in ordered)
