"""GPU parity: the gfx950 kernels through the C-ABI against the oracle.

Integer / index outputs must be bit-exact; child rewards are f64 sums of
integer-valued (n_rollouts == 1) or rational (n_rollouts > 1) returns and are
compared bit-exactly too (same operation order as mcts.cc)."""
import json
import math
import os

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")

CASES = [
    ("tic_tac_toe", 64, 1000, 4),
    ("connect_four", 128, 1024, 8),
    ("breakthrough", 16, 512, 6),
    ("breakthrough(rows=6,columns=5)", 16, 300, 6),
    ("breakthrough(rows=4,columns=3)", 16, 300, 2),  # narrow boards: edge columns,
    ("breakthrough(rows=5,columns=2)", 16, 200, 2),  # short games, solver proofs
    ("hex(board_size=5)", 96, 400, 6),  # > 64 roots: every lane of a wave64 (block 64)
    ("hex", 72, 200, 4),
    ("go(board_size=7,komi=4.5)", 8, 200, 6),
    ("go(board_size=9)", 8, 160, 8),
    ("go(board_size=11,komi=6.5)", 6, 60, 6),  # 121 points: the lane neighbourhoods' top dword
    ("go(board_size=6)", 8, 120, 4),
]


@pytest.fixture(scope="module")
def E(require_gpu):
  from os_amd import engine
  return engine


def _cmp(E, got, ref):
  bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(got[k], ref[k])]
  assert not bad, bad


# Both search kernels on every game: k_wsearch (one wave per search) and
# k_mcts (one lane per search; its workgroup width `block` only matters there).
LAYOUTS = [("wave", 0), ("lane", 16), ("lane", 64)]


@pytest.mark.parametrize("gs,R,sims,plies", CASES)
@pytest.mark.parametrize("layout,block", LAYOUTS)
def test_search_bit_exact(E, gs, R, sims, plies, layout, block):
  from os_amd import _lib
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 1000, plies)
  bs = np.arange(R, dtype=np.uint32)
  es = bs + np.uint32(1 << 20)
  lay = _lib.LAYOUT_WAVE if layout == "wave" else _lib.LAYOUT_LANE
  got = eng.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                       block_size=block, layout=lay)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                              max_children=eng.max_children, threads=8)
  _cmp(E, got, ref)


@pytest.mark.parametrize("gs", ["tic_tac_toe", "connect_four", "hex(board_size=5)",
                                "go(board_size=5,komi=0.5)"])
@pytest.mark.parametrize("n_rollouts,solve,uct_c", [(3, True, math.sqrt(2)),
                                                    (1, False, 2.0), (2, False, 0.5)])
def test_search_variants(E, gs, n_rollouts, solve, uct_c):
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, 32, 1000, 4)
  bs = np.arange(32, dtype=np.uint32) * 3 + 1
  es = bs + np.uint32(99)
  kw = dict(uct_c=uct_c, max_simulations=500, n_rollouts=n_rollouts, solve=solve)
  got = eng.mcts_batch(acts, offs, bs, es, **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children,
                              threads=8, **kw)
  _cmp(E, got, ref)


# go's lane layout (k_lsearch: one lane per search, every per-search buffer
# batch-SoA in HBM): > 64 searches so every lane of a wave64 runs one, all
# board sizes the device takes, f64 rewards, solver off, a GC budget.
@pytest.mark.parametrize("gs,R,sims,plies,kw", [
    ("go(board_size=5,komi=0.5)", 96, 300, 4, {}),
    ("go(board_size=7,komi=4.5)", 80, 200, 6, dict(n_rollouts=2, solve=False, uct_c=0.9)),
    ("go(board_size=9)", 72, 160, 8, {}),
    ("go(board_size=9)", 40, 120, 20, dict(n_rollouts=3)),
    ("go(board_size=11,komi=6.5)", 66, 80, 6, {}),
    ("go(board_size=5,komi=0.5)", 70, 2000, 2, dict(max_memory_mb=1)),
])
def test_go_lane_layout_bit_exact(E, gs, R, sims, plies, kw):
  from os_amd import _lib
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 4242, plies)
  bs = np.arange(R, dtype=np.uint32) * 7 + 2
  es = bs + np.uint32(1 << 20)
  kw = dict(dict(uct_c=2.0, max_simulations=sims), **kw)
  got = eng.mcts_batch(acts, offs, bs, es, layout=_lib.LAYOUT_LANE, **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children, threads=8,
                              **kw)
  _cmp(E, got, ref)
  if kw.get("max_memory_mb") == 1:
    assert eng.stats()["gc_runs"] > 0


def test_garbage_collection_on_device(E):
  gs = "go(board_size=9)"
  eng = E.Engine(gs)
  acts, offs = np.zeros(0, np.int64), np.array([0, 0], np.int64)
  kw = dict(uct_c=2.0, max_simulations=700, max_memory_mb=1)
  got = eng.mcts_batch(acts, offs, [5], [6], **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, [5], [6], max_children=eng.max_children,
                              **kw)
  _cmp(E, got, ref)


def test_solver_known_answers_on_device(E):
  with open(os.path.join(GOLD, "reference_probes.json")) as f:
    cases = json.load(f)["solver_cases"]["cases"]
  import pyspiel
  game = pyspiel.load_game("tic_tac_toe")
  eng = E.Engine("tic_tac_toe")
  for case in cases:
    st = game.new_initial_state()
    for lab in case["actions"]:
      st.apply_action(st.string_to_action(lab))
    h = st.history()
    o = eng.mcts_batch(np.array(h, np.int64), np.array([0, len(h)]), [42], [42],
                       uct_c=math.sqrt(2), max_simulations=10000, n_rollouts=20,
                       max_memory_mb=10, solve=True)
    assert o["root_out"][0] == case["root_outcome"], case["name"]
    if "best_in" in case:
      assert st.action_to_string(int(o["best_action"][0])) in case["best_in"]


def test_recorded_reference_outputs_on_device(E):
  with open(os.path.join(GOLD, "reference_probes.json")) as f:
    case = json.load(f)["cpp_mcts"][0]
  eng = E.Engine(case["game"])
  o = eng.mcts_batch(np.zeros(0, np.int64), np.array([0, 0]), [case["bot_seed"]],
                     [case["eval_seed"]], uct_c=case["uct_c"],
                     max_simulations=case["max_simulations"])
  nc = o["nchild"][0]
  kids = [[int(a), int(n)] for a, n in zip(o["child_action"][0][:nc],
                                           o["child_n"][0][:nc])]
  assert kids == case["children_in_order"]
  assert o["root_w"][0] == case["root_w"]


# The wave layout plays hex playouts lane-parallel (os_wave.h
# hex_rollout_lanes): every board size it takes, roots deep and shallow, MT
# blocks crossed mid-playout by long searches, n_rollouts > 1.
@pytest.mark.parametrize("gs,R,sims,plies,nr", [
    ("hex(board_size=3)", 32, 300, 2, 1),
    ("hex(board_size=5)", 32, 400, 6, 1), ("hex(board_size=7)", 16, 500, 10, 2),
    ("hex", 16, 600, 4, 1), ("hex", 4, 2048, 0, 1), ("hex", 8, 300, 60, 3)])
def test_hex_wave_lane_playouts_bit_exact(E, gs, R, sims, plies, nr):
  from os_amd import _lib
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 1000, plies)
  bs = np.arange(R, dtype=np.uint32) + 11
  es = bs + np.uint32(1 << 20)
  kw = dict(uct_c=2.0, max_simulations=sims, n_rollouts=nr)
  got = eng.mcts_batch(acts, offs, bs, es, layout=_lib.LAYOUT_WAVE, **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children,
                              threads=8, **kw)
  _cmp(E, got, ref)


@pytest.mark.parametrize("gs,plies", [("hex", 0), ("hex", 40), ("hex(board_size=4)", 3),
                                      ("hex(board_size=3)", 0)])
def test_hex_wave_rollouts_bit_exact(E, gs, plies):
  from os_amd import _lib
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, 1, 77, plies)
  seeds = np.arange(4096, dtype=np.uint32) * 7 + 3
  for nr in (1, 4):
    got = eng.rollouts(acts, seeds, n_rollouts=nr, layout=_lib.LAYOUT_WAVE)
    ref = O.Game(gs).rollouts(acts, seeds, n_rollouts=nr)
    assert np.array_equal(got, ref), nr


@pytest.mark.parametrize("gs,plies", [("connect_four", 10), ("breakthrough", 20),
                                      ("hex", 30), ("go(board_size=9)", 0),
                                      ("go(board_size=9)", 40)])
def test_rollouts_bit_exact(E, gs, plies):
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, 1, 77, plies)
  seeds = np.arange(2048, dtype=np.uint32) * 13 + 5
  got = eng.rollouts(acts, seeds)
  ref = O.Game(gs).rollouts(acts, seeds)
  assert np.array_equal(got, ref)


def test_full_c2_workload_properties_and_prefix_parity(E):
  """BASELINE configs[1] at full size: 4096 roots x 1024 sims."""
  gs, R, sims = "connect_four", 4096, 1024
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 1000, 8)
  bs = np.arange(R, dtype=np.uint32)
  es = bs + np.uint32(1 << 20)
  o = eng.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims)
  nc = o["nchild"]
  child_sum = np.array([o["child_n"][r, :nc[r]].sum() for r in range(R)])
  assert np.array_equal(child_sum, o["root_n"] - 1)     # sim 0 visits the root
  assert (o["root_n"] <= sims).all() and (o["root_n"] >= 2).all()
  early = o["root_n"] < sims                              # solved / single child
  assert ((o["root_out"][early] != 2) | (nc[early] == 1)).all()
  for r in range(0, R, 97):
    assert o["best_action"][r] in o["child_action"][r, :nc[r]]
  sub = 96
  ref = O.Game(gs).mcts_batch(acts[:offs[sub]], offs[:sub + 1], bs[:sub], es[:sub],
                              uct_c=2.0, max_simulations=sims, max_children=7,
                              threads=8)
  for k in E.OUTPUT_KEYS:
    assert np.array_equal(o[k][:sub], ref[k]), k


def test_full_c3_width_properties_and_prefix_parity(E):
  """BASELINE configs[2] at full width: 65536 breakthrough(8x8) roots through
  the automatic layout (the kernel C3 runs in production), sims reduced so the
  oracle can check a 64-root prefix bit-exactly."""
  gs, R, sims = "breakthrough(rows=8,columns=8)", 65536, 128
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 1000, 6)
  bs = np.arange(R, dtype=np.uint32)
  es = bs + np.uint32(1 << 20)
  o = eng.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims)
  nc = o["nchild"]
  child_sum = np.array([o["child_n"][r, :nc[r]].sum() for r in range(R)])
  assert np.array_equal(child_sum, o["root_n"] - 1)
  assert (o["root_n"] <= sims).all() and (o["root_n"] >= 2).all()
  early = o["root_n"] < sims
  assert ((o["root_out"][early] != 2) | (nc[early] == 1)).all()
  for r in range(0, R, 1021):
    assert o["best_action"][r] in o["child_action"][r, :nc[r]]
  for lo in (0, R - 64):  # first and last 64 roots (first and last workgroups)
    sl = slice(lo, lo + 64)
    ref = O.Game(gs).mcts_batch(acts[offs[lo]:offs[lo + 64]], offs[lo:lo + 65] - offs[lo],
                                bs[sl], es[sl], uct_c=2.0, max_simulations=sims,
                                max_children=eng.max_children, threads=8)
    for k in E.OUTPUT_KEYS:
      assert np.array_equal(o[k][sl], ref[k]), (lo, k)


def test_python_drop_in_gpu_path(E):
  """os_amd.mcts on the GPU == the reference mcts.py vector, and the shared
  RandomState continues exactly as after the host loop."""
  import pyspiel
  from open_spiel.python.algorithms import mcts
  with open(os.path.join(GOLD, "reference_probes.json")) as f:
    case = json.load(f)["python_mcts"][0]
  game = pyspiel.load_game(case["game"])
  rs_gpu = np.random.RandomState(case["seed"])
  bot = mcts.MCTSBot(game, case["uct_c"], case["max_simulations"],
                     mcts.RandomRolloutEvaluator(1, rs_gpu), random_state=rs_gpu,
                     backend="hip")
  root = bot.mcts_search(game.new_initial_state())
  got = sorted([c.action, c.explore_count, c.total_reward] for c in root.children)
  assert got == [[a, n, float(w)] for a, n, w in case["children_sorted"]]
  rs_host = np.random.RandomState(case["seed"])
  hb = mcts.MCTSBot(game, case["uct_c"], case["max_simulations"],
                    mcts.RandomRolloutEvaluator(1, rs_host), random_state=rs_host,
                    backend="host")
  hb.mcts_search(game.new_initial_state())
  assert rs_gpu.randint(2**31) == rs_host.randint(2**31)
  # a second search continues both streams identically
  r2 = sorted((c.action, c.explore_count) for c in bot.mcts_search(
      game.new_initial_state()).children)
  h2 = sorted((c.action, c.explore_count) for c in hb.mcts_search(
      game.new_initial_state()).children)
  assert r2 == h2


def test_cpp_style_bot_plays(E):
  import pyspiel
  from open_spiel.python.algorithms import evaluate_bots
  game = pyspiel.load_game("tic_tac_toe")
  ev = pyspiel.RandomRolloutEvaluator(20, 42)
  bots = [pyspiel.MCTSBot(game, ev, math.sqrt(2), 100, 5, True, 42, False)
          for _ in range(2)]
  v = evaluate_bots.evaluate_bots(game.new_initial_state(), bots, np.random)
  assert v[0] + v[1] == 0
  # first search of a fresh bot == the oracle's fresh search
  bot = pyspiel.MCTSBot(game, pyspiel.RandomRolloutEvaluator(1, 7), 2.0, 300,
                        1000, True, 3, False)
  root = bot.mcts_search(game.new_initial_state())
  ref = O.Game("tic_tac_toe").mcts_batch(np.zeros(0, np.int64), np.array([0, 0]),
                                         [3], [7], uct_c=2.0, max_simulations=300)
  assert [c.action for c in root.children] == list(ref["child_action"][0][:9])
  assert [c.explore_count for c in root.children] == list(ref["child_n"][0][:9])


@pytest.mark.gpu
@pytest.mark.parametrize("gs", ["tic_tac_toe", "connect_four", "hex(board_size=5)",
                                "breakthrough(rows=5,columns=5)"])
@pytest.mark.parametrize("uct_c,solve", [(0.0, True), (0.0, False), (0.01, True),
                                         (10.0, False), (2.0, False)])
def test_uct_screen_ties_and_near_ties(E, gs, uct_c, solve):
  """The wave kernel's f32 UCT screen (os_wave.h uct_argmax_screen) against the
  oracle where its fallback matters: uct_c = 0 makes equal ratios w/n from
  different (n, w) exact ties (1/2 vs 2/4), a tiny uct_c makes them near ties,
  a large one stretches the bound."""
  from os_amd import _lib
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, 24, 1000, 3)
  bs = np.arange(24, dtype=np.uint32) * 7 + 5
  es = bs + np.uint32(1 << 20)
  kw = dict(uct_c=uct_c, max_simulations=600, solve=solve)
  got = eng.mcts_batch(acts, offs, bs, es, layout=_lib.LAYOUT_WAVE, **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children, threads=8,
                              **kw)
  _cmp(E, got, ref)


# ChildSelectionPolicy::PUCT with the random-rollout evaluator (mcts.cc:102-111,
# uniform Prior :73-86): both search kernels, n_rollouts > 1 (f64 rewards),
# solver on and off.  The numpy policy's PUCT is pinned by the reference-Python
# fixtures (tests/golden/python_mcts_puct_*.json, test_python_goldens.py).
@pytest.mark.parametrize("gs,R,sims,plies", [
    ("tic_tac_toe", 32, 600, 4), ("connect_four", 64, 700, 8),
    ("breakthrough(rows=6,columns=6)", 16, 300, 4), ("hex(board_size=5)", 24, 400, 6),
    ("hex", 4, 300, 4), ("go(board_size=7,komi=4.5)", 6, 150, 6)])
@pytest.mark.parametrize("layout", ["wave", "lane"])
@pytest.mark.parametrize("nr,solve,uct_c", [(1, True, 2.0), (2, False, 0.7)])
def test_puct_bit_exact(E, gs, R, sims, plies, layout, nr, solve, uct_c):
  from os_amd import _lib
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, R, 1000, plies)
  bs = np.arange(R, dtype=np.uint32) * 3 + 1
  es = bs + np.uint32(1 << 20)
  kw = dict(uct_c=uct_c, max_simulations=sims, n_rollouts=nr, solve=solve)
  lay = _lib.LAYOUT_WAVE if layout == "wave" else _lib.LAYOUT_LANE
  got = eng.mcts_batch(acts, offs, bs, es, layout=lay, child_selection=_lib.SELECT_PUCT, **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children, threads=8,
                              puct=True, **kw)
  _cmp(E, got, ref)


def test_puct_pig_chance_search(E):
  from os_amd import _lib
  gs = "pig(horizon=30,winscore=10)"
  eng = E.Engine(gs)
  acts, offs = E.make_roots(gs, 32, 1000, 6)
  bs = np.arange(32, dtype=np.uint32) + 9
  es = bs + np.uint32(1 << 20)
  kw = dict(uct_c=2.0, max_simulations=400)
  got = eng.mcts_batch(acts, offs, bs, es, child_selection=_lib.SELECT_PUCT, **kw)
  ref = O.Game(gs).mcts_batch(acts, offs, bs, es, max_children=eng.max_children, puct=True,
                              **kw)
  _cmp(E, got, ref)


def test_cpp_style_puct_bot_matches_oracle(E):
  """pyspiel.MCTSBot(..., ChildSelectionPolicy.PUCT) (pyspiel.cc:512-524)."""
  import pyspiel
  game = pyspiel.load_game("connect_four")
  bot = pyspiel.MCTSBot(game, pyspiel.RandomRolloutEvaluator(1, 7), 2.0, 400, 1000, True, 3,
                        False, pyspiel.ChildSelectionPolicy.PUCT)
  root = bot.mcts_search(game.new_initial_state())
  ref = O.Game("connect_four").mcts_batch(np.zeros(0, np.int64), np.array([0, 0]), [3], [7],
                                          uct_c=2.0, max_simulations=400, puct=True)
  assert [c.action for c in root.children] == list(ref["child_action"][0][:7])
  assert [c.explore_count for c in root.children] == list(ref["child_n"][0][:7])
  assert root.best_child().action == ref["best_action"][0]
