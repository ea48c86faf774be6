"""Multi-process (gloo, world_size 2) tests of the multi-GPU drivers (os_amd/dist.py).

The drivers' sharding, seeding and reduction logic runs here on the CPU with a
host backend: the product engine (csrc/os_mcts.h) compiled for the host
(tests/hostcheck), returning CPU tensors so gloo can reduce them.  Results are
compared with the oracle (reference-faithful CPU restatement of mcts.cc): a
root-parallel sum over W ranks x T trees must equal the sum of the W*T
single-tree oracle searches, whatever W is.  GPU variants of
the same checks (HipBackend, RCCL-free world 1) are marked `gpu`.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import hostcheck_lib as hc
import oracle_lib
from os_amd import dist as D

HEX5 = "hex(board_size=5)"
SIMS = 48


class HostBackend:
  """Test double for dist.HipBackend: host-compiled product engine."""

  def __init__(self, game_string):
    self.gs = game_string
    self.og = oracle_lib.Game(game_string)
    self.A = self.og.num_distinct_actions
    self.mc = self.A

  def search(self, acts, offs, bot_seeds, eval_seeds, **params):
    return hc.mcts_batch(self.gs, acts, offs, bot_seeds, eval_seeds, self.mc,
                         **_hc_params(params))

  def root_sums(self, history, bot_seeds, eval_seeds, **params):
    T = len(bot_seeds)
    acts = np.tile(np.asarray(history, np.int64), T)
    offs = np.arange(T + 1, dtype=np.int64) * len(history)
    o = self.search(acts, offs, bot_seeds, eval_seeds, **params)
    return _action_sums(o, self.A)

  def playout_counts(self, history, seeds, n_rollouts=1):
    assert n_rollouts == 1
    r = hc.rollouts(self.gs, history, seeds)[:, 0]
    return torch.tensor([(r > 0).sum(), (r < 0).sum(), (r == 0).sum()], dtype=torch.int64)


def _hc_params(p):
  keep = ("uct_c", "max_simulations", "n_rollouts", "max_memory_mb", "solve")
  return {k: v for k, v in p.items() if k in keep}


def _action_sums(o, A):
  v = torch.zeros(A, dtype=torch.int64)
  w = torch.zeros(A, dtype=torch.float64)
  for r in range(len(o["nchild"])):
    for k in range(int(o["nchild"][r])):
      a = int(o["child_action"][r, k])
      v[a] += int(o["child_n"][r, k])
      w[a] += float(o["child_w"][r, k])
  return v, w


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def _worker(rank, world, port, q, hip=False):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    # hip: every rank drives the real device engine (HipBackend) on cuda:0;
    # gloo reduces the device tensors root_parallel / sharded_playouts return.
    mk = (lambda gs: D.HipBackend(gs, device=0)) if hip else HostBackend
    be = mk(HEX5)
    v, w = D.root_parallel(be, [12], trees_per_rank=3, max_simulations=SIMS)
    c = D.sharded_playouts(mk("connect_four"), [3, 3], total=37)
    acts, offs = _c4_roots(5)
    g = D.independent_searches(mk("connect_four"), acts, offs, gather=True,
                               max_simulations=SIMS)
    q.put((rank, v.cpu().numpy(), w.cpu().numpy(), c.cpu().numpy(),
           {k: np.asarray(x) for k, x in g.items()}))
  finally:
    dist.destroy_process_group()


def _c4_roots(R):
  hs = [[(i * 3 + j) % 7 for j in range(i % 4)] for i in range(R)]
  offs = np.zeros(R + 1, np.int64)
  for i, h in enumerate(hs):
    offs[i + 1] = offs[i] + len(h)
  return np.array([a for h in hs for a in h], np.int64), offs


def _oracle_root_parallel(gs, history, n_trees, sims):
  og = oracle_lib.Game(gs)
  ids = np.arange(n_trees, dtype=np.uint32)
  acts = np.tile(np.asarray(history, np.int64), n_trees)
  offs = np.arange(n_trees + 1, dtype=np.int64) * len(history)
  o = og.mcts_batch(acts, offs, ids, ids + np.uint32(D.EVAL_SEED_OFFSET),
                    max_simulations=sims)
  return _action_sums(o, og.num_distinct_actions)


@pytest.mark.parametrize("total,world", [(0, 1), (1, 2), (7, 2), (8, 8), (37, 3),
                                          (1 << 20, 8), (5, 8)])
def test_shard_partitions_exactly(total, world):
  seen = np.zeros(total, np.int32)
  prev_end = 0
  for r in range(world):
    s, n = D.shard(total, world, r)
    assert s == prev_end
    seen[s:s + n] += 1
    prev_end = s + n
  assert prev_end == total and (seen == 1).all()


def test_world1_matches_oracle():
  be = HostBackend(HEX5)
  v, w = D.root_parallel(be, [12], trees_per_rank=4, max_simulations=SIMS)
  ov, ow = _oracle_root_parallel(HEX5, [12], 4, SIMS)
  assert torch.equal(v, ov) and torch.equal(w, ow)
  assert int(v.sum()) == 4 * (SIMS - 1)  # sim 0 evaluates the root itself


def test_gloo_world2_matches_single_process():
  _check_world2(hip=False)


@pytest.mark.gpu
def test_gpu_gloo_world2_hip_backend(require_gpu):
  """The same drivers over two rank processes that both drive the HIP engine
  (one GPU on this box, so the ranks share device 0; gloo in place of RCCL,
  which refuses two ranks on one device)."""
  _check_world2(hip=True)


def _check_world2(hip):
  world, port = 2, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_worker, args=(r, world, port, q, hip)) for r in range(world)]
  for p in procs:
    p.start()
  res = [q.get(timeout=300) for _ in range(world)]
  for p in procs:
    p.join(60)
    assert p.exitcode == 0
  res.sort(key=lambda t: t[0])
  # C4: root-parallel over 2 ranks x 3 trees == 6 oracle trees, on every rank.
  ov, ow = _oracle_root_parallel(HEX5, [12], 6, SIMS)
  for _, v, w, _, _ in res:
    np.testing.assert_array_equal(v, ov.numpy())
    np.testing.assert_array_equal(w, ow.numpy())
  # C5: 37 playouts split 19/18, counts == oracle over seeds 0..36.
  r = oracle_lib.Game("connect_four").rollouts([3, 3], np.arange(37, dtype=np.uint32))[:, 0]
  want = [(r > 0).sum(), (r < 0).sum(), (r == 0).sum()]
  for _, _, _, c, _ in res:
    np.testing.assert_array_equal(c, want)
  # C2/C3: gathered independent searches == one-process oracle batch.
  acts, offs = _c4_roots(5)
  ids = np.arange(5, dtype=np.uint32)
  ref = oracle_lib.Game("connect_four").mcts_batch(
      acts, offs, ids, ids + np.uint32(D.EVAL_SEED_OFFSET), max_simulations=SIMS,
      max_children=7)
  for _, _, _, _, g in res:
    for k in ("child_action", "child_n", "child_w", "root_n", "best_action"):
      np.testing.assert_array_equal(g[k], ref[k], err_msg=k)


# ---------------------------------------------------------------------------
# The cross-rank reward sum in a fixed order: with
# non-integer f64 rewards (n_rollouts = 3 averages; pig with 4 players credits
# -1/3) the association order of the sum changes its last bits, so the ranks
# add their parts in rank order (dist._all_reduce_root_sums), not in whatever
# order the collective library reduces.  World 3: with two ranks every order
# gives s0 + s1, so it takes three to tell orders apart.
WORLD3_CASES = (("hex(board_size=5)", [12], dict(max_simulations=SIMS, n_rollouts=3)),
                ("pig(players=4,horizon=8,winscore=6)", [],
                 dict(max_simulations=40)))


def _worker_fixed_order(rank, world, port, q):
  os.environ["MASTER_ADDR"] = "127.0.0.1"
  os.environ["MASTER_PORT"] = str(port)
  dist.init_process_group("gloo", rank=rank, world_size=world)
  try:
    out = []
    for gs, hist, kw in WORLD3_CASES:
      v, w = D.root_parallel(HostBackend(gs), hist, trees_per_rank=4, **kw)
      out.append((v.numpy(), w.numpy()))
    q.put((rank, out))
  finally:
    dist.destroy_process_group()


def _oracle_rank_sums(gs, hist, world, T, kw):
  og = oracle_lib.Game(gs)
  parts_v, parts_w = [], []
  for g in range(world):
    ids = np.arange(g * T, (g + 1) * T, dtype=np.uint32)
    acts = np.tile(np.asarray(hist, np.int64), T)
    offs = np.arange(T + 1, dtype=np.int64) * len(hist)
    o = og.mcts_batch(acts, offs, ids, ids + np.uint32(D.EVAL_SEED_OFFSET), **kw)
    v, w = _action_sums(o, og.num_distinct_actions)
    parts_v.append(v.numpy())
    parts_w.append(w.numpy())
  return parts_v, parts_w


def test_gloo_world3_reward_sum_in_rank_order():
  world, port = 3, _free_port()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  procs = [ctx.Process(target=_worker_fixed_order, args=(r, world, port, q))
           for r in range(world)]
  for p in procs:
    p.start()
  res = [q.get(timeout=300) for _ in range(world)]
  for p in procs:
    p.join(60)
    assert p.exitcode == 0
  inexact = 0
  for i, (gs, hist, kw) in enumerate(WORLD3_CASES):
    pv, pw = _oracle_rank_sums(gs, hist, world, 4, kw)
    want_w = D.fixed_order_sum(pw)
    want_v = np.sum(pv, axis=0)
    # the other association, s0 + (s1 + s2): differs where the order matters
    other = pw[0] + (pw[1] + pw[2])
    inexact += int((other != want_w).sum())
    for _, out in res:
      v, w = out[i]
      np.testing.assert_array_equal(v, want_v)
      assert w.tobytes() == want_w.tobytes(), gs
  assert inexact > 0  # the cases do exercise a non-associative sum


def test_fixed_order_sum_is_left_to_right():
  a = np.array([0.1, 1e16]), np.array([0.2, 1.0]), np.array([0.3, -1e16])
  got = D.fixed_order_sum(a)
  assert got.tobytes() == ((a[0] + a[1]) + a[2]).tobytes()
  assert got[1] == 0.0  # (1e16 + 1) - 1e16 in f64


@pytest.mark.gpu
def test_gpu_root_parallel_world1(require_gpu):
  be = D.HipBackend(HEX5)
  v, w = D.root_parallel(be, [12], trees_per_rank=16, max_simulations=SIMS)
  ov, ow = _oracle_root_parallel(HEX5, [12], 16, SIMS)
  assert torch.equal(v.cpu(), ov) and torch.equal(w.cpu(), ow)


@pytest.mark.gpu
def test_gpu_root_parallel_lane_layout(require_gpu):
  from os_amd import _lib
  be = D.HipBackend("tic_tac_toe")
  v, w = D.root_parallel(be, [], trees_per_rank=64, max_simulations=100,
                         layout=_lib.LAYOUT_LANE)
  ov, ow = _oracle_root_parallel("tic_tac_toe", [], 64, 100)
  assert torch.equal(v.cpu(), ov) and torch.equal(w.cpu(), ow)


@pytest.mark.gpu
@pytest.mark.parametrize("n_engines", [1, 3])
def test_gpu_c_abi_root_parallel_matches_oracle(require_gpu, n_engines):
  """os_root_parallel (one process, several engines; on a 1-GPU box they share
  device 0, which exercises the same peer-copy + fixed-order device sum)."""
  import torch as _t
  from os_amd import engine as E
  ndev = _t.cuda.device_count()
  engines = [E.Engine(HEX5, device=g % ndev) for g in range(n_engines)]
  T = 5
  v, w, sims = E.root_parallel(engines, [12], T, seed_base=0, max_simulations=SIMS)
  ov, ow = _oracle_root_parallel(HEX5, [12], n_engines * T, SIMS)
  np.testing.assert_array_equal(v, ov.numpy())
  np.testing.assert_array_equal(w, ow.numpy())
  assert sims == n_engines * T * SIMS


@pytest.mark.gpu
def test_gpu_c_abi_root_parallel_rejects_duplicate_engine(require_gpu):
  from os_amd import engine as E
  e = E.Engine(HEX5, device=0)
  with pytest.raises(RuntimeError):
    E.root_parallel([e, e], [12], 2, max_simulations=SIMS)


@pytest.mark.gpu
def test_gpu_playout_counts(require_gpu):
  be = D.HipBackend("go(board_size=9)")
  seeds_total = 300
  c = D.sharded_playouts(be, [], total=seeds_total)
  r = oracle_lib.Game("go(board_size=9)").rollouts(
      [], np.arange(seeds_total, dtype=np.uint32))[:, 0]
  assert c.cpu().tolist() == [(r > 0).sum(), (r < 0).sum(), (r == 0).sum()]


# ---------------------------------------------------------------------------
# bench.py's own multi-rank path (launcher, rank/seed assignment, all-reduces),
# rehearsed on the CPU: `--gpus 2` spawns two ranks under torch.distributed.run,
# `--rehearse-host` swaps gloo + the host-compiled engine in for RCCL + the GPU.
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")


def _bench(*args, env=None):
  import json
  import subprocess
  import sys
  e = dict(os.environ)
  e.pop("WORLD_SIZE", None)
  e.update(env or {})
  p = subprocess.run([sys.executable, BENCH, "--rehearse-host", "--steps", "1", "--warmup",
                      "1", "--no-cpu-baseline"] + list(args),
                     capture_output=True, text=True, timeout=600, env=e)
  lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
  return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus2_spawns_ranks_root_parallel():
  rc, line, err = _bench("--gpus", "2", "--config", "c4", "--roots", "3", "--sims",
                         str(SIMS), "--parity-roots", "3")
  assert rc == 0, err[-2000:]
  assert line["n_gpus"] == 2 and line["data"].startswith("REHEARSAL")
  assert line["parity"]["bit_exact"] and line["parity"]["allreduce_equals_sum_of_trees"]
  # rank g grew trees g*3 .. g*3+2: the all-reduced visits are those of 6 trees.
  ov, _ = _oracle_root_parallel("hex(board_size=11)", [], 6, SIMS)
  top = sorted(((int(n), a) for a, n in enumerate(ov.tolist())), reverse=True)[:5]
  assert [tuple(x) for x in line["root_visits_top5"]] == top


def test_bench_gpus2_spawns_ranks_playouts():
  rc, line, err = _bench("--gpus", "2", "--config", "c5", "--roots", "9")
  assert rc == 0, err[-2000:]
  assert line["n_gpus"] == 2 and line["parity"]["counts_equal_returns"]
  r = oracle_lib.Game("go(board_size=9)").rollouts([], np.arange(9, dtype=np.uint32))[:, 0]
  o = line["outcomes"]
  assert [o["p0_wins"], o["p1_wins"], o["draws"]] == \
      [int((r > 0).sum()), int((r < 0).sum()), int((r == 0).sum())]


def test_bench_gpus2_spawns_ranks_search():
  rc, line, err = _bench("--gpus", "2", "--config", "c2", "--roots", "4", "--sims",
                         str(SIMS), "--parity-roots", "4")
  assert rc == 0, err[-2000:]
  assert line["n_gpus"] == 2 and line["parity"]["bit_exact"]
  assert "dp2" in line["config"]["parallelism"]


def test_bench_rejects_world_size_mismatch():
  rc, line, err = _bench("--gpus", "2", "--config", "c2", "--roots", "2", "--sims", "8",
                         env={"WORLD_SIZE": "1"})
  assert rc != 0 and line is None and "WORLD_SIZE" in err
