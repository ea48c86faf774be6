"""Multi-GPU drivers: one process per GPU over torch.distributed.

The reference has no multi-device MCTS; these drivers scale its per-search
semantics (each tree is one bit-exact `MCTSBot::MCTSearch`, mcts.cc:325-428):

* `independent_searches` (C2/C3): global roots [0, R*W) are split into
  contiguous blocks, rank g searching roots [g*R, (g+1)*R) with bot seed = global
  root id and evaluator seed = id + 2^20.  No data-path collective; results can
  be gathered to every rank with one all_gather.
* `root_parallel` (C4): every rank grows T trees on the SAME position, tree
  t of rank g seeded (g*T + t, g*T + t + 2^20).  Root child visits/rewards are
  summed action-indexed on the device, then ONE all-reduce of one f64[2A]
  message (RCCL over xGMI on the GPU; gloo in the CPU tests) combines them.  The result equals the sum of
  the W*T single-tree reference searches, whatever W is.
* `sharded_playouts` (C5): global playouts [0, N) split into contiguous blocks,
  evaluator seed = global playout id; per-rank outcome counts (p0 wins, p1 wins,
  draws) computed on the device and all-reduced.

Compute goes through a *backend*: `HipBackend` drives libos_mcts.so (device
buffers, HIP stream of the current torch device, no host round trip before
the collective).  The CPU test-suite supplies its own backend (the product
engine compiled for the host) to check the sharding/seeding/reduction logic
under gloo without a GPU.
"""
import numpy as np

EVAL_SEED_OFFSET = 1 << 20  # evaluator seed = bot seed + 2^20


def shard(total, world, rank):
  """Contiguous block of `total` items owned by `rank`: (start, count).

  The first `total % world` ranks get one extra item, so every item is owned
  exactly once for any world size.
  """
  base, extra = divmod(int(total), int(world))
  start = rank * base + min(rank, extra)
  return start, base + (1 if rank < extra else 0)


def _world(group):
  import torch.distributed as dist
  if not dist.is_available() or not dist.is_initialized():
    return 1, 0
  return dist.get_world_size(group), dist.get_rank(group)


def independent_searches(backend, root_actions, root_offsets, gather=False,
                         group=None, **params):
  """C2/C3: this rank's block of the global root list (histories).

  root_actions/root_offsets describe ALL global roots (every rank passes the
  same lists).  Returns (start, outputs-of-this-rank) or, with gather=True,
  the outputs of every root concatenated in global order on every rank.
  """
  world, rank = _world(group)
  offs = np.asarray(root_offsets, np.int64)
  R = len(offs) - 1
  start, count = shard(R, world, rank)
  ids = np.arange(start, start + count, dtype=np.uint32)
  acts = np.asarray(root_actions, np.int64)[offs[start]:offs[start + count]]
  loc_offs = offs[start:start + count + 1] - offs[start]
  out = backend.search(acts, loc_offs, ids, ids + np.uint32(EVAL_SEED_OFFSET), **params)
  if not gather or world == 1:
    return (start, out) if not gather else out
  return _gather_outputs(out, R, world, group)


def _gather_outputs(out, R, world, group):
  """all_gather of per-rank output blocks (padded to the largest block)."""
  import torch
  import torch.distributed as dist
  maxc = max(shard(R, world, g)[1] for g in range(world))
  res = {}
  for k in sorted(out):
    a = np.asarray(out[k])
    pad = np.zeros((maxc,) + a.shape[1:], a.dtype)
    pad[:len(a)] = a
    t = torch.from_numpy(pad.view(np.uint8).reshape(maxc, -1).copy())
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t, group=group)
    blocks = []
    for g in range(world):
      n = shard(R, world, g)[1]
      blocks.append(parts[g].numpy().reshape(-1).view(a.dtype).reshape(
          (maxc,) + a.shape[1:])[:n])
    res[k] = np.concatenate(blocks)
  return res


def root_parallel(backend, history, trees_per_rank, group=None, **params):
  """C4: root-parallel MCTS on one position; returns (visits, rewards).

  visits int64[A] / rewards f64[A] (A = NumDistinctActions) summed over the
  root children of all W*T trees, action-indexed.  The tensors live on the
  backend's device; the all-reduce runs on them in place.
  """
  import torch.distributed as dist
  world, rank = _world(group)
  T = int(trees_per_rank)
  ids = np.arange(rank * T, (rank + 1) * T, dtype=np.uint32)
  visits, rewards = backend.root_sums(np.asarray(history, np.int64), ids,
                                      ids + np.uint32(EVAL_SEED_OFFSET), **params)
  if world > 1:
    visits, rewards = _all_reduce_root_sums(visits, rewards, group)
  return visits, rewards


def _all_reduce_root_sums(visits, rewards, group):
  """The root sums of every rank, added in RANK ORDER on every rank.

  Each rank sends its concatenated f64[2A] (visits, rewards) message through
  ONE all_gather (~2 KB per rank: latency-bound on xGMI, so one collective per
  step), then every rank adds the W parts left to right: rank 0's sums, plus
  rank 1's, ...  The result is therefore fixed by the data alone, not by the
  collective library's ring or tree order: with f64 rewards that are not
  integers (n_rollouts > 1, pig's -1/(n-1)) an all-reduce's association
  order changes the last bits, and this order does not.  Within a rank,
  k_root_reduce sums each action over the rank's trees in ascending tree
  order.  Visit counts travel as f64 and come back exact
  (every partial sum is an integer below 2^53: 8 ranks x 8192 trees x 2048
  sims ~ 1.3e8).
  """
  import torch
  import torch.distributed as dist
  A = visits.numel()
  msg = torch.cat((visits.to(torch.float64), rewards))
  world = dist.get_world_size(group)
  parts = [torch.empty_like(msg) for _ in range(world)]
  dist.all_gather(parts, msg, group=group)
  acc = parts[0].clone()
  for p in parts[1:]:
    acc += p
  return acc[:A].to(torch.int64), acc[A:]


def fixed_order_sum(per_rank):
  """The reduction _all_reduce_root_sums performs, on host arrays: rank 0's
  f64 sums, plus rank 1's, ... (the order tests hold the oracle to)."""
  acc = np.array(per_rank[0], np.float64, copy=True)
  for p in per_rank[1:]:
    acc += np.asarray(p, np.float64)
  return acc


def sharded_playouts(backend, history, total, group=None, n_rollouts=1):
  """C5: `total` random playouts from one position split across ranks;
  returns int64[3] (player-0 wins, player-1 wins, draws) over all ranks."""
  import torch.distributed as dist
  world, rank = _world(group)
  start, count = shard(total, world, rank)
  seeds = np.arange(start, start + count, dtype=np.uint32)
  counts = backend.playout_counts(np.asarray(history, np.int64), seeds, n_rollouts)
  if world > 1:
    dist.all_reduce(counts, group=group)
  return counts


class HipBackend:
  """libos_mcts.so on one GPU; results stay in HBM until the collective.

  `engine` replaces the device engine only in the CPU rehearsal of bench.py
  (tests/bench_rehearsal.py); then tensors live on the CPU for gloo.
  """

  def __init__(self, game_string, device=0, engine=None):
    import torch
    from . import engine as E
    self.torch = torch
    if engine is None:
      self.eng = E.Engine(game_string, device)
      self.device = torch.device("cuda", device)
    else:
      self.eng = engine
      self.device = torch.device("cpu")
    self.num_actions = self.eng.num_distinct_actions

  def _stream(self):
    if self.device.type != "cuda":
      return None
    return self.torch.cuda.current_stream(self.device).cuda_stream

  def search(self, acts, offs, bot_seeds, eval_seeds, **params):
    return self.eng.mcts_batch(acts, offs, bot_seeds, eval_seeds, **params)

  def prepare_root_parallel(self, history, bot_seeds, eval_seeds, **params):
    T = len(bot_seeds)
    h = np.asarray(history, np.int64)
    acts = np.tile(h, T)
    offs = np.arange(T + 1, dtype=np.int64) * len(h)
    self.eng.prepare(acts, offs, bot_seeds, eval_seeds, **params)

  def run_root_parallel(self):
    """Launches the T searches + the action-indexed reduction (async).

    The sums are those of the launched run: if it is a paged batch that runs
    out of pool pages, `fetch` reruns it on the reserved arena and the sums
    must be taken again (`root_sums` does; see os_engine_arena_info)."""
    torch = self.torch
    st = self._stream()
    self.eng.run_async(st)
    v = torch.empty(self.num_actions, dtype=torch.int64, device=self.device)
    w = torch.empty(self.num_actions, dtype=torch.float64, device=self.device)
    self.eng.root_sums_async(self.num_actions, v.data_ptr(), w.data_ptr(), st)
    return v, w

  def root_sums(self, history, bot_seeds, eval_seeds, **params):
    self.prepare_root_parallel(history, bot_seeds, eval_seeds, **params)
    reruns = self._reruns()
    v, w = self.run_root_parallel()
    self.eng.fetch()  # synchronises and raises on any per-tree failure
    if self._reruns() != reruns:
      # A paged batch ran out of pool pages: the fetch reran it on the reserved
      # arena (same seeds, full searches), so the sums queued above belong to
      # the overflowed run.  Sum the rerun's children instead.
      st = self._stream()
      self.eng.root_sums_async(self.num_actions, v.data_ptr(), w.data_ptr(), st)
      if self.device.type == "cuda":
        self.torch.cuda.current_stream(self.device).synchronize()
    return v, w

  def _reruns(self):
    arena_info = getattr(self.eng, "arena_info", None)
    return arena_info()["reruns"] if arena_info else 0

  def prepare_playouts(self, history, seeds, n_rollouts=1):
    self.eng.rollouts_prepare(history, seeds, n_rollouts)

  def run_playouts(self):
    torch = self.torch
    st = self._stream()
    self.eng.rollouts_run_async(st)
    c = torch.empty(3, dtype=torch.int64, device=self.device)
    self.eng.rollouts_outcomes_async(c.data_ptr(), st)
    return c

  def playout_counts(self, history, seeds, n_rollouts=1):
    self.prepare_playouts(history, seeds, n_rollouts)
    return self.run_playouts()
