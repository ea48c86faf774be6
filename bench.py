#!/usr/bin/env python3
"""Headline benchmark: random-rollout MCTS simulations/s on connect_four.

BASELINE.json metric: "MCTS simulations/sec (random rollout) on connect_four
at 1/2/4/8 MI355X"; workload = configs[1] (`--config c2`, the default): 4096
independent roots x 1024 simulations per GPU (weak scaling: every rank searches
its own 4096 roots, seeded by global root id; no data-path collective).

The other BASELINE configs are reachable for measurement and parity runs:
  c3  breakthrough(rows=8,columns=8), 65536 roots x 2048 sims per GPU
  c4  hex(board_size=11), root-parallel: T trees per GPU on the initial
      position, 2048 sims each, action-indexed root visits all-reduced over
      RCCL inside every timed step
  c5  go(board_size=9), 2^20 random playouts split across the ranks
      (strong scaling), outcome counts all-reduced inside every timed step

One step = one pass of the hot path over the rank's batch (roots and seeds
already resident in HBM).  Rank 0 prints ONE JSON line.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

`--gpus N` (N > 1) without a torch.distributed environment starts the N rank
processes itself (torch.distributed.run as a child process, before anything
touches the GPU) and exits with its status; with WORLD_SIZE set, N must equal
it.  `--rehearse-host` is for the CPU test-suite only: the same rank/seed
assignment and all-reduces under gloo, with a host-compiled engine from
tests/ (never a measurement; its line says so).
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_CUS = 256
CLOCK_HZ = 2.4e9  # max engine clock (MI355X_MICROARCH.md)
EVAL_OFFSET = 1 << 20

# name: (mode, game string, units per GPU (or total for c5), sims, root plies)
CONFIGS = {
    "c2": ("search", "connect_four", 4096, 1024, 8),
    "c3": ("search", "breakthrough(rows=8,columns=8)", 65536, 2048, 6),
    "c4": ("root_parallel", "hex(board_size=11)", 8192, 2048, 0),
    "c5": ("playouts", "go(board_size=9)", 1 << 20, 0, 0),
    # SURVEY §8f rank 1 (not a BASELINE config): full self-play games, two
    # MCTSBots + one shared evaluator per game, one wave per game.
    "sp": ("selfplay", "connect_four", 4096, 256, 4),
    # SURVEY §8f rank 2 (not a BASELINE config): PUCT search with an external
    # (network) evaluator, batched across searches; AlphaZero root noise.
    "az": ("az", "connect_four", 16384, 128, 4),
    # go search (not a BASELINE config): independent go9 roots, random
    # rollouts + solver, as c2 on connect_four.
    "g9": ("search", "go(board_size=9)", 65536, 256, 6),
}
KERNEL = {"wave": "k_wsearch", "lane": "k_mcts"}
PAGED_ABOVE = 4 << 30  # --arena auto: page the arena when the reservation exceeds this


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=5)
  ap.add_argument("--warmup", type=int, default=2)
  ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
  ap.add_argument("--roots", type=int, default=0,
                  help="override roots / trees / playouts of the config")
  ap.add_argument("--sims", type=int, default=0, help="override simulations")
  ap.add_argument("--block", type=int, default=0, help="lanes per workgroup (lane layout)")
  ap.add_argument("--arena-nodes", type=int, default=0)
  ap.add_argument("--layout", default="auto", choices=("auto", "wave", "lane"),
                  help="search kernel: one wave per search / one lane per search")
  ap.add_argument("--arena", default="auto", choices=("auto", "paged", "reserved"),
                  help="search-tree arena (c2/c3): a page pool sized from the warmup "
                       "run, the worst case per root, or (auto) the pool when the "
                       "worst case would exceed %d GB" % (PAGED_ABOVE >> 30))
  ap.add_argument("--no-cpu-baseline", action="store_true")
  ap.add_argument("--cpu-seconds", type=float, default=12.0,
                  help="target CPU-baseline sample duration")
  ap.add_argument("--parity-roots", type=int, default=32)
  ap.add_argument("--no-parity-sweep", dest="parity_sweep", action="store_false",
                  help="c2: skip the bit-exact sweep over the other kernels (C3/C4/C5 "
                       "shapes, go lane layout, PUCT, numpy policy, chance nodes), run "
                       "after the timed region")
  ap.add_argument("--no-configs", dest="configs", action="store_false",
                  help="c2: skip the timed full-size C3 / C4 / C5 / g9 entries run after "
                       "the headline line (the `configs` sub-object)")
  ap.add_argument("--az-graph", type=int, default=1,
                  help="az: replay each evaluator round as one captured HIP graph (1) "
                       "or launch it op by op (0)")
  ap.add_argument("--az-layout", default="auto", choices=("auto", "wave", "lane"),
                  help="az: one wavefront per search (k_waz_step), one lane per search "
                       "(k_az_step) or auto (wave unless GC can fire)")
  ap.add_argument("--az-overlap", type=int, default=1,
                  help="az: stage step k+1's host work (root replay, Dirichlet draws; "
                       "os_az_stage) on a worker thread while step k searches (1), or "
                       "prepare each step serially (0)")
  ap.add_argument("--az-requests", default="fused", choices=("fused", "separate"),
                  help="az: one evaluator round per simulation (pure evaluator) or "
                       "the reference's separate Prior / Evaluate rounds")
  ap.add_argument("--rehearse-host", action="store_true",
                  help="CPU test-suite rehearsal of the rank plumbing (gloo, host "
                       "engine from tests/); not a measurement")
  return ap.parse_args()


def _free_port():
  with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    return s.getsockname()[1]


def launch_ranks(args):
  """--gpus N > 1 outside torch.distributed: run N ranks of this script under
  torch.distributed.run (one process per GPU) as a CHILD process and return
  its exit status.  Nothing here touches the GPU, so the parent never holds a
  device context (no exec from a GPU-initialised process)."""
  cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
         "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
         "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
  env = dict(os.environ)
  env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
  return subprocess.call(cmd, env=env)


class Ctx:
  """Rank / device / collective plumbing (one process per GPU)."""

  def __init__(self, args):
    import torch
    import torch.distributed as dist
    self.torch, self.dist = torch, dist
    self.world = int(os.environ.get("WORLD_SIZE", "1"))
    self.rank = int(os.environ.get("RANK", "0"))
    self.local = int(os.environ.get("LOCAL_RANK", "0"))
    if self.world != args.gpus:
      raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, self.world))
    self.rehearse = args.rehearse_host
    if self.rehearse:  # CPU test-suite: gloo + host engine, no GPU call
      self.dev = torch.device("cpu")
      self.stream = None
      if self.world > 1:
        dist.init_process_group("gloo")
      return
    self.dev = torch.device("cuda", self.local)
    torch.cuda.set_device(self.local)
    if self.world > 1:
      dist.init_process_group("nccl", device_id=self.dev)
    self.stream = torch.cuda.current_stream()

  @property
  def handle(self):
    return None if self.stream is None else self.stream.cuda_stream

  def engine(self, game):
    """The search engine of this rank: libos_mcts.so on this rank's GPU."""
    if self.rehearse:
      sys.path.insert(0, os.path.join(ROOT, "tests"))
      import bench_rehearsal
      return bench_rehearsal.HostEngine(game)
    from os_amd import engine as E
    return E.Engine(game, device=self.local)

  def backend(self, game):
    from os_amd import dist as D
    if self.rehearse:
      return D.HipBackend(game, engine=self.engine(game))
    return D.HipBackend(game, self.local)

  def barrier(self):
    if self.world > 1:
      self.dist.barrier()

  def sync(self):
    if not self.rehearse:
      self.torch.cuda.synchronize()

  def timed(self, step, steps):
    """Barrier + sync, K steps, sync + barrier; (wall max over ranks, event ms).

    The events are recorded on the stream the kernels are launched on."""
    torch = self.torch
    self.barrier()
    self.sync()
    if not self.rehearse:
      ev0 = torch.cuda.Event(enable_timing=True)
      ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if not self.rehearse:
      ev0.record(self.stream)
    for _ in range(steps):
      step()
    if not self.rehearse:
      ev1.record(self.stream)
    self.sync()
    self.barrier()
    elapsed = time.perf_counter() - t0
    if self.world > 1:
      t = torch.tensor([elapsed], dtype=torch.float64, device=self.dev)
      self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
      elapsed = float(t.item())
    if self.rehearse:
      return elapsed, elapsed * 1e3 / max(steps, 1)
    return elapsed, ev0.elapsed_time(ev1) / max(steps, 1)

  def total(self, x):
    """Sum of a per-rank count over all ranks."""
    if self.world == 1:
      return x
    t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.dev)
    self.dist.all_reduce(t)
    return float(t.item())


def main():
  args = parse()
  if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
    sys.exit(launch_ranks(args))
  ctx = Ctx(args)
  from os_amd import _lib
  layouts = {"auto": _lib.LAYOUT_AUTO, "wave": _lib.LAYOUT_WAVE, "lane": _lib.LAYOUT_LANE}
  mode = CONFIGS[args.config][0]
  fn = {"search": bench_search, "root_parallel": bench_root_parallel,
        "playouts": bench_playouts, "selfplay": bench_selfplay, "az": bench_az}[mode]
  line = fn(args, ctx, layouts[args.layout])
  if ctx.rank == 0:
    if ctx.rehearse:
      line["data"] = "REHEARSAL: host-compiled engine under gloo (tests only, not a measurement)"
      line["roofline"] = None
    print(json.dumps(line), flush=True)
  if ctx.world > 1:
    ctx.dist.destroy_process_group()


def _resolved_layout(eng):
  """The layout the engine ran the last prepared batch on (os_engine_get_layout:
  OS_LAYOUT_AUTO resolved by the engine's own rule)."""
  from os_amd import _lib
  if not hasattr(eng, "layout"):  # --rehearse-host's host engine: the line
    return "wave"                  # is a plumbing check, never a result
  return "wave" if eng.layout() == _lib.LAYOUT_WAVE else "lane"


def _base_line(args, ctx, metric, value, unit, elapsed, config):
  return {
      "metric": metric, "value": value, "unit": unit, "n_gpus": ctx.world,
      "steps": args.steps, "warmup": args.warmup,
      "ms_per_step": elapsed / max(args.steps, 1) * 1e3, "higher_is_better": True,
      "scaling": "weak" if args.config != "c5" else "strong",
      "vs_baseline": None, "dtype": "int32+f64",
      "data": "synthetic (seeded random roots; no dataset)", "config": config,
  }


def _roofline(kernel, game, alg_bytes, kernel_ms, units, unit_name):
  """HBM roofline of the dominant kernel (the contract's bound/achieved/peak/
  frac/traffic), plus the instruction-issue roofline that actually binds these
  integer kernels, named in `binding`."""
  achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
  pmc = pmc_record(kernel, game)
  issue = _issue_roofline(pmc, units, kernel_ms)
  hbm_frac = achieved / HBM_PEAK_GBS
  binding = ("hbm" if issue is None or hbm_frac >= issue["frac"] else issue["bound"])
  return {
      "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
      "frac": hbm_frac, "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
      "binding": binding,
      "binding_frac": hbm_frac if binding == "hbm" else issue["frac"],
      "kernel": kernel, "kernel_ms_per_launch": kernel_ms,
      "algorithmic_bytes_per_launch": alg_bytes,
      "algorithmic_bytes_per_%s" % unit_name: alg_bytes / max(units, 1),
      "issue": issue,
      "pmc_source": _pmc_provenance(pmc),
  }


def _issue_roofline(pmc, units, kernel_ms):
  """The bound that does apply: instruction issue.  One CU
  issues at most one SALU instruction per clock and, over its four SIMDs, two
  wave64 VALU instructions per clock (each takes 2 cycles on its SIMD).
  Instructions per unit come from the committed PMC summary of this kernel
  (SQ_INSTS_SALU / SQ_INSTS_VALU per sim), the rate from this run's live kernel
  time; `bound` names whichever pipe is closer to its peak."""
  if not pmc:
    return None
  out = {}
  for pipe, counter, per_clock in (("salu", "SQ_INSTS_SALU", 1.0),
                                   ("valu", "SQ_INSTS_VALU", 2.0)):
    per = pmc.get("per_sim", {}).get(counter)
    if per is None:
      return None
    rate = per * units / (kernel_ms / 1e3)
    peak = N_CUS * CLOCK_HZ * per_clock
    out[pipe] = {"per_unit": per, "achieved": rate / 1e9, "peak": peak / 1e9,
                 "unit": "G instr/s", "frac": rate / peak}
  top = max(out, key=lambda p: out[p]["frac"])
  return dict(out, bound="%s-issue" % top, frac=out[top]["frac"])


# ---------------------------------------------------------------------------
# c2 / c3: independent searches
def bench_search(args, ctx, layout):
  from os_amd import engine as E
  _, game, R, sims, plies = CONFIGS[args.config]
  R = args.roots or R
  sims = args.sims or sims
  params = dict(uct_c=2.0, max_simulations=sims, n_rollouts=1, max_memory_mb=1000,
                solve=True, block_size=args.block, arena_nodes=args.arena_nodes,
                layout=layout)
  base = ctx.rank * R  # global root ids of this rank
  acts, offs = E.make_roots(game, R, seed_base=1000 + base, max_plies=plies)
  gid = np.arange(base, base + R, dtype=np.uint32)
  bot_seeds, eval_seeds = gid, gid + np.uint32(EVAL_OFFSET)

  eng = ctx.engine(game)
  eng.set_arena_mode("reserved" if args.arena == "reserved" else "paged")
  eng.prepare(acts, offs, bot_seeds, eval_seeds, **params)
  lay = _resolved_layout(eng)
  handle = ctx.handle
  for _ in range(max(args.warmup, 1)):  # at least one: it sizes the arena / page pool
    eng.run_async(handle)
  out = eng.fetch()  # synchronises; validates per-root status
  arena_mode = args.arena
  if arena_mode == "auto":
    arena_mode = ("paged" if eng.arena_info().get("reserved_bytes", 0) > PAGED_ABOVE
                  else "reserved")
    eng.set_arena_mode(arena_mode)
  if arena_mode == "paged":
    # The warmup run (reserved arena) sized the page pool: prepare again on
    # it and check one run before timing.
    eng.prepare(acts, offs, bot_seeds, eval_seeds, **params)
    eng.run_async(handle)
    out = eng.fetch()
  arena0 = eng.arena_info()
  sims_per_step = eng.last_sims()
  alg_bytes = eng.algorithmic_bytes(R)
  stats = eng.stats()

  parity = None
  ref = None
  if ctx.rank == 0 and args.parity_roots > 0:
    og = _oracle(game)
    pr = min(args.parity_roots, R)
    ref = og.mcts_batch(acts[:offs[pr]], offs[:pr + 1], bot_seeds[:pr], eval_seeds[:pr],
                        uct_c=2.0, max_simulations=sims, max_children=eng.max_children,
                        threads=host_cores()[0])
    bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(out[k][:pr], ref[k])]
    parity = {"roots_checked": pr, "bit_exact": not bad, "mismatch_fields": bad}

  elapsed, kernel_ms = ctx.timed(lambda: eng.run_async(handle), args.steps)
  total_sims = ctx.total(sims_per_step * args.steps)
  out_timed = eng.fetch()  # the last TIMED run's results
  arena = eng.arena_info()
  if arena["reruns"] != arena0["reruns"] or eng.last_sims() != sims_per_step:
    raise RuntimeError("a timed run overflowed the page pool: %r" % (arena,))
  if ref is not None:
    bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(out_timed[k][:pr], ref[k])]
    parity["timed_run_bit_exact"] = not bad
    parity["timed_run_mismatch_fields"] = bad
  sweep = None
  if (ctx.rank == 0 and args.config == "c2" and args.parity_sweep and not ctx.rehearse):
    sweep = parity_sweep(ctx)
  subs = None
  if args.config == "c2" and args.configs and not ctx.rehearse and ctx.world == 1:
    subs = timed_configs(args, ctx, layout)

  cpu = None
  if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
    cpu = cpu_baseline_search(game, acts, offs, bot_seeds, eval_seeds, sims,
                              args.cpu_seconds)
  if ctx.rank != 0:
    return None
  metric = ("MCTS simulations/sec (random rollout) on connect_four at 1/2/4/8 MI355X"
            if args.config == "c2" else
            "MCTS simulations/sec (random rollout) on %s" % game)
  line = _base_line(args, ctx, metric, total_sims / elapsed, "sims/s", elapsed, {
      "workload": "%s, %d independent roots x %d sims per GPU" % (game, R, sims),
      "game": game, "roots_per_gpu": R, "sims_per_root": sims, "uct_c": 2.0,
      "n_rollouts": 1, "solve": True, "max_memory_mb": 1000,
      "root_plies": "k~U[0,%d] from mt19937(1000+i)" % plies,
      "parallelism": "dp%d (independent roots, no collective)" % ctx.world,
      "layout": lay,
      "searches_per_wave": eng.searches_per_wave() if hasattr(eng, "searches_per_wave") else 1,
      "sims_per_step_per_gpu": sims_per_step})
  kern = "k_lsearch" if game.startswith("go") and lay == "lane" else KERNEL[lay]
  line["roofline"] = _roofline(kern, game, alg_bytes, kernel_ms, sims_per_step, "sim")
  line["cpu_baseline"] = cpu
  line["parity"] = parity
  if sweep is not None:
    line["parity_sweep"] = sweep
  if subs is not None:
    line["configs"] = subs
  line["tree_stats"] = stats
  line["arena"] = dict(arena, mode=arena_mode)
  return line


# ---------------------------------------------------------------------------
# c4: root-parallel MCTS on one position + RCCL all-reduce of root visits
def bench_root_parallel(args, ctx, layout):
  from os_amd import dist as D
  _, game, T, sims, _ = CONFIGS[args.config]
  T = args.roots or T
  sims = args.sims or sims
  params = dict(uct_c=2.0, max_simulations=sims, n_rollouts=1, max_memory_mb=1000,
                solve=True, block_size=args.block, arena_nodes=args.arena_nodes,
                layout=layout)
  be = ctx.backend(game)
  ids = np.arange(ctx.rank * T, (ctx.rank + 1) * T, dtype=np.uint32)
  be.prepare_root_parallel([], ids, ids + np.uint32(EVAL_OFFSET), **params)
  torch = ctx.torch

  def step():
    v, w = be.run_root_parallel()
    if ctx.world > 1:  # one f64[2A] message (os_amd/dist.py)
      v, w = D._all_reduce_root_sums(v, w, None)
    return v, w

  be.eng.set_arena_mode("reserved" if args.arena == "reserved" else "paged")
  for _ in range(args.warmup):
    v, w = step()
  out = be.eng.fetch()
  arena_mode = args.arena
  if arena_mode == "auto":
    arena_mode = ("paged" if be.eng.arena_info().get("reserved_bytes", 0) > PAGED_ABOVE
                  else "reserved")
    be.eng.set_arena_mode(arena_mode)
  if arena_mode == "paged":  # as in bench_search: one checked run on the pool
    be.prepare_root_parallel([], ids, ids + np.uint32(EVAL_OFFSET), **params)
    v, w = step()
    out = be.eng.fetch()
  arena0 = be.eng.arena_info()
  lay = _resolved_layout(be.eng)
  sims_per_step = be.eng.last_sims()
  alg_bytes = be.eng.algorithmic_bytes(T)
  stats = be.eng.stats()
  # Self-consistency of the device reduction + oracle parity on a prefix.
  local_v = np.zeros(be.num_actions, np.int64)
  for r in range(T):
    for k in range(int(out["nchild"][r])):
      local_v[out["child_action"][r, k]] += out["child_n"][r, k]
  lv = torch.from_numpy(local_v).to(ctx.dev)
  if ctx.world > 1:
    ctx.dist.all_reduce(lv)
  reduce_ok = bool(torch.equal(lv, v))
  parity = None
  if ctx.rank == 0 and args.parity_roots > 0:
    og = _oracle(game)
    pr = min(args.parity_roots, 8, T)
    acts = np.zeros(0, np.int64)
    offs = np.zeros(pr + 1, np.int64)
    ref = og.mcts_batch(acts, offs, ids[:pr], ids[:pr] + np.uint32(EVAL_OFFSET),
                        uct_c=2.0, max_simulations=sims, max_children=be.eng.max_children,
                        threads=host_cores()[0])
    bad = [k for k in ("child_action", "child_n", "child_w", "root_n", "best_action")
           if not np.array_equal(out[k][:pr], ref[k])]
    parity = {"trees_checked": pr, "bit_exact": not bad, "mismatch_fields": bad,
              "allreduce_equals_sum_of_trees": reduce_ok}

  elapsed, kernel_ms = ctx.timed(step, args.steps)
  total_sims = ctx.total(sims_per_step * args.steps)
  be.eng.fetch()
  arena = be.eng.arena_info()
  if arena["reruns"] != arena0["reruns"] or be.eng.last_sims() != sims_per_step:
    raise RuntimeError("a timed run overflowed the page pool: %r" % (arena,))
  cpu = None
  if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
    acts = np.zeros(0, np.int64)
    offs = np.zeros(T + 1, np.int64)
    cpu = cpu_baseline_search(game, acts, offs, ids, ids + np.uint32(EVAL_OFFSET), sims,
                              args.cpu_seconds)
  if ctx.rank != 0:
    return None
  line = _base_line(args, ctx, "MCTS simulations/sec (random rollout) on %s, "
                    "root-parallel" % game, total_sims / elapsed, "sims/s", elapsed, {
                        "workload": "%s initial position, %d trees x %d sims per GPU, "
                                    "action-indexed root visits all-reduced" % (game, T, sims),
                        "game": game, "trees_per_gpu": T, "sims_per_tree": sims,
                        "parallelism": "root-parallel x%d (one RCCL all_reduce of "
                                       "f64[%d] = visits + rewards per step)"
                                       % (ctx.world, 2 * be.num_actions),
                        "layout": lay, "sims_per_step_per_gpu": sims_per_step})
  line["roofline"] = _roofline(KERNEL[lay], game, alg_bytes, kernel_ms, sims_per_step, "sim")
  line["arena"] = dict(arena, mode=arena_mode)
  line["cpu_baseline"] = cpu
  line["parity"] = parity
  line["root_visits_top5"] = sorted(
      ((int(n), int(a)) for a, n in enumerate(v.cpu().tolist())), reverse=True)[:5]
  line["tree_stats"] = stats
  return line


# ---------------------------------------------------------------------------
# c5: sharded random playouts (no tree)
def bench_playouts(args, ctx, layout):
  from os_amd import dist as D
  _, game, N, _, _ = CONFIGS[args.config]
  N = args.roots or N
  start, count = D.shard(N, ctx.world, ctx.rank)
  seeds = np.arange(start, start + count, dtype=np.uint32)
  be = ctx.backend(game)
  be.prepare_playouts([], seeds)

  def step():
    c = be.run_playouts()
    if ctx.world > 1:
      ctx.dist.all_reduce(c)
    return c

  for _ in range(args.warmup):
    c = step()
  returns = be.eng.rollouts_fetch()
  alg_bytes = None if ctx.rehearse else be.eng.rollouts_algorithmic_bytes(count)
  rstats = None if ctx.rehearse else be.eng.rollouts_stats()
  ret0 = returns[:, 0]
  local = np.array([(ret0 > 0).sum(), (ret0 < 0).sum(), (ret0 == 0).sum()], np.int64)
  lc = ctx.torch.from_numpy(local).to(ctx.dev)
  if ctx.world > 1:
    ctx.dist.all_reduce(lc)
  parity = None
  if ctx.rank == 0:
    # per-playout returns spot-checked on 4096 seeds spread
    # over the batch, plus the all-reduced outcome counts
    pick = np.arange(0, count, max(count // 4096, 1), dtype=np.int64)[:4096]
    ref = _oracle(game).rollouts([], seeds[pick])
    parity = {"playouts_checked": int(len(pick)),
              "bit_exact": bool(np.array_equal(ref, returns[pick])),
              "counts_equal_returns": bool(ctx.torch.equal(lc, c))}
  elapsed, kernel_ms = ctx.timed(step, args.steps)
  cpu = None
  if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
    cpu = cpu_baseline_playouts(game, args.cpu_seconds)
  if ctx.rank != 0:
    return None
  line = _base_line(args, ctx, "random playouts/sec on %s" % game, N * args.steps / elapsed,
                    "playouts/s", elapsed, {
                        "workload": "%s initial position, %d playouts split over %d GPUs"
                                    % (game, N, ctx.world),
                        "game": game, "playouts_total": N,
                        "parallelism": "sharded x%d (RCCL all_reduce int64[3] per step)"
                                       % ctx.world, "layout": "lane",
                        "playouts_per_step_per_gpu": count})
  line["roofline"] = (None if alg_bytes is None else
                      _roofline("k_rollouts", game, alg_bytes, kernel_ms, count, "playout"))
  line["playout_stats"] = rstats
  line["kernel_ms_per_launch"] = kernel_ms
  line["cpu_baseline"] = cpu
  line["parity"] = parity
  line["outcomes"] = {"p0_wins": int(c[0]), "p1_wins": int(c[1]), "draws": int(c[2])}
  return line


# ---------------------------------------------------------------------------
# sp: self-play games
def bench_selfplay(args, ctx, layout):
  from os_amd import engine as E
  _, game, G, sims, plies = CONFIGS[args.config]
  G = args.roots or G
  sims = args.sims or sims
  base = ctx.rank * G
  acts, offs = E.make_roots(game, G, seed_base=1000 + base, max_plies=plies)
  gid = np.arange(base, base + G, dtype=np.uint32)
  bot = np.stack([2 * gid, 2 * gid + 1], axis=1).astype(np.uint32)
  ev = gid + np.uint32(EVAL_OFFSET)
  eng = E.Engine(game, device=ctx.local)  # self-play: GPU only
  L = eng.max_game_length
  eng.selfplay_prepare(acts, offs, bot, ev, max_len=L, record_visits=True,
                       max_simulations=sims, uct_c=2.0)
  handle = ctx.handle
  for _ in range(args.warmup):
    eng.selfplay_run_async(handle)
  out = eng.selfplay_fetch()
  moves = int(out["length"].sum())
  sims_step = eng.last_sims()
  parity = None
  if ctx.rank == 0 and args.parity_roots > 0:
    pg = min(args.parity_roots, 8, G)
    ref = _oracle(game).selfplay(acts[:offs[pg]], offs[:pg + 1], bot[:pg], ev[:pg], L,
                                 max_simulations=sims)
    bad = [k for k in ("actions", "length", "returns", "visits")
           if not np.array_equal(out[k][:pg], ref[k])]
    parity = {"games_checked": pg, "bit_exact": not bad, "mismatch_fields": bad}
  elapsed, kernel_ms = ctx.timed(lambda: eng.selfplay_run_async(handle), args.steps)
  total_moves = ctx.total(moves * args.steps)
  total_sims = ctx.total(sims_step * args.steps)
  out = eng.selfplay_fetch()
  st = eng.stats()  # summed over the games of the last timed launch
  # Algorithmic bytes of one k_wselfplay launch: every move is
  # one search with the tree traffic of algorithmic_bytes (one root state per
  # move), plus the move's outputs -- its action (8 B) and the root's visit
  # row (4 B x num_distinct_actions, zeroed then filled).
  A = eng.num_distinct_actions
  alg = eng.algorithmic_bytes(moves) + moves * (8 + 4 * A)
  cpu = None
  if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
    cpu = cpu_baseline_selfplay(game, acts, offs, bot, ev, L, sims, args.cpu_seconds)
  if ctx.rank != 0:
    return None
  line = _base_line(args, ctx, "self-play MCTS moves/sec on %s (%d sims per move)"
                    % (game, sims), total_moves / elapsed, "moves/s", elapsed, {
                        "workload": "%s, %d games per GPU, two MCTSBots + shared "
                                    "RandomRolloutEvaluator per game, %d sims/move"
                                    % (game, G, sims),
                        "game": game, "games_per_gpu": G, "sims_per_move": sims,
                        "parallelism": "dp%d (independent games)" % ctx.world,
                        "layout": "wave", "moves_per_step_per_gpu": moves,
                        "sims_per_step_per_gpu": sims_step})
  line["sims_per_s"] = total_sims / elapsed
  line["kernel_ms_per_launch"] = kernel_ms
  line["roofline"] = _roofline("k_wselfplay", game, alg, kernel_ms, sims_step, "sim")
  line["cpu_baseline"] = cpu
  line["tree_stats"] = st
  line["parity"] = parity
  line["outcomes"] = {"p0_wins": int((out["returns"][:, 0] > 0).sum()),
                      "p1_wins": int((out["returns"][:, 0] < 0).sum()),
                      "draws": int((out["returns"][:, 0] == 0).sum())}
  return line


# ---------------------------------------------------------------------------
# az: external-evaluator PUCT search
def _az_network(obs_size, A, torch, dev, hidden=256):
  """A random-init policy/value MLP standing in for the AlphaZero network
  (bf16 matmuls, f64 priors/values at the boundary)."""
  g = torch.Generator().manual_seed(0)
  w1 = (torch.randn(obs_size, hidden, generator=g) / obs_size ** 0.5).to(dev, torch.bfloat16)
  wp = (torch.randn(hidden, A, generator=g) / hidden ** 0.5).to(dev, torch.bfloat16)
  wv = (torch.randn(hidden, 1, generator=g) / hidden ** 0.5).to(dev, torch.bfloat16)

  wpv = torch.cat([wp, wv], dim=1).contiguous()  # policy logits, then the value logit

  class Evaluator:
    def __call__(self, obs, legal, kind):  # the plain protocol (tensors out)
      x = obs.reshape(obs.shape[0], -1).to(torch.bfloat16)
      h = torch.relu(x @ w1)
      logits = (h @ wp).double().masked_fill(~legal, -1e32)
      prior = torch.softmax(logits, dim=-1)
      value = torch.tanh((h @ wv).double()).squeeze(-1)
      return prior, value

    def evaluate_into(self, obs, legal, kind, prior, value):
      # the whole round in one kernel: both products on the matrix cores,
      # then the heads write the engine's response buffers
      # (os_az_mlp_heads_async; the same network as __call__ above)
      mlp.heads_into(obs, legal, prior, value)

  from os_amd.az import MlpNetwork
  mlp = MlpNetwork(w1, wpv)
  return Evaluator()


def _az_toy_evaluator(A, torch):
  sys.path.insert(0, os.path.join(ROOT, "tests"))
  from test_az import toy_eval

  def evaluator(obs, legal, kind):
    ob = obs.cpu().numpy().reshape(obs.shape[0], -1)
    lg, kd = legal.cpu().numpy(), kind.cpu().numpy()
    pr = np.zeros((ob.shape[0], A), np.float64)
    v = np.zeros(ob.shape[0], np.float64)
    for i in np.nonzero(kd)[0]:
      pr[i], v[i] = toy_eval(ob[i], lg[i], int(kd[i]))
    return torch.from_numpy(pr).to(obs.device), torch.from_numpy(v).to(obs.device)
  return evaluator


def bench_az(args, ctx, layout):
  """One step = every search of the rank's batch run to completion: k_az_step
  launches alternating with one batched network call per launch."""
  from os_amd import engine as E
  from os_amd.az import ExternalEvaluatorSearch
  torch = ctx.torch
  _, game, R, sims, plies = CONFIGS[args.config]
  R = args.roots or R
  sims = args.sims or sims
  alpha, eps, c = 1.0, 0.25, 1.25
  base = ctx.rank * R
  acts, offs = E.make_roots(game, R, seed_base=1000 + base, max_plies=plies)
  seeds = np.arange(base, base + R, dtype=np.uint32)
  search = ExternalEvaluatorSearch(game, device=ctx.local)
  A = search.num_actions
  obs_size = int(np.prod(search.obs_shape))
  net = _az_network(obs_size, A, torch, ctx.dev)
  kw = dict(puct=True, max_simulations=sims, uct_c=c, dirichlet_alpha=alpha,
            dirichlet_epsilon=eps, stream=ctx.stream, requests=args.az_requests,
            block_size=args.block, layout=args.az_layout)
  parity = None
  if ctx.rank == 0 and args.parity_roots > 0:  # exact toy evaluator on a prefix vs the oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import test_az
    pr = min(args.parity_roots, R)
    got = search.run(acts[:offs[pr]], offs[:pr + 1], seeds[:pr], _az_toy_evaluator(A, torch),
                     **kw)
    ref = _oracle(game).mcts_external(
        acts[:offs[pr]], offs[:pr + 1], seeds[:pr], test_az._oracle_eval_fn(game), puct=True,
        uct_c=c, max_simulations=sims, max_children=search.eng.max_children,
        dirichlet_alpha=alpha, dirichlet_epsilon=eps)
    bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(got[k], ref[k])]
    parity = {"roots_checked": pr, "evaluator": "exact toy (tests/test_az.py)",
              "bit_exact": not bad, "mismatch_fields": bad}

  stage_kw = dict(puct=True, max_simulations=sims, uct_c=c, dirichlet_alpha=alpha,
                  dirichlet_epsilon=eps, block_size=args.block)
  pool = None
  pending = []
  if args.az_overlap:
    # Step k's batch was staged (host work: root replay, Dirichlet draws)
    # while step k-1 searched; step k stages step k+1's the same way.  The
    # first batch is staged before the warmup, the last staged batch is
    # never run (its host work is still inside the timed region).
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=1)
    search.stage(acts, offs, seeds, **stage_kw)

  def stage_next():
    pending.append(pool.submit(search.stage, acts, offs, seeds, **stage_kw))

  def step():
    if pool is None:
      search.run(acts, offs, seeds, net, graph=args.az_graph, **kw)
      return
    search.run(acts, offs, seeds, net, graph=args.az_graph, staged=True,
               after_prepare=stage_next, **kw)
    pending.pop().result()  # the next batch is staged

  for _ in range(args.warmup):
    step()
  elapsed, _ = ctx.timed(step, args.steps)
  if pool is not None:
    pool.shutdown()
  # One more instrumented run: per-launch k_az_step time and the tree stats.
  search.run(acts, offs, seeds, net, time_steps=True, **kw)
  step_ms = search.step_ms()
  launches = search.steps
  requests = search.requests
  st = search.eng.stats()  # of the run's final os_az_fetch
  sims_step = st["sims"]
  total_sims = ctx.total(sims_step * args.steps)
  if ctx.rank != 0:
    return None
  # Algorithmic bytes of the k_az_step launches of one search batch
  # (DESIGN.md §7): tree traffic as in the search kernels with 24-B f64 nodes
  # plus an 8-B prior per child read by PUCT; per request, the observation,
  # legal mask and kind written and the response read; per launch per live
  # search, its continuation header + working state read and written; fused
  # requests also park each leaf's priors (8 B per legal action, written once,
  # read at the expansion).
  sb = st["state_bytes"]
  nb = 24
  tree = (st["scanned"] * (nb + 8) + st["backed"] * 2 * nb + st["expanded"] * (nb + 8) +
          st["solver_scanned"] * nb + st["rng_words"] * 8)
  if args.az_requests == "fused":
    tree += (st["used"] - R) * 8 + st["expanded"] * 8
  io = requests * (obs_size * 4 + A + 4 + A * 8 + 8)
  cont = requests * 2 * (sb + 64)
  alg = tree + io + cont
  kernel_ms = step_ms / max(launches, 1)
  line = _base_line(args, ctx, "PUCT MCTS simulations/sec with a batched network evaluator "
                    "on %s" % game, total_sims / elapsed, "sims/s", elapsed, {
                        "workload": "%s, %d searches x %d sims per GPU, PUCT c=%g, Dirichlet "
                                    "alpha=%g eps=%g, random-init MLP evaluator (bf16, %d "
                                    "hidden) on the same GPU" % (game, R, sims, c, alpha, eps, 256),
                        "game": game, "searches_per_gpu": R, "sims_per_search": sims,
                        "parallelism": "dp%d (independent searches)" % ctx.world,
                        "layout": ("wave (k_waz_step: one wavefront per search)"
                                   if search.eng_az_wave() else
                                   "lane (k_az_step: one lane per search)"),
                        "searches_per_wave": 1 if search.eng_az_wave() else (args.block or 64),
                        "evaluator_requests": args.az_requests,
                        "rounds": "hip graph replay" if args.az_graph else "eager",
                        "host_prepare": ("staged on a worker thread during the previous "
                                         "step's search" if args.az_overlap else "serial"),
                        "sims_per_step_per_gpu": sims_step,
                        "units_per_launch": requests / max(launches, 1)})
  line["az"] = {"launches_per_step": launches, "requests_per_step": requests,
                "k_az_step_ms_total": step_ms,
                "k_az_step_share_of_step": step_ms / (elapsed / max(args.steps, 1) * 1e3),
                # the search alone (k_az_step time, no network): the figure
                # comparable with cpu_baseline, whose evaluator is free
                "search_only_sims_per_s": sims_step / max(step_ms * 1e-3, 1e-12)}
  line["roofline"] = _roofline("k_waz_step" if search.eng_az_wave() else "k_az_step", game,
                               alg / max(launches, 1), kernel_ms,
                               requests / max(launches, 1), "request")
  cpu = None
  if ctx.world == 1 and not args.no_cpu_baseline:
    cpu = cpu_baseline_az(game, acts, offs, seeds, sims, c, alpha, eps, args.cpu_seconds)
  line["cpu_baseline"] = cpu
  line["parity"] = parity
  line["tree_stats"] = st
  return line


# ---------------------------------------------------------------------------
# the other BASELINE configs, timed at full size after the headline line
# name: (timed steps, warmup steps).  C3 is ~1 s per step, g9 ~0.45 s.
SUB_CONFIGS = {"c3": (2, 1), "c4": (5, 1), "c5": (10, 2), "g9": (3, 1)}
SUB_CPU_SECONDS = 3.0


def timed_configs(args, ctx, layout):
  """C3, C4 (this GPU's share), C5 and g9 at their full BASELINE sizes, each
  timed exactly as its own `--config` run would be (barrier + sync around K
  steps), with its roofline, a >= 3 s CPU baseline and a bit-exact oracle
  prefix at the config's full depth (C3: 32 roots x 2048 sims; C4: 8 trees x
  2048 sims plus the device root sums against every tree; C5: 4096 seeds;
  g9: 32 roots x 256 sims).  Single-GPU only: at N > 1 the driver's per-N
  lines are the C2 headline."""
  import gc
  out = {}
  t_all = time.perf_counter()
  for name, (steps, warmup) in SUB_CONFIGS.items():
    sub = argparse.Namespace(**vars(args))
    sub.config, sub.steps, sub.warmup = name, steps, warmup
    sub.cpu_seconds, sub.parity_roots = SUB_CPU_SECONDS, 32
    sub.roots = sub.sims = sub.arena_nodes = sub.block = 0
    sub.arena = "auto"
    mode = CONFIGS[name][0]
    fn = {"search": bench_search, "root_parallel": bench_root_parallel,
          "playouts": bench_playouts}[mode]
    t0 = time.perf_counter()
    try:
      line = fn(sub, ctx, layout)
    except Exception as e:  # reported in the line, never hidden
      line = {"error": "%s: %s" % (type(e).__name__, e)}
    gc.collect()  # the config's engine (and its arena) goes before the next one
    line["seconds_total"] = round(time.perf_counter() - t0, 2)
    for k in ("tree_stats", "n_gpus", "higher_is_better", "data"):
      line.pop(k, None)
    out[name] = line
  out["all_bit_exact"] = all(_entry_exact(v) for v in out.values() if isinstance(v, dict))
  out["seconds"] = round(time.perf_counter() - t_all, 2)
  return out


def _entry_exact(line):
  p = line.get("parity")
  if not p:
    return False
  flags = [p.get("bit_exact"), p.get("timed_run_bit_exact", True),
           p.get("allreduce_equals_sum_of_trees", True), p.get("counts_equal_returns", True)]
  return all(bool(f) for f in flags)


# ---------------------------------------------------------------------------
# parity sweep: every kernel of the library, bit-exact against the oracle
def parity_sweep(ctx):
  """Runs after the C2 timed region on rank 0 (never timed): one reduced-size
  case per kernel / layout / policy the library ships, each compared
  bit-exactly with the oracle (mcts.cc:325-428 searches,
  :42-71 playouts).  The sizes keep the whole sweep to seconds, while the
  launches keep each config's full width where that is what a kernel's
  indexing depends on (C3's 65536 searches on the paged arena, C4's 8192
  trees, C5's 2^20 playouts).  Returns {case: {...,"bit_exact": bool}} plus
  "all_bit_exact"."""
  from os_amd import _lib
  from os_amd import engine as E
  torch = ctx.torch
  res = {}
  t_start = time.perf_counter()

  def cmp(got, ref, keys=E.OUTPUT_KEYS, rows=None):
    sel = (lambda a: a) if rows is None else (lambda a: a[rows])
    return [k for k in keys if not np.array_equal(sel(got[k]), ref[k])]

  def case(name, fn):
    t0 = time.perf_counter()
    try:
      r = fn()
    except Exception as e:  # a failing case is reported, not hidden
      r = {"bit_exact": False, "error": "%s: %s" % (type(e).__name__, e)}
    r["seconds"] = round(time.perf_counter() - t0, 3)
    res[name] = r

  def seeds(R, mul=1, add=0):
    b = np.arange(R, dtype=np.uint32) * np.uint32(mul) + np.uint32(add)
    return b, b + np.uint32(EVAL_OFFSET)

  def c3():
    # C3 shape: 65536 breakthrough 8x8 roots on the paged arena (the pool
    # sized by a first reserved run), 256 sims (a page must fit twice in the
    # worst-case reservation for paging to apply); first and last 64 roots.
    gs, R, sims = "breakthrough(rows=8,columns=8)", 65536, 256
    acts, offs = E.make_roots(gs, R, seed_base=1000, max_plies=6)
    bs, es = seeds(R)
    eng = E.Engine(gs, device=ctx.local)
    kw = dict(uct_c=2.0, max_simulations=sims)
    eng.set_arena_mode("paged")
    eng.prepare(acts, offs, bs, es, **kw)
    eng.run_async(ctx.handle)
    eng.fetch()
    eng.prepare(acts, offs, bs, es, **kw)
    eng.run_async(ctx.handle)
    got = eng.fetch()
    info = eng.arena_info()
    og = _oracle(gs)
    rows = np.r_[0:64, R - 64:R]
    sub_offs = np.concatenate([offs[:65], offs[R - 63:R + 1] - offs[R - 64] + offs[64]])
    sub_acts = np.concatenate([acts[:offs[64]], acts[offs[R - 64]:offs[R]]])
    ref = og.mcts_batch(sub_acts, sub_offs, bs[rows], es[rows], max_children=eng.max_children,
                        threads=host_cores()[0], **kw)
    bad = cmp(got, ref, rows=rows)
    eng.close()
    return {"roots": R, "sims": sims, "roots_checked": 128, "paged": bool(info["paged"]),
            "reruns": info["reruns"], "bit_exact": not bad and bool(info["paged"]),
            "mismatch_fields": bad}

  def c4():
    # C4 shape: 8192 hex-11 trees on the initial position (paged), 256 sims;
    # device action-indexed root sums vs the fetched children, 16-tree prefix.
    gs, T, sims = "hex(board_size=11)", 8192, 256
    eng = E.Engine(gs, device=ctx.local)
    A = eng.num_distinct_actions
    bs, es = seeds(T)
    acts, offs = np.zeros(0, np.int64), np.zeros(T + 1, np.int64)
    kw = dict(uct_c=2.0, max_simulations=sims)
    eng.set_arena_mode("paged")
    eng.prepare(acts, offs, bs, es, **kw)
    eng.run_async(ctx.handle)
    eng.fetch()
    eng.prepare(acts, offs, bs, es, **kw)
    eng.run_async(ctx.handle)
    v = torch.empty(A, dtype=torch.int64, device=ctx.dev)
    w = torch.empty(A, dtype=torch.float64, device=ctx.dev)
    eng.root_sums_async(A, v.data_ptr(), w.data_ptr(), ctx.handle)
    got = eng.fetch()
    paged = bool(eng.arena_info()["paged"])
    lv, lw = np.zeros(A, np.int64), np.zeros(A, np.float64)
    for r in range(T):
      nc = int(got["nchild"][r])
      np.add.at(lv, got["child_action"][r, :nc], got["child_n"][r, :nc])
      np.add.at(lw, got["child_action"][r, :nc], got["child_w"][r, :nc])
    sums_ok = (np.array_equal(v.cpu().numpy(), lv) and np.array_equal(w.cpu().numpy(), lw))
    ref = _oracle(gs).mcts_batch(acts, offs[:17], bs[:16], es[:16],
                                 max_children=eng.max_children, threads=host_cores()[0], **kw)
    bad = cmp(got, ref, rows=slice(0, 16))
    eng.close()
    return {"trees": T, "sims": sims, "trees_checked": 16, "paged": paged,
            "root_sums_equal_children": bool(sums_ok),
            "bit_exact": not bad and bool(sums_ok), "mismatch_fields": bad}

  def c5():
    gs, N = "go(board_size=9)", 1 << 20
    eng = E.Engine(gs, device=ctx.local)
    s = np.arange(N, dtype=np.uint32)
    eng.rollouts_prepare([], s)
    eng.rollouts_run_async(ctx.handle)
    c = torch.empty(3, dtype=torch.int64, device=ctx.dev)
    eng.rollouts_outcomes_async(c.data_ptr(), ctx.handle)
    ret = eng.rollouts_fetch()
    pick = np.arange(0, N, N // 4096, dtype=np.int64)[:4096]
    ref = _oracle(gs).rollouts([], s[pick])
    r0 = ret[:, 0]
    counts = [int((r0 > 0).sum()), int((r0 < 0).sum()), int((r0 == 0).sum())]
    cok = c.cpu().tolist() == counts
    eng.close()
    return {"playouts": N, "playouts_checked": 4096, "device_counts_equal_returns": cok,
            "bit_exact": bool(np.array_equal(ret[pick], ref)) and cok}

  def search(gs, R, sims, plies, layout, seed_mul=1, **kw):
    def fn():
      acts, offs = E.make_roots(gs, R, seed_base=4242, max_plies=plies)
      bs, es = seeds(R, seed_mul, 1)
      eng = E.Engine(gs, device=ctx.local)
      got = eng.mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                           layout=layout, **kw)
      puct = kw.pop("child_selection", 0) == _lib.SELECT_PUCT
      ref = _oracle(gs).mcts_batch(acts, offs, bs, es, uct_c=2.0, max_simulations=sims,
                                   max_children=eng.max_children, threads=host_cores()[0],
                                   puct=puct, **kw)
      bad = cmp(got, ref)
      eng.close()
      return {"roots": R, "sims": sims, "bit_exact": not bad, "mismatch_fields": bad}
    return fn

  def numpy_policy(gs, histories, sims):
    # python/algorithms/mcts.py semantics: one RandomState shared by the bot
    # and its evaluator (mcts_test.py:41-54), continued across the search.
    def fn():
      eng = E.Engine(gs, device=ctx.local)
      og = _oracle(gs)
      bad = []
      for i, h in enumerate(histories):
        seed = 17 + i
        _, key, pos, _, _ = np.random.RandomState(seed).get_state()
        got, (k2, p2), _ = eng.mcts_stateful(h, (key, pos), None, uct_c=2.0,
                                             max_simulations=sims, policy=_lib.POLICY_NUMPY)
        ref = og.mcts_numpy(h, seed, uct_c=2.0, max_simulations=sims)
        rs = np.random.RandomState()
        rs.set_state(("MT19937", k2, p2, 0, 0.0))
        bad += cmp(got, ref)
        if rs.randint(0, 2 ** 32, dtype=np.uint32) != ref["next_word"][0]:
          bad.append("random_state_after")
      eng.close()
      return {"searches": len(histories), "sims": sims, "bit_exact": not bad,
              "mismatch_fields": sorted(set(bad))}
    return fn

  W, L = _lib.LAYOUT_WAVE, _lib.LAYOUT_LANE
  PUCT = _lib.SELECT_PUCT
  case("c3_breakthrough_65536_paged", c3)
  case("c4_hex11_8192_root_sums", c4)
  case("c5_go9_2^20_playouts", c5)
  case("go9_lane_layout", search("go(board_size=9)", 72, 160, 8, L))
  case("go9_wave_layout", search("go(board_size=9)", 8, 96, 8, W))
  case("tic_tac_toe_wave", search("tic_tac_toe", 64, 1000, 4, W))
  case("connect_four_lane", search("connect_four", 64, 1024, 8, L))
  case("puct_connect_four_wave", search("connect_four", 64, 512, 8, W, child_selection=PUCT))
  case("puct_hex5_lane", search("hex(board_size=5)", 64, 400, 6, L, child_selection=PUCT,
                                n_rollouts=2, solve=False))
  case("numpy_policy_connect_four", numpy_policy("connect_four", [[], [3, 3, 2], [0, 6]], 500))
  case("numpy_policy_go9", numpy_policy("go(board_size=9)", [[], [40]], 120))
  case("pig_3p_chance", search("pig(players=3)", 64, 300, 6, L))
  res["all_bit_exact"] = all(v.get("bit_exact") for v in res.values() if isinstance(v, dict))
  res["seconds"] = round(time.perf_counter() - t_start, 2)
  return res


# ---------------------------------------------------------------------------
def _oracle(game):
  sys.path.insert(0, os.path.join(ROOT, "tests"))
  import oracle_lib
  return oracle_lib.Game(game)


def calibration(game):
  """Restatement/reference CPU speed ratio for `game`, measured in the build
  container by tools/calibrate_cpu.py against SURVEY.md §6's single-core
  probes of the (shim-built) reference mcts.cc on the same CPU."""
  path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
  key = game if game.startswith("go") else game.split("(")[0]
  try:
    with open(path) as f:
      g = json.load(f)["games"][key]
  except (OSError, KeyError, ValueError):
    return "uncalibrated: no profiles/cpu_calibration.json entry for %s" % game
  return {"oracle_over_reference": g["ratio"], "oracle_sims_per_s_1core": g["oracle_sims_per_s"],
          "reference_sims_per_s_1core": g["reference_sims_per_s"], "sims": g["sims"],
          "conditions": "initial position, seeds 1-3, one thread, build container",
          "source": "profiles/cpu_calibration.json (tools/calibrate_cpu.py; SURVEY.md §6)"}


def host_cores():
  """CPUs this process may actually run on: the affinity mask, capped by the
  cgroup CPU quota when one is set (a GPU box shares its host; nproc there
  shows the whole machine).  Returns (threads, description)."""
  aff = len(os.sched_getaffinity(0))
  quota = None
  try:
    with open("/sys/fs/cgroup/cpu.max") as f:
      q, period = f.read().split()
    if q != "max":
      quota = max(1, int(int(q) // int(period)))
  except (OSError, ValueError):
    pass
  threads = aff if quota is None else min(aff, quota)
  desc = "nproc %d, affinity %d, cgroup quota %s -> %d threads" % (
      os.cpu_count() or 0, aff, "none" if quota is None else "%d CPUs" % quota, threads)
  return threads, desc


def cpu_baseline_search(game, acts, offs, bot_seeds, eval_seeds, sims, seconds):
  """Oracle (reference-faithful restatement, "port") on every usable host core;
  the batch (or a prefix of it) is repeated until >= `seconds` are timed."""
  og = _oracle(game)
  threads, cores_desc = host_cores()
  R = len(offs) - 1
  # Calibrate on a small prefix, then size one pass to ~`seconds` (<= R roots).
  probe = min(R, 2 * threads)
  secs, n = og.time_mcts_batch(acts[:offs[probe]], offs[:probe + 1], bot_seeds[:probe],
                               eval_seeds[:probe], max_simulations=sims, threads=threads)
  per_root = max(secs, 1e-9) / probe * threads  # seconds per root on one thread
  want = int(min(R, max(probe, seconds * threads / per_root)))
  total_s, total_n, passes = 0.0, 0, 0
  while total_s < seconds or passes == 0:
    secs, n = og.time_mcts_batch(acts[:offs[want]], offs[:want + 1], bot_seeds[:want],
                                 eval_seeds[:want], max_simulations=sims, threads=threads)
    total_s, total_n, passes = total_s + secs, total_n + n, passes + 1
  cal = calibration(game)
  ref_eq = (total_n / total_s / cal["oracle_over_reference"]) if isinstance(cal, dict) else None
  return {"value": total_n / total_s, "unit": "sims/s", "cores": threads, "kind": "port",
          "calibration": cal, "reference_equivalent": ref_eq,
          "sample": "%d pass(es) over %d of the %d roots x %d sims (%d sims, %.1f s), "
                    "oracle restatement of mcts.cc; %s" %
                    (passes, want, R, sims, total_n, total_s, cores_desc)}


def cpu_baseline_selfplay(game, acts, offs, bot, ev, max_len, sims, seconds):
  """Oracle self-play (two MCTSBots + shared RandomRolloutEvaluator per game,
  oracle/ref_capi.cc oref_selfplay) on every usable host core over a prefix
  of the same games, grown until one pass takes >= `seconds`."""
  og = _oracle(game)
  threads, cores_desc = host_cores()
  G = len(offs) - 1
  n = min(G, threads)
  secs = moves = passes = 0
  while secs < seconds:
    t0 = time.perf_counter()
    r = og.selfplay(acts[:offs[n]], offs[:n + 1], bot[:n], ev[:n], max_len,
                    max_simulations=sims, with_visits=False, threads=threads)
    dt = time.perf_counter() - t0
    if n < G and dt < seconds:  # grow the prefix; time only full-size passes
      n = min(G, max(n + threads, int(n * min(8.0, 1.2 * seconds / max(dt, 1e-3)))))
      continue
    secs, moves, passes = secs + dt, moves + int(r["length"].sum()), passes + 1
  cal = calibration(game)
  ref_eq = (moves / secs / cal["oracle_over_reference"]) if isinstance(cal, dict) else None
  return {"value": moves / secs, "unit": "moves/s", "cores": threads, "kind": "port",
          "calibration": cal, "reference_equivalent": ref_eq,
          "sample": "%d pass(es) over %d of the %d games (%d moves x %d sims, %.1f s), oracle "
                    "restatement of two MCTSBots sharing one RandomRolloutEvaluator; %s" %
                    (passes, n, G, moves, sims, secs, cores_desc)}


def cpu_baseline_az(game, acts, offs, seeds, sims, uct_c, alpha, eps, seconds):
  """Oracle MCTSBot PUCT searches with Dirichlet root noise and a native
  evaluator that costs nothing (uniform prior, zero value;
  oref_time_mcts_zero_eval): the host's search speed with the network's time
  excluded, on every usable host core."""
  og = _oracle(game)
  threads, cores_desc = host_cores()
  R = len(offs) - 1
  n = min(R, 2 * threads)
  secs = done = passes = 0
  while secs < seconds:
    dt, k = og.time_mcts_zero_eval(acts[:offs[n]], offs[:n + 1], seeds[:n], uct_c=uct_c,
                                   max_simulations=sims, puct=True, dirichlet_alpha=alpha,
                                   dirichlet_epsilon=eps, threads=threads)
    if n < R and dt < seconds:
      n = min(R, max(n + threads, int(n * min(8.0, 1.2 * seconds / max(dt, 1e-3)))))
      continue
    secs, done, passes = secs + dt, done + k, passes + 1
  return {"value": done / secs, "unit": "sims/s", "cores": threads, "kind": "port",
          "sample": "%d pass(es) over %d of the %d searches x %d sims (%d sims, %.1f s), "
                    "oracle MCTSBot (PUCT, Dirichlet) with a free native evaluator -- "
                    "network time excluded, the GPU line's included; %s" %
                    (passes, n, R, sims, done, secs, cores_desc)}


def cpu_baseline_playouts(game, seconds):
  """Oracle RandomRolloutEvaluator::Evaluate on host threads (ctypes drops the GIL)."""
  threads, cores_desc = host_cores()
  t0 = time.perf_counter()
  _oracle(game).rollouts([], np.arange(64, dtype=np.uint32))
  per = (time.perf_counter() - t0) / 64
  n_per = max(64, int(seconds / per))
  games = [_oracle(game) for _ in range(threads)]

  def work(i):
    games[i].rollouts([], np.arange(i * n_per, (i + 1) * n_per, dtype=np.uint32))

  ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
  t0 = time.perf_counter()
  for t in ths:
    t.start()
  for t in ths:
    t.join()
  secs = time.perf_counter() - t0
  return {"value": threads * n_per / secs, "unit": "playouts/s", "cores": threads,
          "kind": "port", "calibration": calibration(game),
          "sample": "%d playouts (seeds 0..%d), %.1f s, oracle restatement of "
                    "RandomRolloutEvaluator; %s" % (threads * n_per, threads * n_per - 1,
                                                    secs, cores_desc)}


# Host-side units: the C-ABI, batch preparation and the small reduction
# kernels (k_root_*, k_outcome_counts, k_sum_devices); the PMC'd kernels
# (k_wsearch, k_mcts, k_rollouts, k_az_step, k_wselfplay) do not include them.
HOST_UNITS = ("os_engine.hip", "os_host.cpp", "os_host.h", "Makefile")


def kernel_source_hash():
  """sha256 over the sources of the PMC'd kernels (csrc/* minus the host
  units): ties a PMC record to the code it was collected on
  (tools/pmc_summary.py stores the same hash)."""
  h = hashlib.sha256()
  src = os.path.join(ROOT, "open_spiel-1_amd", "csrc")
  for name in sorted(os.listdir(src)):
    if name.endswith((".h", ".hip", ".cpp")) and name not in HOST_UNITS:
      with open(os.path.join(src, name), "rb") as f:
        h.update(name.encode() + b"\0" + f.read())
  return h.hexdigest()[:16]


def pmc_record(kernel, game):
  """rocprofv3 PMC summary of `kernel` on `game` (profiles/pmc_traffic.json,
  written by tools/pmc_summary.py), or None."""
  path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
  if not os.path.exists(path):
    return None
  with open(path) as f:
    d = json.load(f)
  return d.get("%s/%s" % (kernel, game.split("(")[0]))


def _pmc_provenance(pmc):
  if not pmc:
    return None
  src = pmc.get("source_hash")
  return {"source_hash": src, "current_source_hash": kernel_source_hash(),
          "stale": src != kernel_source_hash()}


if __name__ == "__main__":
  main()
