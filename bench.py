#!/usr/bin/env python3
"""Headline benchmark: random-rollout MCTS simulations/s on connect_four.

BASELINE.json metric: "MCTS simulations/sec (random rollout) on connect_four
at 1/2/4/8 MI355X"; workload = configs[1]: 4096 independent roots x 1024
simulations per GPU (weak scaling: every rank searches its own 4096 roots,
seeded by global root id; no data-path collective).

One step = one pass of the search kernel over the rank's whole batch (roots
and seeds already resident in HBM).  Rank 0 prints ONE JSON line.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (game string, roots per GPU, sims, root plies)
    "c2": ("connect_four", 4096, 1024, 8),
    "c3": ("breakthrough(rows=8,columns=8)", 65536, 2048, 6),
}


LAYOUTS = {}
KERNEL = {"wave": "k_wsearch", "lane": "k_mcts"}


def parse():
  ap = argparse.ArgumentParser()
  ap.add_argument("--gpus", type=int, default=1)
  ap.add_argument("--steps", type=int, default=5)
  ap.add_argument("--warmup", type=int, default=2)
  ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
  ap.add_argument("--roots", type=int, default=0, help="override roots per GPU")
  ap.add_argument("--sims", type=int, default=0, help="override simulations")
  ap.add_argument("--block", type=int, default=0, help="lanes per workgroup")
  ap.add_argument("--arena-nodes", type=int, default=0)
  ap.add_argument("--layout", default="wave", choices=("wave", "lane"),
                  help="search kernel: one wave per search / one lane per search")
  ap.add_argument("--no-cpu-baseline", action="store_true")
  ap.add_argument("--cpu-seconds", type=float, default=12.0,
                  help="target CPU-baseline sample duration")
  ap.add_argument("--parity-roots", type=int, default=32)
  return ap.parse_args()


def main():
  args = parse()
  import torch
  import torch.distributed as dist
  from os_amd import engine as E
  from os_amd import _lib
  LAYOUTS.update(wave=_lib.LAYOUT_WAVE, lane=_lib.LAYOUT_LANE)

  world = int(os.environ.get("WORLD_SIZE", "1"))
  rank = int(os.environ.get("RANK", "0"))
  local = int(os.environ.get("LOCAL_RANK", "0"))
  if world != args.gpus and world > 1:
    raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
  torch.cuda.set_device(local)
  if world > 1:
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))

  game, R, sims, plies = CONFIGS[args.config]
  R = args.roots or R
  sims = args.sims or sims
  params = dict(uct_c=2.0, max_simulations=sims, n_rollouts=1,
                max_memory_mb=1000, solve=True, block_size=args.block,
                arena_nodes=args.arena_nodes, layout=LAYOUTS[args.layout])
  base = rank * R  # global root ids of this rank
  acts, offs = E.make_roots(game, R, seed_base=1000 + base, max_plies=plies)
  gid = np.arange(base, base + R, dtype=np.uint32)
  bot_seeds = gid
  eval_seeds = gid + np.uint32(1 << 20)

  eng = E.Engine(game, device=local)
  eng.prepare(acts, offs, bot_seeds, eval_seeds, **params)
  stream = torch.cuda.current_stream()
  handle = stream.cuda_stream

  for _ in range(args.warmup):
    eng.run_async(handle)
  out = eng.fetch()  # synchronises; validates per-root status
  sims_per_step = eng.last_sims()
  alg_bytes = eng.algorithmic_bytes(R)
  stats = eng.stats()

  # Parity spot check against the oracle (rank 0, a prefix of the batch).
  parity = None
  cpu = None
  if rank == 0:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    og = oracle_lib.Game(game)
    pr = min(args.parity_roots, R)
    ref = og.mcts_batch(acts[:offs[pr]], offs[:pr + 1], bot_seeds[:pr],
                        eval_seeds[:pr], uct_c=2.0, max_simulations=sims,
                        max_children=eng.max_children)
    bad = [k for k in E.OUTPUT_KEYS if not np.array_equal(out[k][:pr], ref[k])]
    parity = {"roots_checked": pr, "bit_exact": not bad, "mismatch_fields": bad}

  if world > 1:
    dist.barrier()
  torch.cuda.synchronize()
  ev0 = torch.cuda.Event(enable_timing=True)
  ev1 = torch.cuda.Event(enable_timing=True)
  t0 = time.perf_counter()
  ev0.record(stream)
  for _ in range(args.steps):
    eng.run_async(handle)
  ev1.record(stream)
  torch.cuda.synchronize()
  if world > 1:
    dist.barrier()
  t1 = time.perf_counter()
  elapsed = t1 - t0
  kernel_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)

  total_sims = sims_per_step * args.steps
  if world > 1:
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    s = torch.tensor([total_sims], dtype=torch.float64, device="cuda")
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    total_sims = int(s.item())

  if rank == 0 and args.gpus == 1 and not args.no_cpu_baseline:
    cpu = cpu_baseline(game, acts, offs, bot_seeds, eval_seeds, sims,
                       args.cpu_seconds)

  if rank == 0:
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
    traffic = pmc_traffic(KERNEL[args.layout], game)
    line = {
        "metric": "MCTS simulations/sec (random rollout) on connect_four at "
                  "1/2/4/8 MI355X" if args.config == "c2" else
                  "MCTS simulations/sec (random rollout) on %s" % game,
        "value": total_sims / elapsed,
        "unit": "sims/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32+f64",
        "data": "synthetic (seeded random roots; no dataset)",
        "config": {
            "workload": "%s, %d independent roots x %d sims per GPU" %
                        (game, R, sims),
            "game": game, "roots_per_gpu": R, "sims_per_root": sims,
            "uct_c": 2.0, "n_rollouts": 1, "solve": True,
            "max_memory_mb": 1000, "root_plies": "k~U[0,%d] from mt19937(1000+i)" % plies,
            "parallelism": "dp%d (independent roots, no collective)" % world,
            "layout": args.layout,
            "block_size": args.block or (64 if args.layout == "wave" else 16),
            "sims_per_step_per_gpu": sims_per_step,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel": KERNEL[args.layout],
            "kernel_ms_per_launch": kernel_ms,
            "algorithmic_bytes_per_launch": alg_bytes,
            "algorithmic_bytes_per_sim": alg_bytes / max(sims_per_step, 1),
        },
        "cpu_baseline": cpu,
        "parity": parity,
        "tree_stats": stats,
    }
    print(json.dumps(line), flush=True)
  if world > 1:
    dist.destroy_process_group()


def cpu_baseline(game, acts, offs, bot_seeds, eval_seeds, sims, seconds):
  """Oracle (reference-faithful restatement, "port") on the host cores."""
  sys.path.insert(0, os.path.join(ROOT, "tests"))
  import oracle_lib
  og = oracle_lib.Game(game)
  threads = max(1, min(16, len(os.sched_getaffinity(0))))
  R = len(offs) - 1
  # Calibrate on a small prefix, then size the sample to ~`seconds`.
  probe = min(R, 8 * threads)
  secs, n = og.time_mcts_batch(acts[:offs[probe]], offs[:probe + 1],
                               bot_seeds[:probe], eval_seeds[:probe],
                               max_simulations=sims, threads=threads)
  rate = n / max(secs, 1e-9)
  want = int(min(R, max(probe, seconds * rate / max(n / probe, 1))))
  secs, n = og.time_mcts_batch(acts[:offs[want]], offs[:want + 1],
                               bot_seeds[:want], eval_seeds[:want],
                               max_simulations=sims, threads=threads)
  return {"value": n / secs, "unit": "sims/s", "cores": threads,
          "kind": "port",
          "sample": "%d of the %d roots x %d sims (%d sims, %.1f s), oracle "
                    "restatement of mcts.cc, %d threads" %
                    (want, R, sims, n, secs, threads)}


def pmc_traffic(kernel, game):
  """HBM bytes per launch of `kernel` on `game` from the committed rocprofv3
  PMC summary (profiles/pmc_traffic.json, written by tools/pmc_summary.py)."""
  path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
  if not os.path.exists(path):
    return None
  with open(path) as f:
    d = json.load(f)
  return d.get("%s/%s" % (kernel, game), {}).get("hbm_bytes_per_launch")


if __name__ == "__main__":
  main()
