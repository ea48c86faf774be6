#!/usr/bin/env python3
"""One-root `step` latency of the drop-in bots, per game.

For each game, from the initial position, at the reference's simulation
count (1000, python/examples/mcts.py and SURVEY §8d C1):
  cpp_step_ms     pyspiel.MCTSBot.step (C++ MCTSBot semantics), wall
  py_step_ms      open_spiel.python.algorithms.mcts.MCTSBot.step (numpy), wall
  kernel_ms       the device time of the search inside each timed step: the
                  engine brackets its launch with HIP events
                  (os_engine_set_run_timing), read after the step returns
  host_overhead   median over reps of (step - that step's kernel time)
  oracle_1core_ms the oracle MCTSBot (reference-faithful restatement of
                  mcts.cc) for the same search on one host core
Writes JSON + a markdown table to --out (default profiles/r04/step_latency).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "open_spiel-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

GAMES = ["tic_tac_toe", "connect_four", "breakthrough", "hex", "go(board_size=9)",
         "pig"]


def _median_ms(fn, reps):
  ts = []
  for _ in range(reps):
    t0 = time.perf_counter()
    fn()
    ts.append((time.perf_counter() - t0) * 1e3)
  return float(np.median(ts)), ts


def measure(gs, sims, reps, torch):
  import pyspiel
  from open_spiel.python.algorithms import mcts
  from os_amd import engine as E
  import oracle_lib as O
  game = pyspiel.load_game(gs)
  st = game.new_initial_state()
  if st.is_chance_node():
    st.apply_action(st.legal_actions()[0])
  hist = st.history()
  # the drop-in bots: a fresh bot per timed step (built outside the timing), so
  # every timed step is the first search of seeds (3, 7) / RandomState(3) --
  # the same search the kernel-only timing below runs (the first call warms
  # the engine and its arena)
  def cpp_bot():
    return pyspiel.MCTSBot(game, pyspiel.RandomRolloutEvaluator(1, 7), 2.0, sims, 1000, True,
                           3, False)

  def py_bot():
    rs = np.random.RandomState(3)
    return mcts.MCTSBot(game, 2.0, sims, mcts.RandomRolloutEvaluator(1, rs), random_state=rs,
                        solve=True, backend="hip")

  acts = np.array(hist, np.int64)
  offs = np.array([0, len(hist)], np.int64)
  # Step and kernel in the SAME run: the engine the bots drive brackets each
  # search launch with a HIP event pair (os_engine_set_run_timing); every rep
  # reads its own step's kernel time after the step returns.
  from os_amd import _lib
  from os_amd import pyspiel as ospy
  eng = ospy._engine_for(game)
  _lib.check(_lib.lib.os_engine_set_run_timing(eng._h, 1))
  kms = np.zeros(1, np.float64)

  def step_and_kernel(make):
    steps, kernels = [], []
    for _ in range(reps):
      bot = make()
      t0 = time.perf_counter()
      bot.step(st)
      steps.append((time.perf_counter() - t0) * 1e3)
      _lib.check(_lib.lib.os_engine_last_run_ms(eng._h, _lib.ptr(kms)))
      kernels.append(float(kms[0]))
    return steps, kernels

  cpp_bot().step(st)  # warm the engine and its arena
  cpp_steps, cpp_kernels = step_and_kernel(cpp_bot)
  py_bot().step(st)
  py_steps, py_kernels = step_and_kernel(py_bot)
  _lib.check(_lib.lib.os_engine_set_run_timing(eng._h, 0))
  cpp_ms, kernel_ms = float(np.median(cpp_steps)), float(np.median(cpp_kernels))
  py_ms, np_kernel_ms = float(np.median(py_steps)), float(np.median(py_kernels))
  # per-rep host overhead (step - its own kernel), median
  cpp_over = float(np.median(np.array(cpp_steps) - np.array(cpp_kernels)))
  py_over = float(np.median(np.array(py_steps) - np.array(py_kernels)))
  # oracle, one core
  og = O.Game(gs)
  osecs = []
  for _ in range(max(3, reps // 2)):
    s, _n = og.time_mcts_batch(acts, offs, np.array([3], np.uint32), np.array([7], np.uint32),
                               max_simulations=sims, threads=1)
    osecs.append(s * 1e3)
  return {"game": gs, "sims": sims, "cpp_step_ms": cpp_ms, "py_step_ms": py_ms,
          "kernel_ms": kernel_ms, "host_overhead_ms": cpp_over,
          "host_overhead_frac": cpp_over / kernel_ms,
          "np_kernel_ms": np_kernel_ms, "py_overhead_ms": py_over,
          "py_overhead_frac": py_over / np_kernel_ms,
          "cpp_steps_ms": cpp_steps, "cpp_kernels_ms": cpp_kernels,
          "py_steps_ms": py_steps, "py_kernels_ms": py_kernels,
          "oracle_1core_ms": float(np.median(osecs)),
          "gpu_over_oracle": float(np.median(osecs)) / cpp_ms}


def measure_az(gs, sims, reps):
  """One `mcts.MCTSBot.step` of the reference's AlphaZero bot construction
  (alpha_zero.py:185-192: PUCT, Dirichlet (0.25, 1.0), solve=False, uct_c 2,
  the example's 300 simulations) over the AlphaZeroEvaluator drop-in, on the
  device (backend="hip", one evaluator round per simulation) and in the host
  loop (backend="host").  The network is tests/az_toy_model.ToyModel, which
  costs the same few microseconds per call on both paths, so the difference
  is the search machinery.  Both paths must choose the same action and leave
  the RandomState in the same place."""
  import pyspiel
  from open_spiel.python.algorithms import mcts
  from os_amd.az_evaluator import AlphaZeroEvaluator
  from az_toy_model import ToyModel
  game = pyspiel.load_game(gs)
  st = game.new_initial_state()
  model = ToyModel(int(np.prod(game.observation_tensor_shape())), game.num_distinct_actions())

  def bot(backend):
    rs = np.random.RandomState(3)
    ev = AlphaZeroEvaluator(game, model)
    return mcts.MCTSBot(game, 2.0, sims, ev, solve=False, random_state=rs,
                        dirichlet_noise=(0.25, 1.0),
                        child_selection_fn=mcts.SearchNode.puct_value, backend=backend), rs

  row = {"game": gs, "sims": sims, "model": "ToyModel (float64)"}
  picks = {}
  for backend in ("hip", "host"):
    b, _ = bot(backend)
    b.step(st)  # warm: engine, arena, kernels
    ts = []
    for _ in range(reps):
      b, rs = bot(backend)
      t0 = time.perf_counter()
      a = b.step(st)
      ts.append((time.perf_counter() - t0) * 1e3)
    picks[backend] = (a, rs.get_state()[2])
    row[backend + "_step_ms"] = float(np.median(ts))
    row[backend + "_steps_ms"] = ts
  row["same_action_and_stream"] = picks["hip"] == picks["host"]
  row["faster"] = "hip" if row["hip_step_ms"] < row["host_step_ms"] else "host"
  return row


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--az", action="store_true",
                  help="the AlphaZero bot drop-in (device vs host loop) instead")
  ap.add_argument("--az-sims", type=int, default=300)
  ap.add_argument("--sims", type=int, default=1000)
  ap.add_argument("--reps", type=int, default=10)
  ap.add_argument("--games", default=",".join(GAMES))
  ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "step_latency"))
  args = ap.parse_args()
  import torch
  torch.cuda.init()
  if args.az:
    rows = []
    for gs in ("connect_four", "tic_tac_toe"):
      r = measure_az(gs, args.az_sims, args.reps)
      rows.append(r)
      print(json.dumps(r), flush=True)
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, "az_step_latency.json"), "w") as f:
      json.dump(rows, f, indent=1)
    with open(os.path.join(args.out, "az_step_latency.md"), "w") as f:
      f.write("| game | sims | device step ms (backend=hip) | host loop step ms (backend=host) "
              "| same action + stream | faster |\n|---|---|---|---|---|---|\n")
      for r in rows:
        f.write("| %s | %d | %.2f | %.2f | %s | %s |\n" % (
            r["game"], r["sims"], r["hip_step_ms"], r["host_step_ms"],
            r["same_action_and_stream"], r["faster"]))
    return
  rows = []
  for gs in args.games.split(","):
    r = measure(gs, args.sims, args.reps, torch)
    rows.append(r)
    print(json.dumps(r), flush=True)
  os.makedirs(args.out, exist_ok=True)
  with open(os.path.join(args.out, "step_latency.json"), "w") as f:
    json.dump(rows, f, indent=1)
  with open(os.path.join(args.out, "step_latency.md"), "w") as f:
    f.write("| game | sims | pyspiel.MCTSBot.step ms | its kernel ms | host overhead | "
            "mcts.MCTSBot.step ms | its kernel ms (numpy policy) | host overhead | "
            "oracle 1 core ms | oracle / GPU step |\n|---|---|---|---|---|---|---|---|---|---|\n")
    for r in rows:
      f.write("| %s | %d | %.3f | %.3f | %.3f ms (%.1f%%) | %.3f | %.3f | %.3f ms (%.1f%%) | "
              "%.2f | %.2f |\n" % (
                  r["game"], r["sims"], r["cpp_step_ms"], r["kernel_ms"], r["host_overhead_ms"],
                  100 * r["host_overhead_frac"], r["py_step_ms"], r["np_kernel_ms"],
                  r["py_overhead_ms"], 100 * r["py_overhead_frac"], r["oracle_1core_ms"],
                  r["gpu_over_oracle"]))


if __name__ == "__main__":
  main()
