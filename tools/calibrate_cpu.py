#!/usr/bin/env python3
"""CPU-baseline calibration: times the oracle restatement
single-threaded under SURVEY.md §6's probe conditions -- initial position,
uct_c=2, n_rollouts=1, solve=true, max_memory_mb=1000, seeds 1, 2, 3 (bot and
evaluator) -- and states its speed as a ratio of the reference figures §6
measured in this container on the shim-built reference mcts.cc (same Xeon,
g++ -O2, one thread).  Writes profiles/cpu_calibration.json, which bench.py
carries in every cpu_baseline.

    python tools/calibrate_cpu.py [--repeat 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402

# reference C++ MCTS sims/s, one core, this container.
REFERENCE = {
    "tic_tac_toe": (1000, 0.69e6),
    "connect_four": (1024, 136e3),
    "breakthrough": (2048, 17.5e3),
    "hex": (2048, 15.9e3),
    "go(board_size=9)": (1024, 7.3e3),
}


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--repeat", type=int, default=3)
  args = ap.parse_args()
  out = {"_source": "tools/calibrate_cpu.py: oracle (oracle/ref_mcts.h) single-threaded vs "
                    "SURVEY.md §6 reference mcts.cc probes, same container",
         "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": "),
         "games": {}}
  for gs, (sims, ref) in REFERENCE.items():
    og = oracle_lib.Game(gs)
    acts = np.zeros(0, np.int64)
    best = 0.0
    for _ in range(args.repeat):
      n_tot, t_tot = 0, 0.0
      for seed in (1, 2, 3):
        s = np.array([seed], np.uint32)
        secs, n = og.time_mcts_batch(acts, np.array([0, 0], np.int64), s, s,
                                     max_simulations=sims, threads=1)
        n_tot, t_tot = n_tot + n, t_tot + secs
      best = max(best, n_tot / t_tot)
    out["games"][gs] = {"sims": sims, "oracle_sims_per_s": round(best, 1),
                        "reference_sims_per_s": ref, "ratio": round(best / ref, 3)}
    print("%-20s oracle %9.0f sims/s  reference %9.0f  ratio %.3f" % (gs, best, ref, best / ref))
  path = os.path.join(ROOT, "profiles", "cpu_calibration.json")
  with open(path, "w") as f:
    json.dump(out, f, indent=1)
  print("->", os.path.relpath(path, ROOT))


if __name__ == "__main__":
  main()
