#!/usr/bin/env python3
"""Summarises rocprofv3 --pmc passes (tools/pmc.sh output) for one kernel.

  python tools/pmc_summary.py gpurun_out/pmc <kernel> <game> [out.json]

Averages every counter over the kernel's dispatches, divides by the units per
launch (from the bench JSON line each pass printed: config.units_per_launch,
else the sims / playouts per step -- one launch per step), and records the HBM bytes
per launch as MI355X_MICROARCH.md §HBM prescribes for gfx950:
  traffic = 2 x FETCH_SIZE (reported at half the bytes of 128-B requests)
            + WRITE_SIZE, both KB -> bytes.
The result is merged into profiles/pmc_traffic.json under "<kernel>/<game>",
which bench.py reads for its roofline.traffic field.  The record carries the
hash of the kernel sources it was collected on (bench.kernel_source_hash, so
summarise right after collecting); bench.py flags the record `stale` once the
sources change.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
  src, kernel, game = sys.argv[1:4]
  out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles",
                                                           "pmc_traffic.json")
  counters = {}
  sims = None
  for d in sorted(glob.glob(os.path.join(src, "p*/"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
      continue
    agg = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
      if kernel not in r["Kernel_Name"]:
        continue
      agg[r["Counter_Name"]] += float(r["Counter_Value"])
      disp.add(r["Dispatch_Id"])
    for c, v in agg.items():
      counters[c] = v / max(len(disp), 1)
    log = d.rstrip("/") + ".log"
    if os.path.exists(log):
      for line in open(log):
        if line.startswith("{"):
          cfg = json.loads(line)["config"]
          sims = cfg.get("units_per_launch", cfg.get("sims_per_step_per_gpu",
                                                     cfg.get("playouts_per_step_per_gpu")))
  sys.path.insert(0, ROOT)
  import bench
  rec = {"kernel": kernel, "game": game, "sims_per_launch": sims,
         "counters_per_launch": counters, "source_hash": bench.kernel_source_hash()}
  if sims:
    rec["per_sim"] = {c: v / sims for c, v in counters.items()
                      if c.startswith("SQ_INSTS") or c in ("FETCH_SIZE", "WRITE_SIZE")}
  if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
    rec["hbm_bytes_per_launch"] = (2 * counters["FETCH_SIZE"] +
                                   counters["WRITE_SIZE"]) * 1024
    rec["traffic_note"] = ("2*FETCH_SIZE + WRITE_SIZE (KB->B); gfx950 FETCH_SIZE "
                           "halving per MI355X_MICROARCH.md; Infinity-Cache hits "
                           "are counted by these counters")
  if "SQ_WAVE_CYCLES" in counters:
    wc = counters["SQ_WAVE_CYCLES"]
    rec["wave_cycle_split"] = {k: counters.get(k, 0) / wc for k in
                               ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")}
  db = {}
  if os.path.exists(out):
    db = json.load(open(out))
  db["%s/%s" % (kernel, game)] = rec
  with open(out, "w") as f:
    json.dump(db, f, indent=1, sort_keys=True)
  print(json.dumps(rec, indent=1))


if __name__ == "__main__":
  main()
