#!/usr/bin/env python3
"""Steady-state per-launch kernel times from a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats averages every dispatch of a kernel, the first (cold)
launch included: on the headline config that first launch is ~15% slower
than the rest (HBM pages touched for the first time, code object load), so
the average sits above the bench line's ms_per_step.  This summary drops the
first `--skip` dispatches of each kernel and reports count / mean / median /
min / max of the rest beside the all-dispatch mean, so a profile can be held
to the driver-timed figure.

    python tools/kernel_steady.py run_kernel_trace.csv [--skip 1] [--out x.json]
"""
import argparse
import csv
import json
import re
import statistics
import sys


def short(name):
  name = re.sub(r"\(.*\)$", "", name)  # drop the argument list
  return name.replace("osx::", "").replace("osm::", "").replace("void ", "")


def summarise(path, skip):
  times = {}
  with open(path, newline="") as f:
    for row in csv.DictReader(f):
      if row.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
        continue
      ms = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
      times.setdefault(short(row["Kernel_Name"]), []).append(ms)
  out = {}
  for k, ts in times.items():
    rest = ts[skip:] if len(ts) > skip else ts
    out[k] = {"dispatches": len(ts), "all_mean_ms": statistics.fmean(ts),
              "first_ms": ts[0], "skipped": len(ts) - len(rest),
              "steady_count": len(rest), "steady_mean_ms": statistics.fmean(rest),
              "steady_median_ms": statistics.median(rest), "steady_min_ms": min(rest),
              "steady_max_ms": max(rest)}
  return out


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("trace")
  ap.add_argument("--skip", type=int, default=1, help="leading dispatches dropped per kernel")
  ap.add_argument("--out")
  args = ap.parse_args()
  res = summarise(args.trace, args.skip)
  doc = {"source": args.trace, "skip_first": args.skip, "kernels": res}
  text = json.dumps(doc, indent=1)
  if args.out:
    with open(args.out, "w") as f:
      f.write(text + "\n")
  for k, v in sorted(res.items(), key=lambda kv: -kv[1]["steady_mean_ms"] * kv[1]["steady_count"]):
    print("%-70s n=%4d all %.4f  first %.4f  steady mean %.4f median %.4f min %.4f ms" % (
        k[:70], v["dispatches"], v["all_mean_ms"], v["first_ms"], v["steady_mean_ms"],
        v["steady_median_ms"], v["steady_min_ms"]))
  return 0


if __name__ == "__main__":
  sys.exit(main())
