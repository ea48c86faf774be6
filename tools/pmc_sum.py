#!/usr/bin/env python3
"""Per-dispatch means of rocprofv3 --pmc counters for kernels matching a name.

  python tools/pmc_sum.py KERNEL_SUBSTR DIR [DIR ...]
"""
import collections
import csv
import glob
import sys


def main():
  pat = sys.argv[1]
  tot = {}
  for d in sys.argv[2:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
      agg = collections.defaultdict(float)
      disp = set()
      for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
          continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
      for k, v in agg.items():
        tot[k] = v / max(len(disp), 1)
      tot["dispatches(%s)" % d.rstrip("/").split("/")[-1]] = len(disp)
  for k in sorted(tot):
    print("%-28s %.6g" % (k, tot[k]))


if __name__ == "__main__":
  main()
