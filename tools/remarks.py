#!/usr/bin/env python3
"""Tabulates hipcc -Rpass-analysis=kernel-resource-usage remarks (one row per
kernel: VGPRs, SGPRs, spills, scratch, occupancy)."""
import re
import subprocess
import sys

FIELDS = ("VGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
          "Occupancy [waves/SIMD]")


def main(path):
  rows, cur = [], None
  for line in open(path, errors="replace"):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
      cur = {"name": m.group(1)}
      rows.append(cur)
      continue
    for f in FIELDS:
      m = re.search(re.escape(f) + r": (\d+)", line)
      if m and cur is not None:
        cur[f] = int(m.group(1))
  names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                         capture_output=True, text=True).stdout.split("\n")
  for r, n in zip(rows, names):
    n = n.replace("(anonymous namespace)::", "").replace("osm::", "")
    if "VGPRs" not in r:
      continue
    print("%-58s v%3d s%3d vsp%4d ssp%4d scr%5d occ%d" % (
        n[:58], r["VGPRs"], r.get("TotalSGPRs", 0), r.get("VGPRs Spill", 0),
        r.get("SGPRs Spill", 0), r.get("ScratchSize [bytes/lane]", 0),
        r.get("Occupancy [waves/SIMD]", 0)))


if __name__ == "__main__":
  main(sys.argv[1])
