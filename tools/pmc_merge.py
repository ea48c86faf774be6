#!/usr/bin/env python3
"""Merges gpurun_out/pmc_rec_<config>.json records (tools/pmc_configs.sh,
summarised on the GPU box) into profiles/pmc_traffic.json.

    python tools/pmc_merge.py [rec.json ...]   (default: gpurun_out/pmc_rec_*.json)
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
  recs = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_rec_*.json")))
  path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
  db = json.load(open(path)) if os.path.exists(path) else {}
  for f in recs:
    for k, v in json.load(open(f)).items():
      db[k] = v
      print("%s <- %s (source %s)" % (k, os.path.basename(f), v.get("source_hash")))
  with open(path, "w") as f:
    json.dump(db, f, indent=1, sort_keys=True)
  return 0


if __name__ == "__main__":
  sys.exit(main())
