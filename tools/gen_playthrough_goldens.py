#!/usr/bin/env python3
"""Extract game-transition golden vectors from the reference playthrough files.

Runs ONLY in the build container (reads /root/reference as data, never imports
or executes anything from it).  Writes compact JSON fixtures under
tests/golden/playthrough_<game>.json.  The reference's own integration test
(open_spiel/integration_tests/playthrough_test.py:50-77) replays these same
files; here each recorded state becomes one record:

    {"history": [...], "is_terminal": bool, "current_player": int,
     "returns": [r0, r1], "legal_actions": [...], "string_legal_actions": [...],
     "observation_string": "..."}

Usage:  python tools/gen_playthrough_goldens.py
"""
import json
import os
import re
import sys

REF = "/root/reference/open_spiel/integration_tests/playthroughs"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")

FILES = {
    "tic_tac_toe": "tic_tac_toe.txt",
    "connect_four": "connect_four.txt",
    "breakthrough": "breakthrough.txt",
    "hex(board_size=5)": "hex(board_size=5).txt",
    "go(board_size=7,komi=4.5)": "go.txt",
    # chance nodes: n-player playthroughs pin the rules
    "pig(players=3,horizon=10,winscore=10)": "pig_3p.txt",
    "pig(players=4,horizon=10,winscore=10)": "pig_4p.txt",
    "pig(players=5,horizon=100,winscore=20)": "pig_5p.txt",
}


def _unquote(s):
  s = s.strip()
  assert s[0] == '"' and s[-1] == '"', s
  return json.loads(s)  # playthrough strings use JSON-compatible escapes


def _int_list(s):
  s = s.strip()
  assert s[0] == "[" and s[-1] == "]", s
  body = s[1:-1].strip()
  return [int(x) for x in body.split(",")] if body else []


def _float_list(s):
  s = s.strip()
  body = s[1:-1].strip()
  return [float(x) for x in body.split(",")] if body else []


def _str_list(s):
  return json.loads(s.strip())


_GLYPH = {"◯": 0, "◉": 1}  # ◯ = 0.0, ◉ = 1.0 (binary tensors only)


def _tensor_rows(lines, i):
  """Glyph rows of an ObservationTensor(p): block starting at lines[i]:
  each row holds the C planes of one tensor row, separated by two spaces.
  Returns ([C][H][W] nested lists, next index)."""
  rows = []
  while i < len(lines) and lines[i] and lines[i][0] in _GLYPH:
    rows.append([[_GLYPH[ch] for ch in plane] for plane in lines[i].split("  ")])
    i += 1
  C = len(rows[0])
  return [[row[c] for row in rows] for c in range(C)], i


def parse(path):
  states = []
  cur = None
  header = {}
  with open(path) as f:
    lines = f.read().split("\n")
  i = 0
  while i < len(lines):
    line = lines[i]
    i += 1
    if line.startswith("# State "):
      cur = {}
      states.append(cur)
      continue
    mt = re.match(r"^ObservationTensor\(([01])\):$", line)
    if cur is not None and mt:
      t, i = _tensor_rows(lines, i)
      cur.setdefault("observation_tensor", [None, None])[int(mt.group(1))] = t
      continue
    m = re.match(r"^([A-Za-z]+)\(\) = (.*)$", line)
    if cur is None:
      if m:
        header[m.group(1)] = m.group(2)
      continue
    if line.startswith("IsTerminal() = "):
      cur["is_terminal"] = line.endswith("True")
    elif line.startswith("History() = "):
      cur["history"] = _int_list(line.split(" = ", 1)[1])
    elif line.startswith("CurrentPlayer() = "):
      cur["current_player"] = int(line.split(" = ", 1)[1])
    elif line.startswith("Returns() = "):
      cur["returns"] = _float_list(line.split(" = ", 1)[1])
    elif line.startswith("LegalActions() = "):
      cur["legal_actions"] = _int_list(line.split(" = ", 1)[1])
    elif line.startswith("StringLegalActions() = "):
      cur["string_legal_actions"] = _str_list(line.split(" = ", 1)[1])
    elif line.startswith("IsChanceNode() = "):
      cur["is_chance_node"] = line.endswith("True")
    elif line.startswith("ChanceOutcomes() = "):
      body = line.split(" = ", 1)[1].strip()[1:-1]
      cur["chance_outcomes"] = [[int(a), float(p)] for a, p in
                                re.findall(r"\{(\d+), ([0-9.e-]+)\}", body)]
    elif line.startswith("ObservationString(0) = "):
      cur["observation_string"] = _unquote(line.split(" = ", 1)[1])
  for s in states:
    s.setdefault("legal_actions", [])
    s.setdefault("string_legal_actions", [])
  meta = {
      "num_distinct_actions": int(header["NumDistinctActions"]),
      "max_game_length": int(header["MaxGameLength"]),
      "max_utility": float(header["MaxUtility"]),
      "min_utility": float(header["MinUtility"]),
      "game_to_string": _unquote(header["ToString"]),
      "observation_tensor_shape": _int_list(header["ObservationTensorShape"]),
  }
  return meta, states


def main():
  os.makedirs(OUT, exist_ok=True)
  for game, fname in FILES.items():
    meta, states = parse(os.path.join(REF, fname))
    short = game.split("(")[0]
    if short == "pig":
      short = os.path.splitext(fname)[0]
    rec = {"game": game, "source": "open_spiel/integration_tests/playthroughs/"
           + fname, "meta": meta, "states": states}
    out = os.path.join(OUT, "playthrough_%s.json" % short)
    with open(out, "w") as f:
      json.dump(rec, f, indent=None, separators=(",", ":"))
    print("wrote", out, len(states), "states", file=sys.stderr)


if __name__ == "__main__":
  main()
