"""ObservationTensor export against the reference's own
playthrough fixtures (integration_tests/playthroughs/*.txt ObservationTensor
blocks, converted by tools/gen_playthrough_goldens.py): every recorded state,
both players, every game."""
import json
import os

import numpy as np
import pytest

from os_amd import pyspiel

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GAMES = ["tic_tac_toe", "connect_four", "breakthrough", "hex", "go"]


def _load(short):
  with open(os.path.join(GOLD, "playthrough_%s.json" % short)) as f:
    return json.load(f)


@pytest.mark.parametrize("short", GAMES)
def test_observation_tensor_matches_playthrough(short):
  d = _load(short)
  game = pyspiel.load_game(d["game"])
  assert game.observation_tensor_shape() == d["meta"]["observation_tensor_shape"]
  size = int(np.prod(game.observation_tensor_shape()))
  assert game.observation_tensor_size() == size
  checked = 0
  for rec in d["states"]:
    st = game.new_initial_state()
    for a in rec["history"]:
      st.apply_action(a)
    for p in (0, 1):
      want = np.array(rec["observation_tensor"][p], np.float32).reshape(-1)
      got = np.array(st.observation_tensor(p), np.float32)
      np.testing.assert_array_equal(got, want, err_msg="%s state %s player %d" %
                                    (short, rec["history"], p))
      checked += 1
  assert checked == 2 * len(d["states"])
