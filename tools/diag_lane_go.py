import sys, time, numpy as np
sys.path.insert(0, "open_spiel-1_amd"); sys.path.insert(0, "tests")
from os_amd import engine as E, _lib
import oracle_lib as O
gs = "go(board_size=7,komi=4.5)"
acts, offs = E.make_roots(gs, 6, 1000, 4)
bs = np.arange(6, dtype=np.uint32) * 3 + 1
es = bs + np.uint32(1 << 20)
eng = E.Engine(gs)
for R in (1, 6):
  got = eng.mcts_batch(acts[:offs[R]], offs[:R+1], bs[:R], es[:R], layout=_lib.LAYOUT_LANE, uct_c=0.7,
                       max_simulations=1, n_rollouts=2, solve=False)
  ref = O.Game(gs).mcts_batch(acts[:offs[R]], offs[:R+1], bs[:R], es[:R], max_children=eng.max_children, uct_c=0.7,
                              max_simulations=1, n_rollouts=2, solve=False)
  print(R, got["root_w"], ref["root_w"], flush=True)
