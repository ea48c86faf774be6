// hex 12 x 12 .. 19 x 19 kernels of libos_mcts.so: lane-layout searches
// (k_lsearch over B384 bitboards) only; see os_kernels.h.
#include "os_kernels.h"

OS_DEFINE_SEARCH_ONLY_LAUNCHERS(HexBig)
