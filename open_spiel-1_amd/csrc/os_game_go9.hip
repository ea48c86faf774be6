// go up to 9 x 9 on the lane kernels of libos_mcts.so: k_lsearch and
// k_rollouts over three-word bitboards (os_games.h Go9), called from go's
// launchers (os_kernels.h LaunchSearch / RollLaunch).  Its own translation
// unit so the device code builds beside go's.
#include "os_kernels.h"

namespace osx {

int LaunchGo9Search(os_engine* e, const DevArgs& a, hipStream_t stream) {
  return e->node_double ? LaunchLs<Go9, double>(e, a, stream)
                        : LaunchLs<Go9, int32_t>(e, a, stream);
}

int LaunchGo9Rollouts(os_engine* e, hipStream_t stream) { return RollLaunch<Go9>(e, stream); }

}  // namespace osx
