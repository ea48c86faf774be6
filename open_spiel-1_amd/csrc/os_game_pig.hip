// pig kernels of libos_mcts.so (one translation unit per game so the device
// code builds in parallel; see os_kernels.h).  pig has chance nodes: only the
// lane-layout search (os_chance.h) and the lane rollouts are instantiated.
#include "os_kernels.h"

OS_DEFINE_LAUNCHERS(Pig, 0)
