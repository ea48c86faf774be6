// go kernels of libos_mcts.so (one translation unit per game so the
// device code builds in parallel; see os_kernels.h).
#include "os_kernels.h"

OS_DEFINE_LAUNCHERS(Go, 1)
