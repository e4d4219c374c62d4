// skq_map1.hip — the fused map's one-k instantiations (k_map1, launch_map1), compiled as its own
// translation unit of skq_kernels.hip (part 1) so the build runs the kernel parts side by side.
#define SKQ_PART 1
#include "skq_kernels.hip"
