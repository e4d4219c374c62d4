// skq_map1_pass.hip — the fused map's multi-k pass instantiations (k_map1<..., PASS, FINAL>,
// launch_map1_pass), compiled as its own translation unit of skq_kernels.hip (part 2).
#define SKQ_PART 2
#include "skq_kernels.hip"
