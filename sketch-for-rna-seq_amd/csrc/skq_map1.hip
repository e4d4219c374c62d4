// skq_map1.hip — the fused map's one-k instantiations (k_map1, launch_map1): a translation unit
// of its own (part 1 of skq_kernels.hip's helpers), built beside the other kernel parts.
#define SKQ_PART 1
#include "skq_kernels.hip"
#include "skq_map1.h"

namespace skq {

constexpr int MW = MAP_MW;

int launch_map1(const SketchParams& p0, const ChainParams& cp, void* stream) {
    if (p0.n == 0) return 0;
    const dim3 grid((unsigned)((p0.n + MW - 1) / MW));
    const bool chn = cp.chain[0] != nullptr;
    SketchParams p = p0;
    if (cp.wide != 1 && cp.wide != 3) return -4;
    // (TAB: 0 wide, 2 compact, 3 chained over wide, 4 chained over compact)
    const int tab = chn ? (cp.wide == 3 ? 4 : 3) : cp.wide == 3 ? 2 : 0;
    const size_t lds = map1_layout(p, tab, p.hcap, MW);
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    using K = void (*)(SketchParams, ChainParams);
    K kern = nullptr;
    // (MB: gather rounds in flight)
    switch (p.hcap * 8 + tab) {
    case 132: kern = k_map1<16, 4, 4, false, false, MW>; break;
    case 260: kern = k_map1<32, 4, 4, false, false, MW>; break;
    case 131: kern = k_map1<16, 4, 3, false, false, MW>; break;
    case 259: kern = k_map1<32, 4, 3, false, false, MW>; break;
    case 128: kern = k_map1<16, 4, 0, false, false, MW>; break;
    case 130: kern = k_map1<16, 4, 2, false, false, MW>; break;
    case 256: kern = k_map1<32, 4, 0, false, false, MW>; break;
    case 258: kern = k_map1<32, 4, 2, false, false, MW>; break;
    default: return -4;
    }
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    launch_timed(kern, grid, dim3(MW), lds, st, p, cp);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace skq
