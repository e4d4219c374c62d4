// skq_map1.hip — the fused map's one-k instantiations (k_map1, launch_map1): a translation unit
// of its own (part 1 of skq_kernels.hip's helpers), built beside the other kernel parts.
#define SKQ_PART 1
#include "skq_kernels.hip"
#include "skq_map1.h"

namespace skq {

constexpr int MW = MAP_MW;
bool map1_bins_ok() { return MW == WG; }

// SKQ_MAP1_OCC=1: print each k_map1 launch shape's resident workgroups per CU once (stderr)
static void map1_report_occupancy(const void* kern, size_t lds) {
    static const bool on = [] {
        const char* e = std::getenv("SKQ_MAP1_OCC");
        return e && std::atoi(e) != 0;
    }();
    if (!on) return;
    static std::mutex mu;
    static std::vector<std::pair<const void*, size_t>> seen;
    std::lock_guard<std::mutex> g(mu);
    for (auto& x : seen)
        if (x.first == kern && x.second == lds) return;
    seen.emplace_back(kern, lds);
    int nb = -1;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, MW, lds);
    std::fprintf(stderr, "[skq] k_map1 %p: %zu B LDS, %d workgroups per CU\n", kern, lds, nb);
}

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
    // (development: SKQ_LDS_PAD bytes of unused LDS per workgroup lower the occupancy, to price it)
    static const size_t pad = std::getenv("SKQ_LDS_PAD") ? std::strtoull(std::getenv("SKQ_LDS_PAD"), nullptr, 10) : 0;
    if (lds + pad > 64 * 1024) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)(lds + pad));
    map1_report_occupancy(reinterpret_cast<const void*>(kern), lds + pad);
    hipLaunchKernelGGL(kern, grid, dim3(MW), lds + pad, st, p, cp);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace skq
