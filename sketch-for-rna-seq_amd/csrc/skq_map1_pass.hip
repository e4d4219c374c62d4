// skq_map1_pass.hip — the fused map's multi-k pass instantiations (k_map1<..., PASS, FINAL>,
// launch_map1_pass): a translation unit of its own (part 2 of skq_kernels.hip's helpers).
#define SKQ_PART 2
#include "skq_kernels.hip"
#include "skq_map1.h"

namespace skq {

int launch_map1_pass(const SketchParams& p0, const ChainParams& cp, uint32_t cap, bool final_pass, void* stream) {
    if (p0.n == 0) return 0;
    if ((cp.wide != 1 && cp.wide != 3) || cap > p0.hcap || p0.kslot >= SKQ_MAX_K) return -4;
    constexpr int MW = PASS_MW;
    const dim3 grid((unsigned)((p0.n + MW - 1) / MW));
    SketchParams p = p0;
    // (the pass's k slot has chained tables: TAB 3 over wide entries, 4 over compact ones)
    const int tab = cp.chain[p0.kslot] ? (cp.wide == 3 ? 4 : 3) : cp.wide == 3 ? 2 : 0;
    const size_t lds = map1_layout(p, tab, cap, MW);
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (cap * 16 + tab * 2 + (final_pass ? 1 : 0)) {
    case 256: launch_timed((k_map1<16, 4, 0, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 257: launch_timed((k_map1<16, 4, 0, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 260: launch_timed((k_map1<16, 4, 2, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 261: launch_timed((k_map1<16, 4, 2, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 262: launch_timed((k_map1<16, 4, 3, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 263: launch_timed((k_map1<16, 4, 3, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 264: launch_timed((k_map1<16, 4, 4, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 265: launch_timed((k_map1<16, 4, 4, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 512: launch_timed((k_map1<32, 4, 0, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 513: launch_timed((k_map1<32, 4, 0, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 516: launch_timed((k_map1<32, 4, 2, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 517: launch_timed((k_map1<32, 4, 2, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 518: launch_timed((k_map1<32, 4, 3, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 519: launch_timed((k_map1<32, 4, 3, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 520: launch_timed((k_map1<32, 4, 4, true, false, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 521: launch_timed((k_map1<32, 4, 4, true, true, MW>), grid, dim3(MW), lds, st, p, cp); break;
    default: return -4;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// every k slot in one launch (k_mapk): one capacity for all (the largest the k slots need) and
// one table kind (every k slot chained, or none); -5: the k slots' table kinds differ
int launch_mapk(const SketchParams& p0, const ChainParams& cp, uint32_t cap, void* stream) {
    if (p0.n == 0) return 0;
    if ((cp.wide != 1 && cp.wide != 3) || cap > p0.hcap || p0.nk < 2 || p0.nk > (uint32_t)NK_FAST) return -4;
    for (uint32_t i = 1; i < p0.nk; ++i)
        if ((cp.chain[i] != nullptr) != (cp.chain[0] != nullptr)) return -5;
    constexpr int MW = PASS_MW;
    const dim3 grid((unsigned)((p0.n + MW - 1) / MW));
    SketchParams p = p0;
    const int tab = cp.chain[0] ? (cp.wide == 3 ? 4 : 3) : cp.wide == 3 ? 2 : 0;
    const size_t lds = map1_layout(p, tab, cap, MW);
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (cap * 8 + tab) {
    case 128: launch_timed((k_mapk<16, 4, 0, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 130: launch_timed((k_mapk<16, 4, 2, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 131: launch_timed((k_mapk<16, 4, 3, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 132: launch_timed((k_mapk<16, 4, 4, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 256: launch_timed((k_mapk<32, 4, 0, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 258: launch_timed((k_mapk<32, 4, 2, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 259: launch_timed((k_mapk<32, 4, 3, MW>), grid, dim3(MW), lds, st, p, cp); break;
    case 260: launch_timed((k_mapk<32, 4, 4, MW>), grid, dim3(MW), lds, st, p, cp); break;
    default: return -4;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace skq
