// skq_kernels.hip — gfx950 kernels for the FracMinHash sketch + sparse-chain hot path.
//
//   k_sketch       reads (ASCII) -> per (read, k) sorted set of retained 32-bit ntHash values.
//                  Restates createSketch_FracMinhash_direct (reference src/sketch.cpp:24-39) and
//                  the read filters of process_fastq_single_pass (src/main.cpp:132-138).
//                  One workgroup = 256 reads. The workgroup's byte span is staged once into LDS
//                  with coalesced 16-B loads and converted to 2-bit codes + an invalid-base mask;
//                  each lane then rolls the 33-bit ntHash lane over its own read, 16 windows per
//                  step from two funnel-shifted code words (in-bases, out-bases).
//   k_chain        per read: probe every retained hash in the device index, count per
//                  (transcript, k), per-k max, keep transcripts with count >= fraction*max at
//                  every k, score = sum of counts, sort (score desc, tid asc). Restates
//                  sparse_chain (src/sparse_chaining.cpp:42-111). One lane per read; each probe
//                  reads one 64-B bucket mapping keys to postings-list equivalence classes;
//                  counts are kept per distinct list, then expanded per transcript, in
//                  register tables (packed 8-bit counts per k).
//   *_slow         exact fallbacks for what the fast kernels do not bound (reads > 256 bp, more
//                  than HCAP raw retained hashes, more than 8 distinct lists or 16 distinct
//                  transcripts, > 4 k slots). One workgroup per listed read, sorting in LDS; they walk device-side
//                  work lists with a fixed grid, so no host round trip is needed.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include <type_traits>
#include <utility>

#include <algorithm>

#include "skq_internal.h"

// Three translation units built side by side (make -j): part 0 (this file alone) is every kernel
// but the fused map; part 1 (skq_map1.hip) and part 2 (skq_map1_pass.hip) include this file for
// its device helpers, then k_map1 (skq_map1.h), and instantiate the one-k map and the multi-k
// passes. Templates and inline helpers are visible to all three; every other definition of this
// file sits in part 0.
#ifndef SKQ_PART
#define SKQ_PART 0
#endif


// chained entries read eight lanes to an entry and handed over through LDS (1), or one lane per
// entry (0: development A/B, profiles/r4_chain_coalesced_ab.log)
#ifndef SKQ_HASH_SDWA
#define SKQ_HASH_SDWA 1  // (0: roll-term offsets by shift and mask, development A/B)
#endif
#ifndef SKQ_LIST_NU
#define SKQ_LIST_NU 1  // (0: every entry-list pass runs MB rounds, development A/B)
#endif
#ifndef SKQ_HASH_PAIR
#define SKQ_HASH_PAIR 1  // (0: the round-4 hashing loop, development A/B)
#endif
#ifndef SKQ_CHN_COALESCED
#define SKQ_CHN_COALESCED 1
#endif

namespace skq {

// a launch of the timed kernels (the map, the sketch, probe and count): the scope's events bound
// to the dispatch (skq_internal.h LaunchEvents), the start one only to the scope's first launch
template <typename K, typename... A>
inline void launch_timed(K kern, dim3 grid, dim3 blk, size_t lds, hipStream_t st, A... args) {
    const hipEvent_t a = static_cast<hipEvent_t>(g_launch_ev.start), b = static_cast<hipEvent_t>(g_launch_ev.stop);
    g_launch_ev.start = nullptr;
    hipExtLaunchKernelGGL(kern, grid, blk, (uint32_t)lds, st, a, b, 0u, args...);
}

// ---------------------------------------------------------------------------------------------
// small helpers

// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N - 1>{})
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <typename T>
__device__ __forceinline__ void cswap(T& a, T& b) {
    T lo = a < b ? a : b;
    T hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Sorting networks of the fewest known comparators (each a min and a max, both half-rate VALU:
// the bitonic network of 16 has 80, this one 60), entries lo | hi << 8; every one checked on all
// 0-1 inputs (tests/test_sort_networks.py)
constexpr uint16_t kNet8[19] = {0 | 2 << 8, 1 | 3 << 8, 4 | 6 << 8, 5 | 7 << 8, 0 | 4 << 8, 1 | 5 << 8, 2 | 6 << 8, 3 | 7 << 8, 0 | 1 << 8, 2 | 3 << 8, 4 | 5 << 8, 6 | 7 << 8, 2 | 4 << 8, 3 | 5 << 8, 1 | 4 << 8, 3 | 6 << 8, 1 | 2 << 8, 3 | 4 << 8, 5 | 6 << 8};
constexpr uint16_t kNet12[39] = {0 | 8 << 8, 1 | 7 << 8, 2 | 6 << 8, 3 | 11 << 8, 4 | 10 << 8, 5 | 9 << 8, 0 | 1 << 8, 2 | 5 << 8, 3 | 4 << 8, 6 | 9 << 8, 7 | 8 << 8, 10 | 11 << 8, 0 | 2 << 8, 1 | 6 << 8, 5 | 10 << 8, 9 | 11 << 8, 0 | 3 << 8, 1 | 2 << 8, 4 | 6 << 8, 5 | 7 << 8, 8 | 11 << 8, 9 | 10 << 8, 1 | 4 << 8, 3 | 5 << 8, 6 | 8 << 8, 7 | 10 << 8, 1 | 3 << 8, 2 | 5 << 8, 6 | 9 << 8, 8 | 10 << 8, 2 | 3 << 8, 4 | 5 << 8, 6 | 7 << 8, 8 | 9 << 8, 4 | 6 << 8, 5 | 7 << 8, 3 | 4 << 8, 5 | 6 << 8, 7 | 8 << 8};
constexpr uint16_t kNet16[60] = {0 | 13 << 8, 1 | 12 << 8, 2 | 15 << 8, 3 | 14 << 8, 4 | 8 << 8, 5 | 6 << 8, 7 | 11 << 8, 9 | 10 << 8, 0 | 5 << 8, 1 | 7 << 8, 2 | 9 << 8, 3 | 4 << 8, 6 | 13 << 8, 8 | 14 << 8, 10 | 15 << 8, 11 | 12 << 8, 0 | 1 << 8, 2 | 3 << 8, 4 | 5 << 8, 6 | 8 << 8, 7 | 9 << 8, 10 | 11 << 8, 12 | 13 << 8, 14 | 15 << 8, 0 | 2 << 8, 1 | 3 << 8, 4 | 10 << 8, 5 | 11 << 8, 6 | 7 << 8, 8 | 9 << 8, 12 | 14 << 8, 13 | 15 << 8, 1 | 2 << 8, 3 | 12 << 8, 4 | 6 << 8, 5 | 7 << 8, 8 | 10 << 8, 9 | 11 << 8, 13 | 14 << 8, 1 | 4 << 8, 2 | 6 << 8, 5 | 8 << 8, 7 | 10 << 8, 9 | 13 << 8, 11 | 14 << 8, 2 | 4 << 8, 3 | 6 << 8, 9 | 12 << 8, 11 | 13 << 8, 3 | 5 << 8, 6 | 8 << 8, 7 | 9 << 8, 10 | 12 << 8, 3 | 4 << 8, 5 | 6 << 8, 7 | 8 << 8, 9 | 10 << 8, 11 | 12 << 8, 6 | 7 << 8, 8 | 9 << 8};

// ascending sort of a[0..M) by the network above (fully unrolled: every index is a constant)
template <int M, typename T>
__device__ __forceinline__ void net_sort(T* a) {
    static_assert(M == 8 || M == 12 || M == 16, "networks of 8, 12 and 16");
    static_for<M == 8 ? 19 : (M == 12 ? 39 : 60)>([&](auto c) {
        constexpr uint16_t e = M == 8 ? kNet8[c] : (M == 12 ? kNet12[c] : kNet16[c]);
        cswap(a[e & 255], a[e >> 8]);
    });
}

// ascending sort of a register array: the networks above at 8 and 16, else bitonic (fully
// unrolled: every index is a constant)
template <int N, typename T>
__device__ __forceinline__ void bitonic_sort(T (&a)[N]) {
    if constexpr (N == 8 || N == 16) {
        net_sort<N>(a);
    } else {
#pragma unroll
        for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
            for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    const int l = i ^ j;
                    if (l > i) {
                        if ((i & k) == 0) cswap(a[i], a[l]);
                        else cswap(a[l], a[i]);
                    }
                }
            }
        }
    }
}

// ascending sort of a[0..N) whose entries from n on are padding no smaller than any before
// (n <= N per lane): the active lanes' longest prefix picks the network (a uniform branch;
// cfg3: about 6 retained windows per read, the wave's longest mostly 9-13)
template <int N, typename T>
__device__ __forceinline__ void sort_prefix(T (&a)[N], uint32_t n) {
    if constexpr (N == 16) {
        if (!__any(n > 8)) {
            net_sort<8>(a);
            return;
        }
        if (!__any(n > 12)) {
            net_sort<12>(a);
            return;
        }
    }
    bitonic_sort<N>(a);
}

// ascending bitonic sort of a[0..n) in LDS by the whole workgroup (n a power of two)
template <typename T>
__device__ void block_sort(T* a, uint32_t n) {
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const T x = a[i], y = a[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) {
                        a[i] = y;
                        a[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ uint32_t pow2_at_least(uint32_t m) {
    uint32_t n = 1;
    while (n < m) n <<= 1;
    return n;
}

// inclusive scan of one value per thread over the workgroup; also returns the total
__device__ uint32_t block_incl_scan(uint32_t v, uint32_t* s, uint32_t& total) {
    const uint32_t t = threadIdx.x;
    s[t] = v;
    __syncthreads();
    for (uint32_t o = 1; o < blockDim.x; o <<= 1) {
        const uint32_t add = t >= o ? s[t - o] : 0u;
        __syncthreads();
        s[t] += add;
        __syncthreads();
    }
    const uint32_t r = s[t];
    total = s[blockDim.x - 1];
    __syncthreads();
    return r;
}

// serial shell sort (Ciura gaps) for the rare oversized cases
template <typename T>
__device__ void serial_sort(T* a, uint64_t m) {
    const uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
    for (int g = 0; g < 8; ++g) {
        const uint64_t gap = gaps[g];
        for (uint64_t x = gap; x < m; ++x) {
            const T v = a[x];
            uint64_t b = x;
            while (b >= gap && a[b - gap] > v) {
                a[b] = a[b - gap];
                b -= gap;
            }
            a[b] = v;
        }
    }
}

__device__ __forceinline__ void read_extent(const uint64_t* offs, uint64_t fixed_len, uint64_t r,
                                            uint64_t& start, uint64_t& len) {
    if (offs) {
        start = offs[r];
        len = offs[r + 1] - start;
    } else {
        start = r * fixed_len;
        len = fixed_len;
    }
}

__device__ __forceinline__ uint32_t list_push(uint32_t* ctrl, int counter, int errword,
                                              uint32_t* list, uint32_t cap, uint32_t value,
                                              uint32_t err) {
    uint32_t at = atomicAdd(&ctrl[counter], 1u);
    if (at < cap) list[at] = value;
    else atomicOr(&ctrl[errword], err);
    return at;
}

// ASCII -> 2-bit code ((c >> 1) & 3: A0 C1 T2 G3) for 4 bytes, plus a 4-bit "not uppercase
// ACGT" mask. The expected ASCII of each code is looked up with one v_perm_b32.
__device__ __forceinline__ void encode4(uint32_t w, uint32_t& codes8, uint32_t& bad4) {
    const uint32_t t = (w >> 1) & 0x03030303u;
    const uint32_t expect = __builtin_amdgcn_perm(0u, 0x47544341u /* 'G''T''C''A' */, t);
    const uint32_t x = expect ^ w;
    // per byte: high bit set iff the byte of x is nonzero
    const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    bad4 = ((nz >> 7) | (nz >> 14) | (nz >> 21) | (nz >> 28)) & 0xFu;
    codes8 = (t | (t >> 6) | (t >> 12) | (t >> 18)) & 0xFFu;
}

// 4-bit mask of bytes ntHash treats as invalid: anything but A C G T U, either case
__device__ __forceinline__ uint32_t ntbad4(uint32_t w) {
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t c = ((w >> (8 * b)) & 0xFFu) | 0x20u;
        const bool ok = c == 'a' || c == 'c' || c == 'g' || c == 't' || c == 'u';
        m |= ok ? 0u : (1u << b);
    }
    return m;
}

__device__ __forceinline__ bool ntvalid(uint8_t b) {
    const uint32_t c = b | 0x20u;
    return c == 'a' || c == 'c' || c == 'g' || c == 't' || c == 'u';
}

// one roll step of the 33-bit lane kept as (lo: bits 0..31, hi31: bit 32 held in bit 31):
// rot33 is one funnel shift, then the XOR with the roll term e
__device__ __forceinline__ void roll33b(uint32_t& lo, uint32_t& hi31, uint2 e) {
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi31, 31);
    hi31 = (lo & 0x80000000u) ^ e.y;
    lo = nlo ^ e.x;
}

// one roll step of the 33-bit lane kept as (lo: bits 0..31, hi: bit 32)
__device__ __forceinline__ void roll33(uint32_t& lo, uint32_t& hi, uint64_t e) {
    const uint32_t nlo = (lo << 1) | hi;
    hi = (lo >> 31) ^ (uint32_t)(e >> 32);
    lo = nlo ^ (uint32_t)e;
}

// ---------------------------------------------------------------------------------------------
// K1: sketch

// LDS layout: [tables: nk * 16 u64 (seed(in) ^ rot^k(seed(out))), 4 u64 seeds]
//             per wave: [codes: wave_chunks + 1 u32, padded to 16 B]
//             per wave: [bad: wave_chunks u16, padded to 16 B]
//             [raw retained: (HCAP + 1) x WG u32]
// Each wave stages the bytes of its own 64 reads and synchronises only with itself, so a wave
// waiting for its loads never holds up the other waves of the workgroup.
__host__ __device__ inline size_t sketch_tab_bytes(uint32_t nk) { return ((size_t)nk * 16 + 4) * 8; }
// (codes: wc chunks + the zero word at nch + a sink word; bad: ntHash mode one u16 mask per
// chunk + a sink, quant mode one "any bad byte" bit per chunk)
__host__ __device__ inline size_t sketch_codes_bytes(uint32_t wc) { return (((size_t)wc + 2) * 4 + 15) & ~(size_t)15; }
__host__ __device__ inline size_t sketch_bad_bytes(uint32_t wc, bool nthash) {
    return nthash ? ((((size_t)wc + 1) * 2 + 15) & ~(size_t)15) : (((size_t)wc + 127) / 128) * 16;
}

#if SKQ_PART == 0
size_t sketch_lds_bytes(uint32_t nk, uint32_t wave_chunks, uint32_t hcap, bool nthash) {
    size_t b = sketch_tab_bytes(nk);
    b += (WG / 64) * (sketch_codes_bytes(wave_chunks) + sketch_bad_bytes(wave_chunks, nthash));
    b += ((size_t)hcap + 1) * WG * 4;  // + one spare slot per lane for windows not retained
    return b;
}
#endif  // SKQ_PART == 0

template <int HCAP, bool NTH>
__global__ __launch_bounds__(WG) void k_sketch(SketchParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const uint32_t lane = tid & 63, wv = tid >> 6;
    const uint32_t wc = p.tile_chunks;  // chunks per wave
    // roll terms as {bits 0..31, bit 32 moved to bit 31}
    uint2* s_tab = reinterpret_cast<uint2*>(smem);
    const uint2* s_seed = s_tab + p.nk * 16;
    unsigned char* s_wave = smem + sketch_tab_bytes(p.nk) + wv * (sketch_codes_bytes(wc) + sketch_bad_bytes(wc, NTH));
    uint32_t* s_codes = reinterpret_cast<uint32_t*>(s_wave);
    uint16_t* s_bad = reinterpret_cast<uint16_t*>(s_wave + sketch_codes_bytes(wc));   // ntHash mode
    uint64_t* s_badw = reinterpret_cast<uint64_t*>(s_wave + sketch_codes_bytes(wc));  // quant mode
    uint32_t* s_raw = reinterpret_cast<uint32_t*>(smem + sketch_tab_bytes(p.nk) +
                                                  (WG / 64) * (sketch_codes_bytes(wc) + sketch_bad_bytes(wc, NTH)));
    for (uint32_t e = tid; e < p.nk * 16 + 4; e += WG) {
        const uint64_t v = p.rolltab[e];
        s_tab[e] = make_uint2((uint32_t)v, (uint32_t)(v >> 32) << 31);
    }
    __syncthreads();  // the only workgroup barrier: before any read bytes are loaded

    const uint64_t r0 = (uint64_t)blockIdx.x * WG + wv * 64;  // this wave's first read
    if (r0 >= p.n) return;
    const uint32_t nr = (uint32_t)min((uint64_t)64, p.n - r0);

    // the wave's byte span, in 16-byte chunks of the aligned-down base pointer (a 16-B aligned
    // chunk holding at least one byte of the buffer never crosses a page)
    const uintptr_t base = reinterpret_cast<uintptr_t>(p.reads);
    const uintptr_t abase = base & ~(uintptr_t)15;
    const uint64_t delta = base - abase;
    uint64_t s0, l0, sl, ll;
    read_extent(p.offs, p.fixed_len, r0, s0, l0);
    read_extent(p.offs, p.fixed_len, r0 + nr - 1, sl, ll);
    const uint64_t c0 = (s0 + delta) >> 4;
    const uint64_t c1 = (sl + ll + delta + 15) >> 4;
    const uint32_t nch = (uint32_t)min((uint64_t)wc, c1 - c0);

    // staging: SU loads per lane in flight before any is used (a load inside a guarded loop body
    // would be waited for before the next one issues); indices past the span are clamped to
    // its last chunk, which is valid memory
    const uint4* src = reinterpret_cast<const uint4*>(p.reads - delta) + c0;
    constexpr uint32_t SU = 10;
    for (uint32_t cb = lane; cb < nch; cb += SU * 64) {
        uint4 vv[SU];
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) vv[u] = src[min(cb + u * 64, nch - 1)];
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) {
        const uint32_t c = cb + u * 64;
        const uint4 v = vv[u];
        // unconditional stores (chunks past the span go to the sink slot): a guarded store
        // would let the compiler sink the load into the guard and wait for it there
        const uint32_t cs = c < nch ? c : wc + 1;
        if (NTH) {
            uint32_t a, b, cc, d, ba, bb, bc, bd;
            encode4(v.x, a, ba);
            encode4(v.y, b, bb);
            encode4(v.z, cc, bc);
            encode4(v.w, d, bd);
            ba = ntbad4(v.x);
            bb = ntbad4(v.y);
            bc = ntbad4(v.z);
            bd = ntbad4(v.w);
            s_codes[cs] = a | (b << 8) | (cc << 16) | (d << 24);
            s_bad[c < nch ? c : wc] = (uint16_t)(ba | (bb << 4) | (bc << 8) | (bd << 12));
        } else {
            // quant mode: 2-bit codes ((byte >> 1) & 3) packed by one dot product per word,
            // and one "any byte that is not uppercase A/C/G/T" bit per chunk (XOR with the
            // letter each code stands for), gathered per 64 chunks by a wave ballot
            const uint32_t ta = (v.x >> 1) & 0x03030303u, tb = (v.y >> 1) & 0x03030303u;
            const uint32_t tc = (v.z >> 1) & 0x03030303u, td = (v.w >> 1) & 0x03030303u;
            constexpr uint32_t W4 = 0x40100401u;  // byte weights 1, 4, 16, 64
            const uint32_t code = __builtin_amdgcn_udot4(ta, W4, 0u, false) |
                                  (__builtin_amdgcn_udot4(tb, W4, 0u, false) << 8) |
                                  (__builtin_amdgcn_udot4(tc, W4, 0u, false) << 16) |
                                  (__builtin_amdgcn_udot4(td, W4, 0u, false) << 24);
            constexpr uint32_t GTCA = 0x47544341u;  // 'A' 'C' 'T' 'G' by code
            const uint32_t x = (__builtin_amdgcn_perm(0u, GTCA, ta) ^ v.x) | (__builtin_amdgcn_perm(0u, GTCA, tb) ^ v.y) |
                               (__builtin_amdgcn_perm(0u, GTCA, tc) ^ v.z) | (__builtin_amdgcn_perm(0u, GTCA, td) ^ v.w);
            s_codes[cs] = code;
            const uint64_t wbits = __ballot(x != 0);  // lanes hold one 64-aligned group of chunks
            if (lane == 0 && c < nch) s_badw[c >> 6] = wbits;
        }
        }
    }
    if (lane == 0) s_codes[nch] = 0;
    // wave-level hand-off: LDS operations of one wave complete in order; the fences keep the
    // compiler from moving the reads below above the stores
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    if (lane >= nr) return;
    const uint64_t r = r0 + lane;
    uint64_t start, len;
    read_extent(p.offs, p.fixed_len, r, start, len);
    const uint64_t q0 = start + delta - c0 * 16;  // tile position of this read's first base

    bool slow = len > (uint64_t)LFAST || q0 + len > (uint64_t)nch * 16;
    uint8_t st = SKQ_READ_OK;
    if (!slow && !NTH) {
        // is_valid_sequence (src/data_io.cpp:17-34): every byte uppercase A/C/G/T. A read whose
        // chunks are all clean is valid; one touching a flagged chunk (the bad byte may belong
        // to a neighbour) checks its own bytes. (ntHash mode: invalid bases only skip windows.)
        bool bad = false;
        if (len) {
            const uint32_t ca = (uint32_t)(q0 >> 4), cz = (uint32_t)((q0 + len - 1) >> 4);
            for (uint32_t wd = ca >> 6; wd <= (cz >> 6); ++wd) {
                uint64_t m = s_badw[wd];
                const uint32_t lo = wd == (ca >> 6) ? (ca & 63) : 0u, hi = wd == (cz >> 6) ? (cz & 63) : 63u;
                m &= (hi == 63 ? ~0ull : ((2ull << hi) - 1ull)) & ~((1ull << lo) - 1ull);
                bad |= m != 0;
            }
            if (bad) {
                bad = false;
                const uint8_t* rb = p.reads + start;
                for (uint64_t q = 0; q < len; ++q) {
                    const uint8_t ch = rb[q];
                    bad |= !(ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T');
                }
            }
        }
        if (bad) st = SKQ_READ_INVALID;
        else if (len < p.maxk) st = SKQ_READ_SHORT;  // src/main.cpp:136-138
    }

    if (!slow && st == SKQ_READ_OK) {
        const uint32_t T = p.threshold;
        const uint32_t L = (uint32_t)len;
        // 16 codes starting at tile base q, funnel-shifted out of two code words
        auto codes16 = [&](uint32_t q) -> uint32_t {
            const uint32_t d = q >> 4;
            return __builtin_amdgcn_alignbit(s_codes[d + 1], s_codes[d], (q & 15) * 2);
        };
        // ntHash mode: invalid-base bits of 16 bases from tile position q
        auto bad16 = [&](uint32_t q) -> uint32_t {
            const uint32_t d = q >> 4;
            const uint32_t hi = d + 1 < nch ? (uint32_t)s_bad[d + 1] : 0xFFFFu;
            return ((hi << 16 | (uint32_t)s_bad[d]) >> (q & 15)) & 0xFFFFu;
        };
        for (uint32_t i = 0; i < p.nk && !slow; ++i) {
            const uint32_t k = p.ks[i];
            const uint2* tab = s_tab + i * 16;
            if (NTH && L < k) {  // createSketch on a sequence shorter than k: nothing to hash
                p.hash_cnt[(uint64_t)i * p.n + r] = 0;
                continue;
            }
            // first window (NtHash::init): h = XOR_j rot^(k-1-j) seed(s_j)
            uint32_t hlo = 0, hhi = 0;
            uint32_t nextok = 0;  // ntHash mode: first window start past the last invalid base
            for (uint32_t b = 0; b < k; b += 16) {
                const uint32_t w = codes16((uint32_t)q0 + b);
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (b + j < k) roll33b(hlo, hhi, s_seed[(w >> (2 * j)) & 3u]);
                if (NTH) {
                    uint32_t bb = bad16((uint32_t)q0 + b);
                    if (k - b < 16) bb &= (1u << (k - b)) - 1u;
                    if (bb) nextok = b + 32 - __builtin_clz(bb);  // (highest bad) + 1
                }
            }
            uint32_t* raw = s_raw + tid;
            uint32_t nraw = 0;
            {   // src/sketch.cpp:33-35
                const bool rec = hlo <= T && (!NTH || nextok == 0);
                raw[0] = hlo;
                nraw = rec ? 1u : 0u;
            }
            // windows 1..nw-1, 16 per block: in-base at w + k - 1, out-base at w - 1. The block's
            // 16 roll terms depend only on the bases, so they are read from LDS before the serial
            // roll; every window's value is stored at slot min(nraw, HCAP) (HCAP is a spare
            // slot), so the block has no branches. Windows past nw roll garbage that is never
            // recorded.
            const uint32_t nw = L - k + 1;
            const uint32_t qin = (uint32_t)q0 + k, qout = (uint32_t)q0;
            for (uint32_t w0 = 1; w0 < nw; w0 += 16) {
                const uint32_t win = codes16(qin + w0 - 1);
                const uint32_t wout = codes16(qout + w0 - 1);
                const uint32_t bin = NTH ? bad16(qin + w0 - 1) : 0u;
                const uint32_t jn = nw - w0;  // windows left (this block takes min(jn, 16))
                uint2 e[16];
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    e[j] = tab[((win >> (2 * j)) & 3u) * 4 + ((wout >> (2 * j)) & 3u)];
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    // an invalid base (ntHash mode) rolls in and out with the same term, so it
                    // cancels once it has left the window; windows holding it are skipped
                    roll33b(hlo, hhi, e[j]);
                    if (NTH) nextok = ((bin >> j) & 1u) ? w0 + j + k : nextok;
                    const bool rec = hlo <= T && (uint32_t)j < jn && (!NTH || w0 + j >= nextok);
                    // written at slot nraw either way: only a retained value advances nraw, an
                    // unretained one is overwritten later or lies past nraw
                    raw[min(nraw, (uint32_t)HCAP) * WG] = hlo;
                    nraw += rec ? 1u : 0u;
                }
            }
            if (nraw > HCAP) {
                slow = true;
                break;
            }
            // set semantics (std::unordered_set): sort, drop repeats
            uint32_t v[HCAP];
#pragma unroll
            for (int j = 0; j < HCAP; ++j) v[j] = (uint32_t)j < nraw ? s_raw[j * WG + tid] : 0xFFFFFFFFu;
            sort_prefix<HCAP>(v, nraw);
            // SoA layout: value j of (read r, k slot i) at hashes[(i*hcap + j)*n + r], so the
            // wave's stores of one j are contiguous
            uint32_t* out = p.hashes + (uint64_t)i * p.hcap * p.n + r;
            uint32_t m = 0;
            uint64_t keepm = 0;  // bit j: v[j] is the first of its run (HCAP <= 64)
            static_assert(HCAP <= 64, "keep mask is 64 bits");
#pragma unroll
            for (int j = 0; j < HCAP; ++j) {
                const bool keep = (uint32_t)j < nraw && (j == 0 || v[j] != v[j - 1]);
                if (keep) {
                    out[(uint64_t)(m++) * p.n] = v[j];
                    keepm |= 1ull << j;
                }
            }
            p.hash_cnt[(uint64_t)i * p.n + r] = m;
            if (p.fuse == 2 && p.rank[i]) {
                // fused probe, rank table: block h>>5 holds the bitmap of its 32 keys and the
                // first two keys' list offsets; the rare 3rd+ key reads the overflow array
                const uint4* rk = reinterpret_cast<const uint4*>(p.rank[i]);
                const uint32_t* ro = p.rovf[i];
                const uint64_t nb = p.dir_len[i];
                uint32_t* lout = p.lofs + (uint64_t)i * p.hcap * p.n + r;
                uint32_t mm = 0;
#pragma unroll
                for (int j0 = 0; j0 < HCAP; j0 += 8) {
                    if (!__any((keepm >> j0) & 0xFFull)) break;
                    uint4 bk[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const bool want = ((keepm >> (j0 + u)) & 1ull) && (v[j0 + u] >> 5) < nb;
                        const uint4 x = rk[want ? v[j0 + u] >> 5 : 0u];  // unconditional: all in flight
                        bk[u] = want ? x : make_uint4(0, 0, 0, 0);
                    }
                    uint32_t lo[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t bit = v[j0 + u] & 31u;
                        const uint32_t pos = __builtin_popcount(bk[u].x & ((1u << bit) - 1u));
                        lo[u] = !((bk[u].x >> bit) & 1u) ? ~0u : pos == 0 ? bk[u].z : pos == 1 ? bk[u].w : ro[bk[u].y + pos - 2];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if ((keepm >> (j0 + u)) & 1ull) lout[(uint64_t)(mm++) * p.n] = lo[u];
                }
            } else if (p.fuse && p.dir[i]) {
                // fused probe: every kept hash's list offset, all loads in flight before the
                // stores (a direct table is one 4-B gather per hash, no compare)
                const uint32_t* dir = p.dir[i];
                const uint64_t dl = p.dir_len[i];
                uint32_t lo[HCAP];
#pragma unroll
                for (int j = 0; j < HCAP; ++j) {
                    // every gather issues (index 0 when there is nothing to probe) so all are in
                    // flight together; a guarded load would be waited for one at a time
                    const bool want = ((keepm >> j) & 1ull) && v[j] < dl;
                    const uint32_t x = dir[want ? v[j] : 0u];
                    lo[j] = want ? x : ~0u;
                }
                uint32_t* lout = p.lofs + (uint64_t)i * p.hcap * p.n + r;
                uint32_t mm = 0;
#pragma unroll
                for (int j = 0; j < HCAP; ++j)
                    if ((keepm >> j) & 1ull) lout[(uint64_t)(mm++) * p.n] = lo[j];
            }
        }
    }
    if (slow) {
        st = ST_SLOW1;
        list_push(p.ctrl, C_OVF1, C_ERR1, p.ovf1, p.ovf_cap, (uint32_t)r, E_OVF1_FULL);
    } else if (st != SKQ_READ_OK) {
        for (uint32_t i = 0; i < p.nk; ++i) p.hash_cnt[(uint64_t)i * p.n + r] = 0;
    }
    p.status[r] = st;
    // reads sketched by the slow path, or with more k slots than k_count handles, chain slowly
    if (p.fuse) p.pflag[r] = (slow || p.nk > (uint32_t)NK_FAST) ? 1 : 0;
}

// packed layout: the hashes entry `at` (k slot i, read r: i * n + r) occupies in its wave's region
// — its count, or for a hash_ext run the share its header keeps (a read a pass sketched, that a
// slow path re-sketched later, keeps its place in the region)
__device__ __forceinline__ uint32_t packed_share(const uint32_t* hash_cnt, const uint32_t* hash_ext, uint64_t at) {
    const uint32_t c = hash_cnt[at];
    return (c & HASH_EXT) ? run_share(c) : c;
}

// Slow sketch path: one workgroup per listed read. Windows are split into one contiguous
// segment per thread (each thread rebuilds its segment's first hash, then rolls); retained
// hashes land in LDS (and in a bump-allocated global region beyond SLOW_CAP), then are sorted
// and de-duplicated by the workgroup.
constexpr uint32_t SLOW_CAP = 4096;

#if SKQ_PART == 0
// the workgroup's LDS for one read of k_sketch_slow (also k_general_slow's)
struct SketchSlowLds {
    uint32_t buf[SLOW_CAP];
    uint32_t scan[WG];
    uint32_t cnt, bad;
    unsigned long long at;
};

// one listed read, by the whole workgroup (uniform r)
__device__ __forceinline__ void sketch_slow_read(const SketchParams& p, uint64_t r, SketchSlowLds& L) {
    uint32_t* s_buf = L.buf;
    uint32_t* s_scan = L.scan;
    uint32_t& s_cnt = L.cnt;
    uint32_t& s_bad = L.bad;
    unsigned long long& s_at = L.at;
    const uint32_t t = threadIdx.x;
    unsigned long long* bump = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_H);
    const uint64_t* seed = p.rolltab + p.nk * 16;
    {
        uint64_t start, len;
        read_extent(p.offs, p.fixed_len, r, start, len);
        const uint8_t* s = p.reads + start;
        if (t == 0) s_bad = 0;
        __syncthreads();
        bool bad = false;
        for (uint64_t q = t; q < len && !p.nthash; q += WG) {
            const uint8_t c = s[q];
            bad |= !(c == 'A' || c == 'C' || c == 'G' || c == 'T');
        }
        if (bad) s_bad = 1;
        __syncthreads();
        const uint8_t st = p.nthash ? SKQ_READ_OK
                                    : s_bad ? SKQ_READ_INVALID : (len < p.maxk ? SKQ_READ_SHORT : SKQ_READ_OK);
        // (packed layout: each k slot's count word is replaced when its run is written, the old
        // one still giving the read's share of the wave's region)
        if (!p.hpack)
            for (uint32_t i = t; i < p.nk; i += WG) p.hash_cnt[(uint64_t)i * p.n + r] = 0;
        if (st == SKQ_READ_OK) {
            for (uint32_t i = 0; i < p.nk; ++i) {
                const uint32_t k = p.ks[i];
                if (len < k) continue;  // (ntHash mode only: quant reads are >= every k)
                const uint64_t nw = len - k + 1;
                __syncthreads();
                if (t == 0) {
                    s_cnt = 0;
                    s_at = ~0ull;
                    if (nw > SLOW_CAP) {
                        // (packed layout: room for the run's [count, share] header too, whatever
                        // share of the windows is retained)
                        const uint32_t need = run_words((uint32_t)nw + (p.hpack ? 2u : 0u));
                        const unsigned long long at = atomicAdd(bump, (unsigned long long)need);
                        if (at + need <= p.hash_ext_cap && at + need <= RUN_MAX) s_at = at;
                        else atomicOr(&p.ctrl[C_ERR1], (uint32_t)E_HASH_EXT);
                    }
                }
                __syncthreads();
                if (nw > SLOW_CAP && s_at == ~0ull) continue;  // uniform; error recorded
                uint32_t* ext = nw > SLOW_CAP ? p.hash_ext + s_at : nullptr;
                uint32_t* buf = ext ? ext : s_buf;
                const uint64_t* tab = p.rolltab + i * 16;
                const uint64_t seg = (nw + WG - 1) / WG;
                const uint64_t wa = t * seg, wb = min(nw, wa + seg);
                if (wa < wb) {
                    uint32_t hlo = 0, hhi = 0;
                    uint64_t nextok = wa;  // ntHash mode: windows before it hold an invalid base
                    for (uint64_t q = 0; q < k; ++q) {
                        roll33(hlo, hhi, seed[(s[wa + q] >> 1) & 3u]);
                        if (p.nthash && !ntvalid(s[wa + q])) nextok = wa + q + 1;
                    }
                    for (uint64_t w = wa; w < wb; ++w) {
                        if (w > wa) {
                            roll33(hlo, hhi, tab[((s[w + k - 1] >> 1) & 3u) * 4 + ((s[w - 1] >> 1) & 3u)]);
                            if (p.nthash && !ntvalid(s[w + k - 1])) nextok = w + k;
                        }
                        if (hlo <= p.threshold && w >= nextok) buf[atomicAdd(&s_cnt, 1u)] = hlo;
                    }
                }
                __syncthreads();
                const uint32_t m = s_cnt;
                uint32_t* slot = p.hashes + (uint64_t)i * p.hcap * p.n + r;  // stride p.n
                if (!ext) {
                    const uint32_t n2 = pow2_at_least(m);
                    for (uint32_t x = m + t; x < n2; x += WG) s_buf[x] = 0xFFFFFFFFu;
                    __syncthreads();
                    block_sort(s_buf, n2);
                    // keep the first of every run; write the unique values to their destination
                    const uint32_t per = (m + WG - 1) / WG;
                    const uint32_t a = min(m, t * per), b = min(m, a + per);
                    uint32_t mine = 0;
                    for (uint32_t x = a; x < b; ++x) mine += (x == 0 || s_buf[x] != s_buf[x - 1]);
                    uint32_t u = 0;
                    const uint32_t incl = block_incl_scan(mine, s_scan, u);
                    uint32_t* dst = slot;
                    uint64_t dstride = p.n;
                    uint32_t s_share = 0;  // (thread 0: the read's region share, kept in its run mark)
                    if (u > p.hcap || p.hpack) {  // (packed layout: always a run, [count, share, hashes...])
                        const uint32_t need = run_words(u + (p.hpack ? 2u : 0u));
                        if (t == 0) {
                            s_at = ~0ull;
                            const unsigned long long at = atomicAdd(bump, (unsigned long long)need);
                            if (at + need <= p.hash_ext_cap && at + need <= RUN_MAX) s_at = at;
                            else atomicOr(&p.ctrl[C_ERR1], (uint32_t)E_HASH_EXT);
                        }
                        __syncthreads();
                        if (s_at == ~0ull) continue;  // uniform
                        dst = p.hash_ext + s_at + (p.hpack ? 2u : 0u);
                        dstride = 1;
                        if (t == 0) {
                            if (p.hpack) {
                                s_share = packed_share(p.hash_cnt, p.hash_ext, (uint64_t)i * p.n + r);
                                p.hash_ext[s_at + 1] = s_share;
                                p.hash_ext[s_at] = u;
                            } else {
                                slot[0] = (uint32_t)s_at;
                            }
                        }
                    }
                    uint32_t o = incl - mine;
                    for (uint32_t x = a; x < b; ++x)
                        if (x == 0 || s_buf[x] != s_buf[x - 1]) dst[(uint64_t)(o++) * dstride] = s_buf[x];
                    if (t == 0) p.hash_cnt[(uint64_t)i * p.n + r] = p.hpack ? run_mark(s_at, s_share) : u;
                } else if (t == 0) {  // more windows than LDS holds: serial, in place
                    serial_sort(ext, m);
                    uint32_t u = 0;
                    for (uint32_t x = 0; x < m; ++x)
                        if (x == 0 || ext[x] != ext[u - 1]) ext[u++] = ext[x];
                    if (p.hpack) {  // the run behind its header (allocated nw + 2 words)
                        const uint32_t sh = packed_share(p.hash_cnt, p.hash_ext, (uint64_t)i * p.n + r);
                        for (uint32_t x = u; x > 0; --x) ext[x + 1] = ext[x - 1];
                        ext[1] = sh;
                        ext[0] = u;
                        p.hash_cnt[(uint64_t)i * p.n + r] = run_mark(s_at, sh);
                    } else {
                        if (u <= p.hcap) {
                            for (uint32_t x = 0; x < u; ++x) slot[(uint64_t)x * p.n] = ext[x];
                        } else {
                            slot[0] = (uint32_t)s_at;
                        }
                        p.hash_cnt[(uint64_t)i * p.n + r] = u;
                    }
                }
            }
        }
        if (t == 0) p.status[r] = st;
        __syncthreads();
    }
}

__global__ __launch_bounds__(WG) void k_sketch_slow(SketchParams p) {
    __shared__ SketchSlowLds L;
    const uint32_t cnt = min(p.ctrl[p.ovf_word], p.ovf_cap);
    for (uint32_t j = blockIdx.x; j < cnt; j += gridDim.x) sketch_slow_read(p, p.ovf1[j], L);
}
#endif  // SKQ_PART == 0

// ---------------------------------------------------------------------------------------------
// K2: chain

// the read's hash list at k slot i: (pointer, stride)
__device__ __forceinline__ uint32_t hash_count(const ChainParams& p, uint64_t r, uint32_t i) {
    // one load from a selected index (a load in each arm of the branch would be waited for at
    // the join, before the loads that follow could issue)
    const uint64_t at = p.hash_offs ? r * p.nk + i : (uint64_t)i * p.n + r;
    const uint32_t c = p.hash_cnt[at];
    if (p.hpack && (c & HASH_EXT)) return p.hash_ext[run_at(c)];  // (packed: a run in hash_ext)
    return c;
}

// COOP: every lane of the wave calls it for the same read (the packed layout's offset is then one
// load per lane and a wave sum instead of up to 63 loads in a row)
template <bool COOP = false>
__device__ __forceinline__ const uint32_t* hash_list(const ChainParams& p, uint64_t r, uint32_t i,
                                                     uint32_t cnt, uint64_t& stride) {
    stride = 1;
    if (p.hash_offs) return p.hashes + p.hash_offs[r * p.nk + i];
    if (p.hpack) {  // after the sets of the wave's earlier reads in k slot i's region, or a hash_ext run
        const uint64_t ci = (uint64_t)i * p.n;
        const uint32_t c = p.hash_cnt[ci + r];
        if (c & HASH_EXT) return p.hash_ext + run_at(c) + 2;
        const uint64_t r0 = r & ~63ull;
        uint32_t off = 0;
        if constexpr (COOP) {
            // (k_slow_wave: other workgroups may be turning these reads' count words into run
            // marks meanwhile; either word gives the same share, the mark carrying it itself)
            const uint64_t q = r0 + (threadIdx.x & 63u);
            off = q < r ? packed_share(p.hash_cnt, p.hash_ext, ci + q) : 0u;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) off += (uint32_t)__shfl_xor(off, d, 64);
        } else {
            for (uint64_t q = r0; q < r; ++q) off += packed_share(p.hash_cnt, p.hash_ext, ci + q);
        }
        return p.hashes + ci * p.hcap + r0 * p.hcap + off;
    }
    const uint32_t* slot = p.hashes + (uint64_t)i * p.hcap * p.n + r;
    if (cnt <= p.hcap) {
        stride = p.n;
        return slot;
    }
    return p.hash_ext + slot[0];
}

// scalar probe (slow path): postings of `key` as (pointer, count)
__device__ bool probe_list(const ChainParams& p, const DevTable& t, uint32_t key, const uint32_t*& ptr,
                           uint32_t& n) {
    uint32_t b = home_bucket(key, t.nbuckets);
    for (uint32_t q = 0; q < t.max_probe; ++q) {
        const uint32_t* B = p.buckets + (t.bucket_base + b) * BUCKET_WORDS;
        const uint32_t hdr = B[0];
        const uint32_t m = hdr & 7u;
        for (uint32_t j = 0; j < m; ++j) {
            if (B[1 + j] == key) {
                const uint32_t* L = p.lists + B[BUCKET_LIST0 + j];
                n = L[0];
                ptr = L + 1;
                return true;
            }
        }
        if (!((hdr >> 3) & 1u)) return false;
        b = b + 1 == t.nbuckets ? 0 : b + 1;
    }
    return false;
}

// Count table in registers: N (id, packed per-k counts) entries. The first 8 entries are
// always compared; entries 8.. only when some lane of the wave uses them (wave-uniform test),
// so the common read (a handful of distinct ids) pays no ballots on the compare path.
template <int N>
struct CountTable {
    uint32_t ids[N], cnts[N];
    uint32_t nd;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int d = 0; d < N; ++d) {
            ids[d] = 0xFFFFFFFFu;
            cnts[d] = 0;
        }
        nd = 0;
    }
    // cnts[id] += inc (packed bytes); false when an (N+1)th distinct id shows up
    __device__ __forceinline__ bool add(uint32_t x, uint32_t inc) {
        constexpr int N0 = N < 8 ? N : 8;
        bool found = false;
#pragma unroll
        for (int d = 0; d < N0; ++d) {
            const bool hit = ids[d] == x;
            cnts[d] += hit ? inc : 0u;
            found |= hit;
        }
        if (N > 8 && __any(nd > 8u)) {
#pragma unroll
            for (int d = N0; d < N; ++d) {
                const bool hit = ids[d] == x;
                cnts[d] += hit ? inc : 0u;
                found |= hit;
            }
        }
        if (!found && nd == (uint32_t)N) return false;
#pragma unroll
        for (int d = 0; d < N0; ++d) {
            if (!found && (uint32_t)d == nd) {
                ids[d] = x;
                cnts[d] = inc;
            }
        }
        if (N > 8 && __any(!found && nd >= 8u)) {
#pragma unroll
            for (int d = N0; d < N; ++d) {
                if (!found && (uint32_t)d == nd) {
                    ids[d] = x;
                    cnts[d] = inc;
                }
            }
        }
        nd += found ? 0u : 1u;
        return true;
    }
};

constexpr int DLISTS = 8;  // distinct postings lists per read on the fast path

// Probe `key` (one 64-B bucket, 4 x 16-B loads of the same line; further buckets only while
// the bucket is marked "continue"): returns the key's list offset, or ~0u on a miss.
__device__ __forceinline__ uint32_t probe_ec(const uint32_t* tb, const DevTable& t, uint32_t key) {
    uint32_t b = home_bucket(key, t.nbuckets);
    for (uint32_t q = 0; q < t.max_probe; ++q) {
        const uint4* B = reinterpret_cast<const uint4*>(tb + (uint64_t)b * BUCKET_WORDS);
        const uint4 w0 = B[0], w1 = B[1], w2 = B[2], w3 = B[3];
        const uint32_t m = w0.x & 7u;
        const uint32_t keys[7] = {w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const uint32_t los[7] = {w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z};
        uint32_t lo = ~0u;
#pragma unroll
        for (int j = 0; j < 7; ++j)
            if ((uint32_t)j < m && keys[j] == key) lo = los[j];
        if (lo != ~0u || !((w0.x >> 3) & 1u)) return lo;
        b = b + 1 == t.nbuckets ? 0 : b + 1;
    }
    return ~0u;
}

// value `i` (lane-varying, < 8) of an 8-entry register array, via bit-mask selects (a ?: tree
// would become an address select and push the array to scratch)
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t one, uint32_t zero) {
    return (one & m) | (zero & ~m);
}
__device__ __forceinline__ uint32_t pick8(const uint32_t (&w)[8], uint32_t i) {
    const uint32_t m0 = 0u - (i & 1u), m1 = 0u - ((i >> 1) & 1u), m2 = 0u - ((i >> 2) & 1u);
    uint32_t a[4], b[2];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = bsel(m0, w[2 * q + 1], w[2 * q]);
#pragma unroll
    for (int q = 0; q < 2; ++q) b[q] = bsel(m1, a[2 * q + 1], a[2 * q]);
    return bsel(m2, b[1], b[0]);
}

// quad-local lane exchange through DPP (a VALU modifier: no LDS round trip)
template <int CTRL>
__device__ __forceinline__ uint32_t quad_dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t quad_bcast0(uint32_t v) { return quad_dpp<0x00>(v); }    // quad_perm(0,0,0,0)
__device__ __forceinline__ uint32_t quad_or_all(uint32_t v) {
    v |= quad_dpp<0xB1>(v);  // quad_perm(1,0,3,2): xor 1
    v |= quad_dpp<0x4E>(v);  // quad_perm(2,3,0,1): xor 2
    return v;
}

// inclusive prefix sum over the 64 lanes of a wave
// Inclusive prefix sum over the wave's 64 lanes by DPP: shifts by 1, 2, 4, 8 within each row of 16
// lanes, then the row broadcasts of lanes 15 (into rows 1 and 3) and 31 (into rows 2 and 3). Twelve
// VALU and no LDS: the __shfl_up form (SKQ_SCAN_DPP=0) is six dependent ds_bpermute round trips
// and keeps six 64-bit lane masks in SGPRs, which k_map1 spills to VGPR lanes.
#ifndef SKQ_SCAN_DPP
#define SKQ_SCAN_DPP 1
#endif
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v) {
    // (bound_ctrl off: a lane whose source is out of its row, or whose row is masked, adds the 0)
    return v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#if SKQ_SCAN_DPP
    (void)lane;
    v = dpp_add<0x111, 0xF>(v);  // row_shr:1
    v = dpp_add<0x112, 0xF>(v);  // row_shr:2
    v = dpp_add<0x114, 0xF>(v);  // row_shr:4
    v = dpp_add<0x118, 0xF>(v);  // row_shr:8
    v = dpp_add<0x142, 0xA>(v);  // row_bcast:15
    v = dpp_add<0x143, 0xC>(v);  // row_bcast:31
    return v;
#else
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(v, o, 64);
        if (lane >= o) v += x;
    }
    return v;
#endif
}
// lane 63's value, wave-uniform (v_readlane: no LDS round trip)
__device__ __forceinline__ uint32_t wave_last(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// probes per wave held in LDS: 512 per k slot (a 64-read wave of 150 bp reads averages ~384
// at k = 31; a read that does not fit takes the slow path)
__host__ __device__ inline uint32_t probe_cap(uint32_t nk) { return 512u * (nk < 1 ? 1 : (nk > 4 ? 4 : nk)); }
#if SKQ_PART == 0
size_t chain_lds_bytes(uint32_t nk) { return 256 + (size_t)(WG / 64) * probe_cap(nk) * 5; }
#endif  // SKQ_PART == 0

// k_probe: every retained hash -> the offset of its postings list (equivalence class).
//   1. each wave lists its 64 reads' retained hashes (the probes) in LDS (wave prefix sum);
//   2. each quad of lanes resolves probes cooperatively: ONE coalesced 64-B load brings a
//      bucket into the quad (16 B per lane), the key match and the list offset are combined
//      with DPP quad permutes; QU loads per quad are kept in flight;
//   3. each lane writes its read's list offsets out, SoA like the hashes (lofs[(i*lcap + j)*n
//      + r]), and flags reads the fast path cannot take (pflag = 1, listed for k_chain_slow).
#if SKQ_PART == 0
__global__ __launch_bounds__(WG) void k_probe(ChainParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t PW_CAP = probe_cap(p.nk);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // table descriptors in LDS: indexing the kernel-argument array by a lane-varying k slot
    // would load it from memory behind an s_waitcnt vmcnt(0), serialising the bucket loads
    DevTable* s_tabs = reinterpret_cast<DevTable*>(smem);
    uint32_t* sp = reinterpret_cast<uint32_t*>(smem + 256) + wv * PW_CAP;                  // keys, then list offsets
    uint8_t* sk = smem + 256 + (size_t)(WG / 64) * PW_CAP * 4 + (size_t)wv * PW_CAP;       // k slot per probe
    if (threadIdx.x < SKQ_MAX_K) s_tabs[threadIdx.x] = p.tabs[threadIdx.x];
    const uint64_t r = (uint64_t)blockIdx.x * WG + threadIdx.x;
    const bool live = r < p.n;
    const bool ok = live && (!p.status || (p.status[r] & SKQ_STATUS_MASK) == SKQ_READ_OK);
    bool slow = ok && p.nk > (uint32_t)NK_FAST;

    // ---- 1. probe list
    uint32_t cnt[NK_FAST];
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < NK_FAST; ++i) {
        cnt[i] = 0;
        if (!ok || slow || (uint32_t)i >= p.nk || !p.tabs[i].present || (p.present && !p.present[r * p.nk + i]))
            continue;
        cnt[i] = hash_count(p, r, i);
        if (cnt[i] > p.lcap) slow = true;  // (lcap <= HFAST: counts are packed 8 bits per k)
        h += cnt[i];
    }
    if (slow) h = 0;
    const uint32_t incl = wave_incl_scan(h, lane);
    const uint32_t base = incl - h;
    if (incl > PW_CAP) slow = true;
    // the reads that fit form a prefix of the wave (incl is monotone): probes end at the last one
    const uint64_t fit = __ballot(incl <= PW_CAP);
    const uint32_t H = fit ? __shfl(incl, 63 - __builtin_clzll(fit), 64) : 0u;
    if (ok && !slow) {
        uint32_t q = base;
#pragma unroll
        for (int i = 0; i < NK_FAST; ++i) {
            if (!cnt[i]) continue;
            uint64_t hstride;
            const uint32_t* hs = hash_list(p, r, i, cnt[i], hstride);
            for (uint32_t j0 = 0; j0 < cnt[i]; j0 += 8) {  // 8 loads in flight, then the LDS writes
                uint32_t hv[8];
#pragma unroll
                for (uint32_t u = 0; u < 8; ++u) hv[u] = j0 + u < cnt[i] ? hs[(j0 + u) * hstride] : 0u;
#pragma unroll
                for (uint32_t u = 0; u < 8; ++u) {
                    if (j0 + u < cnt[i]) {
                        sp[q] = hv[u];
                        sk[q] = (uint8_t)i;
                        ++q;
                    }
                }
            }
        }
    }
    __syncthreads();

    // ---- 2. quad-cooperative probes: key -> list offset (~0u: miss). Each quad keeps QU
    //         independent bucket loads in flight, then resolves them.
    {
        constexpr uint32_t QU = 8;
        const uint32_t c = lane & 3;
        for (uint32_t p0 = (lane >> 2) * QU; p0 < H; p0 += 16 * QU) {
            uint32_t key[QU], bk[QU], ks[QU];
            uint4 v[QU];
#pragma unroll
            for (uint32_t u = 0; u < QU; ++u) {
                const uint32_t pi = p0 + u;
                key[u] = pi < H ? sp[pi] : 0u;
                ks[u] = pi < H ? (sk[pi] & (SKQ_MAX_K - 1)) : 0u;
                const DevTable& t = s_tabs[ks[u]];
                bk[u] = home_bucket(key[u], t.nbuckets);
                v[u] = pi < H ? *reinterpret_cast<const uint4*>(p.buckets + (t.bucket_base + bk[u]) * BUCKET_WORDS + 4 * c)
                              : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t u = 0; u < QU; ++u) {
                const uint32_t pi = p0 + u;
                if (pi >= H) break;  // uniform within the quad
                uint32_t lo = ~0u;
                uint4 vv = v[u];
                const DevTable& t = s_tabs[ks[u]];
                for (uint32_t q = 0; q < t.max_probe; ++q) {
                    if (q) {
                        bk[u] = bk[u] + 1 == t.nbuckets ? 0 : bk[u] + 1;
                        vv = *reinterpret_cast<const uint4*>(p.buckets + (t.bucket_base + bk[u]) * BUCKET_WORDS + 4 * c);
                    }
                    const uint32_t hdr = quad_bcast0(vv.x);
                    const uint32_t m = hdr & 7u;
                    // words 1..m are keys, word BUCKET_LIST0 + j the list offset of key j
                    const uint32_t wv4[4] = {vv.x, vv.y, vv.z, vv.w};
                    uint32_t match = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint32_t w = 4 * c + e;
                        if (w >= 1 && w <= m && wv4[e] == key[u]) match = w;  // record j = w - 1
                    }
                    match = quad_or_all(match);
                    if (match) {
                        const uint32_t lw = BUCKET_LIST0 + match - 1;  // word holding the list offset
                        uint32_t x = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (4 * c + e == lw) x = wv4[e];
                        lo = quad_or_all(x);
                        break;
                    }
                    if (!((hdr >> 3) & 1u)) break;
                }
                if (c == 0) sp[pi] = lo;
            }
        }
    }
    __syncthreads();
    if (!live) return;
    p.pflag[r] = (ok && slow) ? 1 : 0;  // k_count lists it for k_chain_slow
    if (!ok || slow) return;
    uint32_t q = base;
#pragma unroll
    for (int i = 0; i < NK_FAST; ++i)
        for (uint32_t j = 0; j < cnt[i]; ++j) p.lofs[((uint64_t)i * p.lcap + j) * p.n + r] = sp[q++];
}
#endif  // SKQ_PART == 0

// k_count: one lane per read. Counts the read's list offsets per distinct list (usually 1-3),
// expands each distinct list into the per-transcript table with its packed per-k counts —
// count(t, k) = sum over distinct lists L containing t of count(L, k), exactly the reference's
// per-posting count (src/sparse_chaining.cpp:48-73) — then filters, scores and sorts.
template <int NK>
__global__ __launch_bounds__(WG) void k_count(ChainParams p) {
    const uint64_t r = (uint64_t)blockIdx.x * WG + threadIdx.x;
    if (r >= p.n) return;
    // the per-read words are loaded together, before anything branches on them
    uint32_t cnts[NK];
    const uint8_t st = p.status ? p.status[r] : (uint8_t)SKQ_READ_OK;
    const uint8_t pf = p.pflag[r];
#pragma unroll
    for (int i = 0; i < NK; ++i) cnts[i] = hash_count(p, r, i);
    if ((st & SKQ_STATUS_MASK) != SKQ_READ_OK) {
        p.cand_cnt[r] = 0;  // not sketched (invalid or short read)
        return;
    }
    if (pf) {  // flagged by k_probe / the fused sketch: the slow chain path takes it
        list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
        p.cand_cnt[r] = 0;
        return;
    }
    bool slow = false;
    CountTable<DLISTS> lt;  // list offset -> packed per-k counts
    lt.init();
#pragma unroll
    for (int i = 0; i < NK; ++i) {
        if (!p.tabs[i].present || (p.present && !p.present[r * NK + i])) continue;
        const uint32_t cnt = cnts[i];
        const uint32_t inc = 1u << (8 * i);
        const uint32_t* lo_i = p.lofs + (uint64_t)i * p.lcap * p.n + r;
        for (uint32_t j0 = 0; j0 < cnt && !slow; j0 += 4) {  // 4 coalesced loads in flight
            uint32_t lv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) lv[u] = j0 + u < cnt ? lo_i[(uint64_t)(j0 + u) * p.n] : ~0u;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (lv[u] != ~0u && !lt.add(lv[u], inc)) slow = true;
        }
    }
    CountTable<DCAP> tab;  // transcript -> packed per-k counts
    tab.init();
    // expand the distinct lists: the first 4 heads ([n, t0, t1, t2]) are loaded together,
    // lists beyond 4 (rare) one at a time
    uint4 head[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
        head[e] = (!slow && (uint32_t)e < lt.nd) ? *reinterpret_cast<const uint4*>(p.lists + lt.ids[e])
                                                : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (!__any(!slow && (uint32_t)e < lt.nd)) break;
        if (slow || (uint32_t)e >= lt.nd) continue;
        const uint32_t n = head[e].x;
        for (uint32_t q = 0; q < n; ++q) {
            const uint32_t x = q == 0 ? head[e].y : q == 1 ? head[e].z : q == 2 ? head[e].w : p.lists[lt.ids[e] + 1 + q];
            if (!tab.add(x, lt.cnts[e])) {
                slow = true;
                break;
            }
        }
    }
    for (uint32_t e = 4; e < (uint32_t)DLISTS; ++e) {
        if (!__any(!slow && e < lt.nd)) break;
        if (slow || e >= lt.nd) continue;
        const uint32_t lo = pick8(lt.ids, e);
        const uint32_t inc = pick8(lt.cnts, e);
        const uint32_t n = p.lists[lo];
        for (uint32_t q = 0; q < n; ++q) {
            if (!tab.add(p.lists[lo + 1 + q], inc)) {
                slow = true;
                break;
            }
        }
    }
    if (slow) {
        list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
        p.cand_cnt[r] = 0;
        return;
    }
    // per-k maximum (src/sparse_chaining.cpp:76-82) and the integer form of the double
    // threshold: (double)c >= fraction * max  <=>  c >= ceil(fraction * max)   (:84-87, :93)
    // (counts here are <= 255, so a threshold clamped to 256 rejects the same transcripts; a
    // NaN or non-positive threshold accepts everything, as `c < thr` is then false.)
    uint32_t need[NK];
#pragma unroll
    for (int i = 0; i < NK; ++i) {
        uint32_t m = 0;
#pragma unroll
        for (int d = 0; d < DCAP; ++d) m = max(m, (tab.cnts[d] >> (8 * i)) & 0xFFu);
        const double thr = p.fraction * (double)m;
        uint32_t ti = 0;
        if (thr > 0.0) ti = thr >= 256.0 ? 256u : (uint32_t)ceil(thr);
        need[i] = ti;
    }
    uint64_t key[DCAP];
#pragma unroll
    for (int d = 0; d < DCAP; ++d) {
        bool ok = (uint32_t)d < tab.nd;
        uint32_t score = 0;
#pragma unroll
        for (int i = 0; i < NK; ++i) {
            const uint32_t c = (tab.cnts[d] >> (8 * i)) & 0xFFu;
            ok &= c >= need[i];
            score += c;
        }
        // sort key: score desc, tid asc (src/sparse_chaining.cpp:108-109, ties normalised)
        key[d] = ok ? (((uint64_t)(0xFFFFFFFFu - score) << 32) | tab.ids[d]) : ~0ull;
    }
    // only entries < nd can be candidates: sort 8 when no lane of the wave has more
    if (__any(tab.nd > 8u)) {
        bitonic_sort<DCAP>(key);
    } else {
        uint64_t k8[8];
#pragma unroll
        for (int d = 0; d < 8; ++d) k8[d] = key[d];
        bitonic_sort<8>(k8);
#pragma unroll
        for (int d = 0; d < 8; ++d) key[d] = k8[d];
#pragma unroll
        for (int d = 8; d < DCAP; ++d) key[d] = ~0ull;
    }
    uint32_t nc = 0;
    // SoA layout: candidate j of read r at cand_tid[j*n + r]
    uint32_t* ct = p.cand_tid + r;
    uint32_t* cs = p.cand_score + r;
#pragma unroll
    for (int d = 0; d < DCAP; ++d) {
        if (key[d] != ~0ull) {
            const uint32_t tid = (uint32_t)key[d];
            const uint32_t score = 0xFFFFFFFFu - (uint32_t)(key[d] >> 32);
            ct[(uint64_t)d * p.n] = tid;
            cs[(uint64_t)d * p.n] = score;
            ++nc;
        }
    }
    p.cand_cnt[r] = nc;
}

// More k slots than the count kernels take (NK_FAST): every sketched read goes to the slow chain
// path; the others get no candidates.
#if SKQ_PART == 0
__global__ __launch_bounds__(WG) void k_route_slow(ChainParams p) {
    const uint64_t r = (uint64_t)blockIdx.x * WG + threadIdx.x;
    if (r >= p.n) return;
    p.cand_cnt[r] = 0;
    if (!p.status || (p.status[r] & SKQ_STATUS_MASK) == SKQ_READ_OK)
        list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
}
#endif  // SKQ_PART == 0

// k_count3: one lane per read, like k_count, with
//   * the read's list offsets de-duplicated by a register sorting network (equal offsets form
//     runs; a run of length c adds c to each transcript of that list at this k),
//   * per-read transcript counts in a lane-private open-addressing table in LDS (slot s of
//     lane t at [s][t]: bank-conflict free; one word (tid << 8 | count) per slot when there is
//     one k, else a tid word and a packed-counts word). Every insert makes one branch-free
//     probe (a write that does not land goes to the lane's sink slot); items whose slot is
//     taken by another transcript are parked in a per-lane pending list and placed by one
//     probing loop at the end,
//   * the per-read words and the first 8 list offsets loaded together up front, and the list
//     heads and second quads (tids 3..6) gathered in batches,
//   * 32-bit sort keys ((1023 - score) << 22 | tid; needs ntx <= 2^22, scores <= 4 * 255).
constexpr int TS = DCAP;  // distinct transcripts per read on the fast path (slot TS: sink)
constexpr int PEND = 8;   // parked collisions per read (slot PEND: sink)

// swap with the other lane of the pair (quad_perm(1,0,3,2))
__device__ __forceinline__ uint32_t pair_swap(uint32_t v) { return quad_dpp<0xB1>(v); }
__device__ __forceinline__ uint4 pair_swap(uint4 v) {
    return make_uint4(pair_swap(v.x), pair_swap(v.y), pair_swap(v.z), pair_swap(v.w));
}

// Per-read transcript counter of the fast chain path (src/sparse_chaining.cpp:55-110): a
// lane-private open-addressing table of TS slots in LDS, slot s at tab[s * WG] (slot TS: a sink
// for writes not taken), W words per slot (NK == 1: tid << 8 | count; else tid, then 4 packed
// 8-bit per-k counts), and up to PEND parked items at pend[e * PS] (slot PEND: sink).
template <int NK, int PS>
struct Counter {
    static constexpr int W = NK == 1 ? 1 : 2;
    uint32_t* tab;   // this lane's slot 0
    uint32_t* pend;  // this lane's parked item 0
    uint32_t occ = 0;  // bit s: slot s holds a transcript
    uint32_t np = 0;   // parked items

    __device__ Counter(uint32_t* t, uint32_t* pe) : tab(t), pend(pe) {}
    __device__ static uint32_t slot_of(uint32_t x) { return (x * 0x9E3779B1u) >> 28; }
    __device__ static uint32_t slot2_of(uint32_t x) { return (x * 0x85EBCA77u) >> 28; }
    __device__ uint32_t& at(uint32_t w) { return tab[w * WG]; }

    // transcript x gains rl at k slot i. Two candidate slots, checked in order (slots are never
    // freed, so a transcript found in neither is in neither); both taken by other transcripts:
    // parked for the linear-probing pass that runs after every direct insert
    __device__ __forceinline__ void insert(uint32_t x, uint32_t rl, int i, bool valid) {
        const uint32_t s1 = slot_of(x), s2 = slot2_of(x);
        const bool u1 = (occ >> s1) & 1u, u2 = (occ >> s2) & 1u;
        if (W == 1) {
            const uint32_t e1 = at(s1), e2 = at(s2);
            const bool h1 = u1 && (e1 >> 8) == x, h2 = u2 && (e2 >> 8) == x;
            const bool c1 = !u1 || h1, c2 = !u2 || h2;
            const uint32_t sl = c1 ? s1 : s2, e = c1 ? e1 : e2;
            const bool hit = c1 ? h1 : h2;
            const bool take = valid && (c1 || c2);
            at(take ? sl : (uint32_t)TS) = hit ? e + rl : (x << 8) | rl;
            occ |= take ? (1u << sl) : 0u;
            const bool park = valid && !take;
            pend[min(np, (uint32_t)PEND) * PS] = x | (rl << 22) | ((uint32_t)i << 29);
            np += park ? 1u : 0u;
        } else {
            const uint32_t t1 = at(2 * s1), t2 = at(2 * s2);
            const bool h1 = u1 && t1 == x, h2 = u2 && t2 == x;
            const bool c1 = !u1 || h1, c2 = !u2 || h2;
            const uint32_t sl = c1 ? s1 : s2;
            const bool hit = c1 ? h1 : h2;
            const uint32_t cx = at(2 * sl + 1);
            const bool take = valid && (c1 || c2);
            const uint32_t ws = take ? sl : (uint32_t)TS;
            at(2 * ws) = x;
            at(2 * ws + 1) = (hit ? cx : 0u) + (rl << (8 * i));
            occ |= take ? (1u << sl) : 0u;
            const bool park = valid && !take;
            pend[min(np, (uint32_t)PEND) * PS] = x | (rl << 22) | ((uint32_t)i << 29);
            np += park ? 1u : 0u;
        }
    }

    // parked items: full linear probing. false: more than PEND parked or more than TS distinct
    // transcripts (the read takes the slow chain path)
    __device__ __forceinline__ bool drain() {
        if (np > (uint32_t)PEND) return false;
        for (uint32_t e = 0; e < np; ++e) {
            const uint32_t it = pend[e * PS];
            const uint32_t x = it & 0x3FFFFFu, rl = (it >> 22) & 0x7Fu;
            const int i = (int)(it >> 29);
            uint32_t q = slot_of(x);
            bool done = false;
            for (int z = 0; z < TS && !done; ++z) {
                const bool used = (occ >> q) & 1u;
                if (W == 1) {
                    const uint32_t ev = at(q);
                    if (!used || (ev >> 8) == x) {
                        at(q) = used ? ev + rl : (x << 8) | rl;
                        occ |= 1u << q;
                        done = true;
                    }
                } else {
                    const uint32_t tx = at(2 * q);
                    if (!used || tx == x) {
                        at(2 * q) = x;
                        at(2 * q + 1) = (used ? at(2 * q + 1) : 0u) + (rl << (8 * i));
                        occ |= 1u << q;
                        done = true;
                    }
                }
                q = (q + 1) & (TS - 1);
            }
            if (!done) return false;
        }
        return true;
    }

    // filter and order (src/sparse_chaining.cpp:76-110), write the read's candidates and return
    // their number; key[] holds them first, in output order
    __device__ __forceinline__ uint32_t finish(const ChainParams& p, uint64_t r, uint32_t (&key)[TS]) {
        // two passes over the table (the slots are re-read rather than held in registers):
        // per-k maximum (src/sparse_chaining.cpp:76-82), then the filter
        // (double)c >= fraction * max  <=>  c >= ceil(fraction * max)  (:84-87, :93), as in k_count
        auto slot_counts = [&](int sl) -> uint32_t {
            const uint32_t c = W == 1 ? at(sl) & 0xFFu : at(2 * sl + 1);
            return ((occ >> sl) & 1u) ? c : 0u;
        };
        uint32_t need[NK];
        {
            uint32_t m[NK] = {};
#pragma unroll
            for (int sl = 0; sl < TS; ++sl) {
                const uint32_t c = slot_counts(sl);
#pragma unroll
                for (int i = 0; i < NK; ++i) m[i] = max(m[i], (c >> (8 * i)) & 0xFFu);
            }
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const double thr = p.fraction * (double)m[i];
                uint32_t ti = 0;
                if (thr > 0.0) ti = thr >= 256.0 ? 256u : (uint32_t)ceil(thr);
                need[i] = ti;
            }
        }
#pragma unroll
        for (int sl = 0; sl < TS; ++sl) {
            const uint32_t c = slot_counts(sl);
            const uint32_t tid = W == 1 ? at(sl) >> 8 : at(2 * sl);
            bool ok = (occ >> sl) & 1u;
            uint32_t score = 0;
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const uint32_t ci = (c >> (8 * i)) & 0xFFu;
                ok &= ci >= need[i];
                score += ci;
            }
            // score desc, tid asc (src/sparse_chaining.cpp:108-109, ties normalised)
            key[sl] = ok ? ((1023u - score) << 22) | tid : ~0u;
        }
        bitonic_sort<TS>(key);
        uint32_t nc = 0;
        uint32_t* ct = p.cand_tid + r;
        uint32_t* cs = p.cand_score + r;
#pragma unroll
        for (int d = 0; d < TS; ++d) {
            if (key[d] != ~0u) {
                const uint32_t tid = key[d] & 0x3FFFFFu;
                const uint32_t score = 1023u - (key[d] >> 22);
                ct[(uint64_t)d * p.n] = tid;
                cs[(uint64_t)d * p.n] = score;
                ++nc;
            }
        }
        p.cand_cnt[r] = nc;
        return nc;
    }
};

// Compact tables (ChainParams::wpil): the list offset of a long entry, from bits 22-31 of its
// words 4-7 (the odd lane's half)
__device__ __forceinline__ uint32_t cmp_long_off(const uint4& hi) {
    return (hi.x >> 22) | ((hi.y >> 22) << 10) | ((hi.z >> 22) << 20) | ((hi.w >> 22) << 30);
}
constexpr uint32_t TID_MASK = 0x3FFFFFu;

// Up to 8 retained hashes of k slot i against a wide or compact (CMP) table: dl[u] = the entry's
// word offset or ~0u, hk[u] the hash (compact entries hold their key). Entries are gathered by
// lane pairs (each lane loads one 16-B half of both lanes' entries, so a pair fetches whole 32-B
// entries; then the two swap the half that belongs to the other), 4 per lane in flight; both
// lanes of every pair must run this.
template <int NK, int PS, bool CMP = false, int B = 4>
__device__ __forceinline__ void wide_chunk(Counter<NK, PS>& c, const ChainParams& p, const uint32_t* wd,
                                           const uint32_t (&dl)[8], const uint32_t (&hk)[8], bool odd, int i) {
    static_assert(B == 4 || B == 8, "batch of 4 or 8 entries per lane");
#pragma unroll
    for (int u0 = 0; u0 < 8; u0 += B) {
        bool any = false;
#pragma unroll
        for (int u = 0; u < B; ++u) any |= dl[u0 + u] != ~0u;
        if (!__any(any)) continue;
        uint4 la[B], lb[B], head[B], more[B];
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const uint32_t mine = dl[u0 + u], theirs = pair_swap(mine);
            const uint32_t ea = odd ? theirs : mine, eb = odd ? mine : theirs;
            const uint32_t part = odd ? 4u : 0u;
            la[u] = *reinterpret_cast<const uint4*>(wd + (ea != ~0u ? (uint64_t)ea : 0ull) + part);
            lb[u] = *reinterpret_cast<const uint4*>(wd + (eb != ~0u ? (uint64_t)eb : 0ull) + part);
        }
        uint32_t nn[B];  // tids in the entry (> 7: the list continues at lists[offset])
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const uint4 rcv = pair_swap(odd ? la[u] : lb[u]);
            const uint4 h = odd ? rcv : la[u], m = odd ? lb[u] : rcv;
            const bool v = dl[u0 + u] != ~0u;
            head[u] = v ? h : make_uint4(0, 0, 0, 0);
            more[u] = m;
            if (CMP) nn[u] = head[u].x == hk[u0 + u] ? head[u].y >> 22 : 0u;
            else nn[u] = head[u].x;
        }
        bool lng = false;
#pragma unroll
        for (int u = 0; u < B; ++u) lng |= nn[u] > 3;
        const bool any_long = __any(lng);
        constexpr uint32_t TM = CMP ? TID_MASK : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const uint32_t n = nn[u];  // wide: [0x80000000 | offset] for lists longer than 7
            c.insert(head[u].y & TM, 1, i, n > 0);
            c.insert(head[u].z & TM, 1, i, n > 1);
            c.insert(head[u].w & TM, 1, i, n > 2);
            if (any_long) {
                c.insert(more[u].x & TM, 1, i, n > 3);
                c.insert(more[u].y & TM, 1, i, n > 4);
                c.insert(more[u].z & TM, 1, i, n > 5);
                c.insert(more[u].w & TM, 1, i, n > 6);
            }
        }
        // lists longer than 7 (rare): the rest from the postings list, one at a time
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (__any(nn[u] > 7) && nn[u] > 7) {
                const uint32_t lo = CMP ? cmp_long_off(more[u]) : nn[u] & 0x7FFFFFFFu;
                const uint32_t len = p.lists[lo];
                for (uint32_t q = 7; q < len; ++q) c.insert(p.lists[lo + 1 + q], 1, i, true);
            }
    }
}

// one read of k_count3: writes its candidates (and cand_cnt) and returns their number, the
// first nc of key[] holding them in output order. MODE: 0 = lofs hold list offsets (k_probe or
// the fused dir/rank probe), 1 = wide tables, 3 = compact tables (lofs hold the hashes).
// Wide tables are gathered by lane pairs (wide_chunk), so in MODE 1 every lane of the wave runs
// the gather loops, reads past n and inactive reads with no hashes.
template <int NK, int MODE>
__device__ __forceinline__ uint32_t count_read(const ChainParams& p, uint64_t r, uint32_t t, uint32_t (*s_tab)[WG],
                                               uint32_t (*s_pend)[WG], uint32_t (&key)[TS]) {
    constexpr bool COOP = MODE == 1 || MODE == 3;
    const bool inb = r < p.n;
    const uint64_t rr = inb ? r : p.n - 1;  // (p.n > 0)
    // one round trip for everything the read needs first: offsets past the read's count are
    // read and ignored (the lofs array spans lcap >= 16 slots per k)
    // all per-read loads issue before the first branch: the empty asm consumes them, so the
    // compiler can neither sink a load into the branch that uses it nor split the wait
    uint32_t cnts[NK];
    uint32_t st = p.status[rr];  // (never null for this kernel)
    uint32_t pf = p.pflag[rr];
#pragma unroll
    for (int i = 0; i < NK; ++i) cnts[i] = hash_count(p, rr, i);
    uint32_t lv0[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) lv0[u] = p.lofs[(uint64_t)u * p.n + rr];
    asm volatile("" : "+v"(st), "+v"(pf));
#pragma unroll
    for (int i = 0; i < NK; ++i) asm volatile("" : "+v"(cnts[i]));
#pragma unroll
    for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(lv0[u]));
    const bool ok = inb && (st & SKQ_STATUS_MASK) == SKQ_READ_OK;
    if (ok && pf) list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
    const bool act = ok && !pf;
    if (inb && !act) p.cand_cnt[r] = 0;
    if (!COOP && !act) return 0;
    Counter<NK, WG> c(&s_tab[0][t], &s_pend[0][t]);
    // k slots expanded at compile time (an unrolled loop this size exceeds the unroller's limit,
    // and a rolled one would put cnts/lv0 in scratch)
    static_for<NK>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if (!p.tabs[i].present) return;  // uniform
        const bool pres = !(p.present && !p.present[rr * NK + i]);
        if (!COOP && !pres) return;
        const uint32_t cnt = act && pres ? cnts[i] : 0u;
        const uint32_t cmax = COOP ? max(cnt, pair_swap(cnt)) : cnt;  // the pair's trip count
        const uint32_t* lo_i = p.lofs + (uint64_t)i * p.lcap * p.n + rr;
        const uint32_t* wd = p.wdir[i];
        const uint64_t wlen = p.wdir_len[i];
        for (uint32_t j0 = 0; j0 < cmax; j0 += 8) {
            // this chunk's 8 lofs: the prologue's for the first chunk of k slot 0, else loaded
            // (the asm keeps the compiler from merging the two arms into one load through a
            // selected pointer, which would put lv0 in scratch)
            uint32_t xs[8];
            if (i == 0 && j0 == 0) {  // uniform
#pragma unroll
                for (int u = 0; u < 8; ++u) xs[u] = lv0[u];
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    uint32_t g = lo_i[(uint64_t)min(j0 + u, p.lcap - 1) * p.n];
                    asm volatile("" : "+v"(g));
                    xs[u] = g;
                }
            }
            uint32_t dl[8];
            if (COOP) {
                // lofs holds the read's distinct retained hashes, front-packed: each is one
                // entry; wide: a hash past the table is a miss; compact: the slot from the
                // bucket's pilot (the entry's key decides the hit)
                if (MODE == 3) {
                    uint32_t kh[8], pv[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        kh[u] = cmp_key_hash(xs[u], p.wseed[i]);
                        pv[u] = j0 + u < cnt ? p.wpil[i][cmp_scale(kh[u], p.wnb[i])] : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) dl[u] = j0 + u < cnt ? cmp_slot(kh[u], pv[u], wlen) << 3 : ~0u;
                    wide_chunk<NK, WG, true>(c, p, wd, dl, xs, t & 1u, i);
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) dl[u] = (j0 + u < cnt && xs[u] < wlen) ? xs[u] << 3 : ~0u;
                    wide_chunk<NK, WG, false>(c, p, wd, dl, xs, t & 1u, i);
                }
                continue;
            }
            // list offsets: sort, so repeats of one list (different keys, same postings) are
            // counted once with their run length
            uint32_t lv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) lv[u] = j0 + u < cnt ? xs[u] : ~0u;
            bitonic_sort<8>(lv);  // misses (~0u) sort last
            uint32_t rl[8];
            rl[7] = 1;
#pragma unroll
            for (int u = 6; u >= 0; --u) rl[u] = lv[u] == lv[u + 1] ? rl[u + 1] + 1 : 1;
            // compact the distinct lists to the front: (offset << 3 | run - 1) for run starts
            // (offsets < 2^29 words, runs <= 8), everything else sorts last
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const bool start = lv[u] != ~0u && (u == 0 || lv[u] != lv[u - 1]);
                dl[u] = start ? (lv[u] << 3) | (rl[u] - 1) : ~0u;
            }
            bitonic_sort<8>(dl);
            // distinct lists 4 at a time: heads, then the second quads (tids 3..6) of the
            // lists longer than 3, each batch in flight together
#pragma unroll
            for (int u0 = 0; u0 < 8; u0 += 4) {
                if (u0 && !__any(dl[u0] != ~0u)) break;
                uint4 head[4], more[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool v = dl[u0 + u] != ~0u;
                    const uint4 h = *reinterpret_cast<const uint4*>(p.lists + (v ? dl[u0 + u] >> 3 : 0u));
                    head[u] = v ? h : make_uint4(0, 0, 0, 0);
                }
                bool lng = false;
#pragma unroll
                for (int u = 0; u < 4; ++u) lng |= head[u].x > 3;
                const bool any_long = __any(lng);
                if (any_long) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool l = head[u].x > 3;
                        const uint4 h = *reinterpret_cast<const uint4*>(p.lists + (l ? (dl[u0 + u] >> 3) + 4 : 0u));
                        more[u] = l ? h : make_uint4(0, 0, 0, 0);
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t n = head[u].x;  // 0 past the distinct lists
                    const uint32_t run = (dl[u0 + u] & 7u) + 1;
                    c.insert(head[u].y, run, i, n > 0);
                    c.insert(head[u].z, run, i, n > 1);
                    c.insert(head[u].w, run, i, n > 2);
                    if (any_long) {
                        c.insert(more[u].x, run, i, n > 3);
                        c.insert(more[u].y, run, i, n > 4);
                        c.insert(more[u].z, run, i, n > 5);
                        c.insert(more[u].w, run, i, n > 6);
                    }
                }
                // lists longer than 7 (rare): one at a time
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (__any(head[u].x > 7))
                        for (uint32_t q = 7; q < head[u].x; ++q)
                            c.insert(p.lists[(dl[u0 + u] >> 3) + 1 + q], (dl[u0 + u] & 7u) + 1, i, true);
            }
        }
    });
    if (COOP && !act) return 0;
    if (!c.drain()) {
        list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
        p.cand_cnt[r] = 0;
        return 0;
    }
    return c.finish(p, r, key);
}

// Binning epilogue (totals requested): the workgroup's candidates are binned for k_bin_sum as
// k_bin does, straight from registers: counts per transcript bucket in LDS (s_bc, zeroed before),
// one wave scans them (hdr), entries are placed in LDS (s_mem: >= WG * CCAP words no longer in
// use) and the region leaves in coalesced 16-B stores. Every thread of the workgroup calls it.
// (ZERO: s_bc overlays LDS the waves may still be using, so it is zeroed here, between barriers)
template <bool ZERO = false>
__device__ __forceinline__ void bin_candidates(const ChainParams& p, uint32_t t, uint32_t w, uint32_t nc,
                                               const uint32_t (&key)[TS], uint32_t* s_bc, uint32_t* s_mem) {
    const uint32_t bits = p.bin_bits, nb = p.bin_nb, nW = gridDim.x;
    if (ZERO) {
        __syncthreads();
        if (t <= (uint32_t)WG) s_bc[t] = 0;
        __syncthreads();
    }
#pragma unroll
    for (int d = 0; d < TS; ++d)
        if ((uint32_t)d < nc) atomicAdd(&s_bc[(key[d] & 0x3FFFFFu) >> bits], 1u);
    __syncthreads();
    if (t < 64) {  // one wave scans the (<= 256) bucket counts, 4 per lane
        uint32_t c4[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = 4 * t + u;
            c4[u] = b < nb ? s_bc[b] : 0u;
            sum += c4[u];
        }
        const uint32_t incl = wave_incl_scan(sum, t);
        uint32_t run = incl - sum;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = 4 * t + u;
            if (b < nb) {
                p.bin_hdr[(uint64_t)b * nW + w] = run;
                s_bc[b] = run;
            }
            run += c4[u];
        }
        if (t == 63) p.bin_hdr[(uint64_t)nb * nW + w] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < TS; ++d) {
        if ((uint32_t)d >= nc) continue;
        const uint32_t tid = key[d] & 0x3FFFFFu, score = 1023u - (key[d] >> 22);
        const uint32_t pos = atomicAdd(&s_bc[tid >> bits], 1u);
        s_mem[pos] = (tid & ((1u << bits) - 1u)) | (score << bits);
    }
    __syncthreads();
    const uint32_t total = s_bc[nb - 1];
    uint4* reg = reinterpret_cast<uint4*>(p.bin_region + (uint64_t)w * (WG * CCAP));
    const uint4* sr = reinterpret_cast<const uint4*>(s_mem);
    for (uint32_t q = t; q < (total + 3) / 4; q += WG) reg[q] = sr[q];
}

// The count kernel: count_read per lane, then (totals requested) bin_candidates.
template <int NK, int MODE>
__global__ __launch_bounds__(WG) void k_count3(ChainParams p) {
    constexpr int W = NK == 1 ? 1 : 2;
    constexpr int WORDS = ((TS + 1) * W + PEND + 1) * WG;
    static_assert(WORDS >= WG * CCAP, "the region staging reuses the count tables");
    __shared__ __attribute__((aligned(16))) uint32_t s_mem[WORDS];
    __shared__ uint32_t s_bc[WG + 1];
    auto s_tab = reinterpret_cast<uint32_t(*)[WG]>(s_mem);
    auto s_pend = reinterpret_cast<uint32_t(*)[WG]>(s_mem + (TS + 1) * W * WG);
    const uint32_t t = threadIdx.x, w = blockIdx.x;
    const uint64_t r = (uint64_t)w * WG + t;
    const bool bin = p.accumulate && p.bin_nb;  // uniform
    if (bin) {
        s_bc[t] = 0;
        __syncthreads();
    }
    uint32_t key[TS];
    uint32_t nc = 0;
    if (MODE == 1 || MODE == 3 || r < p.n) nc = count_read<NK, MODE>(p, r, t, s_tab, s_pend, key);
    if (bin) bin_candidates(p, t, w, nc, key, s_bc, s_mem);
}

// Entry-parallel count over wide tables for 2..4 k slots (the multi-k quant path: k_sketch, then
// this): k_map1's count phase with per-k counters. Per wave, the 64 reads' retained hashes of
// every k slot are listed in LDS (hash, owning lane | k slot << 6), in passes of CW_P; lane pairs
// take them round-robin, gather one 32-B wide entry each (the even lane inserts t0..t2, the odd
// lane t3..t6) into the owning read's table: TS slots of two words (tid; 8-bit counts per k
// slot), slot s of read o in column (o + s) & 63 of the wave (distinct LDS banks). Then the
// filter of src/sparse_chaining.cpp:76-110 at every k, the candidates, and the binning epilogue.
// Reads with more than TS distinct transcripts go to the slow chain path, as in k_count3.
// The count phase over wide tables for 2..4 k slots, one wave (k_countw): read r's
// cnts[i] retained hashes of k slot i are at lofs (cnts zero for reads not counted); the wave's
// hashes are listed at hl / ow in passes of `cap`; lane pairs gather the entries and insert into
// the per-read tables in the wave's columns of the 2 * TS rows at colbase (tid words EMPTY and
// count words 0 on entry); flagw (the wave's 64 words, zeroed) marks reads with more than TS
// transcripts. Writes each counted read's candidates, or lists it for the slow chain path;
// returns the candidate count, key[] holding them in output order. Every lane must call it.
// R: rounds of 32 entries in flight together (8 measured 5 % slower in the round-2 fused multi-k
// kernel, which LDS held at 3 waves per SIMD)
template <int NK, bool CMP = false, int R = 4>
__device__ __forceinline__ uint32_t wide_count_wave(const ChainParams& p, uint64_t r, uint64_t rr, bool act,
                                                    uint32_t (&cnts)[NK], uint32_t* colbase, uint32_t* hl,
                                                    uint8_t* ow, uint32_t* sll, uint32_t cap, uint32_t* flagw,
                                                    uint32_t lane, uint32_t (&key)[TS]) {
    constexpr uint32_t EMPTY = 0xFFFFFFFFu;
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < NK; ++i) {
        cnts[i] = act && p.tabs[i].present ? min(cnts[i], p.lcap) : 0u;
        m += cnts[i];
    }
    const uint32_t incl = wave_incl_scan(m, lane);
    const uint32_t M = __shfl(incl, 63, 64);  // the wave's retained hashes, all k slots
    const bool odd = lane & 1u;
    auto wd_of = [&](uint32_t i) -> const uint32_t* {
        const uint32_t* w = p.wdir[0];
#pragma unroll
        for (int q = 1; q < NK; ++q) w = i == (uint32_t)q ? p.wdir[q] : w;
        return w;
    };
    auto wlen_of = [&](uint32_t i) -> uint64_t {
        uint64_t w = p.wdir_len[0];
#pragma unroll
        for (int q = 1; q < NK; ++q) w = i == (uint32_t)q ? p.wdir_len[q] : w;
        return w;
    };
    // compact tables: k slot i's hash seed, and the pilot of hash h's bucket (constant i: the
    // selects fold away)
    auto seed_of = [&](uint32_t i) -> uint32_t {
        uint32_t sd = p.wseed[0];
#pragma unroll
        for (int q = 1; q < NK; ++q) sd = i == (uint32_t)q ? p.wseed[q] : sd;
        return sd;
    };
    auto pilot_of = [&](uint32_t i, uint32_t kh) -> uint32_t {
        const uint16_t* pl = p.wpil[0];
        uint32_t nb = p.wnb[0];
#pragma unroll
        for (int q = 1; q < NK; ++q) {
            pl = i == (uint32_t)q ? p.wpil[q] : pl;
            nb = i == (uint32_t)q ? p.wnb[q] : nb;
        }
        return pl[cmp_scale(kh, nb)];
    };
    // an insert whose home slot holds another transcript probes on (rare: not unrolled)
    auto ins_probe = [&](uint32_t x, uint32_t o, uint32_t inc) {
        uint32_t sl = Counter<1, WG>::slot_of(x);
#pragma unroll 1
        for (int z = 1; z < TS; ++z) {
            sl = (sl + 1) & (TS - 1);
            const uint32_t c = (o + sl) & 63u;
            const uint32_t old = atomicCAS(colbase + (2 * sl) * WG + c, EMPTY, x);
            if (old == EMPTY || old == x) {
                atomicAdd(colbase + (2 * sl + 1) * WG + c, inc);
                return;
            }
        }
        atomicOr(&flagw[o], 1u);  // more than TS distinct transcripts
    };
    auto ins = [&](uint32_t x, uint32_t o, uint32_t inc) {
        const uint32_t sl = Counter<1, WG>::slot_of(x), c = (o + sl) & 63u;
        const uint32_t old = atomicCAS(colbase + (2 * sl) * WG + c, EMPTY, x);
        if (old == EMPTY || old == x) atomicAdd(colbase + (2 * sl + 1) * WG + c, inc);
        else ins_probe(x, o, inc);
    };
    uint32_t hx[NK][8];  // the first 8 hashes of every k slot (loaded once, listed in every pass)
#pragma unroll
    for (int i = 0; i < NK; ++i) {
        const uint32_t* src = p.lofs + (uint64_t)i * p.lcap * p.n + rr;
#pragma unroll
        for (int u = 0; u < 8; ++u) hx[i][u] = (uint32_t)u < cnts[i] ? src[(uint64_t)u * p.n] : 0u;
    }

    for (uint32_t pb = 0; pb < M; pb += cap) {  // wave-uniform
        // this lane's entries that fall in the pass, straight from the sketch's hash rows. The
        // first 8 of every k slot (loaded once, before the passes) go in (k slot, rank) order
        // across the wave's reads, so a round of 32 consecutive entries holds one hash of 32
        // different reads: their inserts go to 32 different count tables (read-major order put
        // most of a round into one read's table: 20x the LDS address conflicts of k_map1). The
        // rest (reads with more than 8 at a k: rare) follow in read order, 8 at a time.
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t base = 0;
#pragma unroll
        for (int i = 0; i < NK; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const bool has = (uint32_t)u < cnts[i];
                const uint64_t bal = __ballot(has);
                const uint32_t ee = base + (uint32_t)__builtin_popcountll(bal & lt);
                if (has && ee >= pb && ee < pb + cap) {
                    hl[ee - pb] = hx[i][u];
                    ow[ee - pb] = (uint8_t)(lane | ((uint32_t)i << 6));
                }
                base += (uint32_t)__builtin_popcountll(bal);
            }
        }
        {
            uint32_t m8 = 0;
#pragma unroll
            for (int i = 0; i < NK; ++i) m8 += cnts[i] > 8 ? cnts[i] - 8 : 0u;
            const uint32_t incl8 = wave_incl_scan(m8, lane);
            uint32_t e = base + incl8 - m8;
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const uint32_t c = cnts[i];
                const uint32_t* src = p.lofs + (uint64_t)i * p.lcap * p.n + rr;
#pragma unroll 1
                for (uint32_t j0 = 8; j0 < c; j0 += 8) {
                    uint32_t x[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = j0 + u < c ? src[(uint64_t)(j0 + u) * p.n] : 0u;
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t ee = e + (j0 - 8) + u;
                        if (j0 + u < c && ee >= pb && ee < pb + cap) {
                            hl[ee - pb] = x[u];
                            ow[ee - pb] = (uint8_t)(lane | ((uint32_t)i << 6));
                        }
                    }
                }
                e += c > 8 ? c - 8 : 0u;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t ne = min(M - pb, cap);
        if constexpr (CMP) {
            // compact tables: every listed hash's slot, one lane per entry (all of the lane's
            // pilot loads in flight together), so the lane pairs gather without a dependent load
            constexpr int SB = 4;  // (8 raised the multi-k kernels' VGPRs past 128)
            for (uint32_t e0 = 0; e0 < ne; e0 += 64 * SB) {
                uint32_t kh[SB], pv[SB];
#pragma unroll
                for (int q = 0; q < SB; ++q) {
                    const uint32_t e = e0 + lane + 64 * q;
                    const uint32_t ee = e < ne ? e : 0;
                    const uint32_t i = ow[ee] >> 6;
                    kh[q] = cmp_key_hash(hl[ee], seed_of(i));
                    pv[q] = e < ne ? pilot_of(i, kh[q]) : 0u;
                }
#pragma unroll
                for (int q = 0; q < SB; ++q) {
                    const uint32_t e = e0 + lane + 64 * q;
                    if (e < ne) sll[e] = cmp_slot(kh[q], pv[q], wlen_of(ow[e] >> 6));
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (uint32_t e0 = 0; e0 < ne; e0 += 32 * R) {
            uint4 w[R];
            uint32_t own[R], hk[R];
            bool okk[R];
            if constexpr (CMP) {
                // one entry each, at the slot listed with the hash
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    const uint32_t e = e0 + 32 * u + (lane >> 1);
                    okk[u] = e < ne;
                    const uint32_t ee = okk[u] ? e : 0;
                    hk[u] = hl[ee];
                    own[u] = ow[ee];
                    w[u] = *reinterpret_cast<const uint4*>(wd_of(own[u] >> 6) + (uint64_t)sll[ee] * 8 + (odd ? 4u : 0u));
                }
            } else {
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    const uint32_t ee = e0 + 32 * u + (lane >> 1);
                    const bool in = ee < ne;
                    hk[u] = hl[in ? ee : 0];
                    own[u] = ow[in ? ee : 0];
                    const uint32_t i = own[u] >> 6;
                    okk[u] = in && hk[u] < wlen_of(i);
                    w[u] = *reinterpret_cast<const uint4*>(wd_of(i) + (okk[u] ? (uint64_t)hk[u] << 3 : 0ull) + (odd ? 4u : 0u));
                }
            }
            constexpr uint32_t TM = CMP ? TID_MASK : 0xFFFFFFFFu;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                // tids in the entry, pair-uniform (> 7: the list continues at lists[offset];
                // wide: [0x80000000 | offset]); compact: the even lane's half holds key and F
                const uint32_t mine = CMP ? (w[u].x == hk[u] ? w[u].y >> 22 : 0u) : w[u].x;
                const uint32_t sw = pair_swap(mine);
                const uint32_t n = okk[u] ? (odd ? sw : mine) : 0u;
                const uint32_t qb = odd ? 3u : 0u;
                const uint32_t o = own[u] & 63u, inc = 1u << (8 * (own[u] >> 6));
                // the first attempts (a CAS at each tid's home slot) issue before any result is
                // looked at; a tid found there gets a non-returning add of its k slot's count
                uint32_t xs[4], olds[4];
                bool vs[4];
                xs[0] = (odd ? w[u].x : w[u].y) & TM;
                xs[1] = (odd ? w[u].y : w[u].z) & TM;
                xs[2] = (odd ? w[u].z : w[u].w) & TM;
                xs[3] = w[u].w & TM;
                vs[0] = n > qb;
                vs[1] = n > qb + 1;
                vs[2] = n > qb + 2;
                vs[3] = odd && n > 6;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t sl = Counter<1, WG>::slot_of(xs[q]);
                    olds[q] = vs[q] ? atomicCAS(colbase + (2 * sl) * WG + ((o + sl) & 63u), EMPTY, xs[q]) : 0u;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (!vs[q]) continue;
                    const uint32_t sl = Counter<1, WG>::slot_of(xs[q]);
                    if (olds[q] == EMPTY || olds[q] == xs[q]) atomicAdd(colbase + (2 * sl + 1) * WG + ((o + sl) & 63u), inc);
                    else ins_probe(xs[q], o, inc);
                }
                // lists longer than 7 (rare): the lane holding the offset (wide: even, compact:
                // odd) inserts the rest of the list
                const bool tl = n > 7 && (CMP ? odd : !odd);
                if (__any(tl) && tl) {
                    const uint32_t lo = CMP ? cmp_long_off(w[u]) : n & 0x7FFFFFFFu;
                    const uint32_t len = p.lists[lo];
                    for (uint32_t q = 7; q < len; ++q) ins(p.lists[lo + 1 + q], o, inc);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    uint32_t nc = 0;
    if (act) {
        if (flagw[lane] == 0) {
            // filter and order (src/sparse_chaining.cpp:76-110), as Counter::finish
            uint32_t tx[TS], cx[TS], mx[NK] = {};
#pragma unroll
            for (int sl = 0; sl < TS; ++sl) {
                const uint32_t c = (lane + sl) & 63u;
                tx[sl] = colbase[(2 * sl) * WG + c];
                cx[sl] = tx[sl] != EMPTY ? colbase[(2 * sl + 1) * WG + c] : 0u;
#pragma unroll
                for (int i = 0; i < NK; ++i) mx[i] = max(mx[i], (cx[sl] >> (8 * i)) & 0xFFu);
            }
            uint32_t need[NK];
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const double thr = p.fraction * (double)mx[i];
                uint32_t ti = 0;
                if (thr > 0.0) ti = thr >= 256.0 ? 256u : (uint32_t)ceil(thr);
                need[i] = ti;
            }
#pragma unroll
            for (int sl = 0; sl < TS; ++sl) {
                bool keep = tx[sl] != EMPTY;
                uint32_t score = 0;
#pragma unroll
                for (int i = 0; i < NK; ++i) {
                    const uint32_t ci = (cx[sl] >> (8 * i)) & 0xFFu;
                    keep &= ci >= need[i];
                    score += ci;
                }
                // score desc, tid asc (src/sparse_chaining.cpp:108-109, ties normalised)
                key[sl] = keep ? ((1023u - score) << 22) | tx[sl] : ~0u;
            }
            bitonic_sort<TS>(key);
            uint32_t* ct = p.cand_tid + r;
            uint32_t* cs = p.cand_score + r;
#pragma unroll
            for (int d = 0; d < TS; ++d) {
                if (key[d] != ~0u) {
                    ct[(uint64_t)d * p.n] = key[d] & 0x3FFFFFu;
                    cs[(uint64_t)d * p.n] = 1023u - (key[d] >> 22);
                    ++nc;
                }
            }
            p.cand_cnt[r] = nc;
        } else {
            list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
            p.cand_cnt[r] = 0;
        }
    }
    return nc;
}

constexpr uint32_t CW_P = 512;
template <int NK, bool CMP>
__global__ __launch_bounds__(WG) void k_countw(ChainParams p) {
    static_assert(NK >= 2 && NK <= NK_FAST, "2..4 k slots (8-bit counts packed per k)");
    static_assert(2 * TS >= CCAP, "the binned region reuses the count tables");
    __shared__ __attribute__((aligned(16))) uint32_t s_tabs[2 * TS * WG];
    __shared__ uint32_t s_hl[WG / 64][CW_P];
    __shared__ uint8_t s_ow[WG / 64][CW_P];
    __shared__ uint32_t s_sl[CMP ? WG / 64 : 1][CMP ? CW_P : 1];
    __shared__ uint32_t s_flag[WG];
    __shared__ uint32_t s_bc[WG + 1];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint64_t r = (uint64_t)blockIdx.x * WG + t;
    const bool inb = r < p.n;
    const uint64_t rr = inb ? r : p.n - 1;  // (p.n > 0)
    const bool bin = p.accumulate && p.bin_nb;  // uniform
    constexpr uint32_t EMPTY = 0xFFFFFFFFu;
#pragma unroll
    for (int sl = 0; sl < TS; ++sl) {
        s_tabs[(2 * sl) * WG + t] = EMPTY;
        s_tabs[(2 * sl + 1) * WG + t] = 0;
    }
    s_flag[t] = 0;
    if (bin) s_bc[t] = 0;
    // the read's status, slow flag and per-k counts (as count_read)
    const uint32_t st = p.status[rr], pf = p.pflag[rr];
    uint32_t cnts[NK];
#pragma unroll
    for (int i = 0; i < NK; ++i) cnts[i] = hash_count(p, rr, i);
    const bool ok = inb && (st & SKQ_STATUS_MASK) == SKQ_READ_OK;
    if (ok && pf) list_push(p.ctrl, C_OVF2, C_ERR2, p.ovf2, p.ovf_cap, (uint32_t)r, E_OVF2_FULL);
    const bool act = ok && !pf;
    if (inb && !act) p.cand_cnt[r] = 0;
    uint32_t key[TS];
    __syncthreads();  // (the tables, flags and binning counts above are set)
    const uint32_t nc = wide_count_wave<NK, CMP>(p, r, rr, act, cnts, s_tabs + wv * 64, s_hl[wv], s_ow[wv],
                                                 CMP ? s_sl[wv] : nullptr, CW_P,
                                            s_flag + wv * 64, lane, key);
    // (bin_candidates places entries only after its barriers, when every wave's tables are dead)
    if (bin) bin_candidates(p, t, blockIdx.x, nc, key, s_bc, s_tabs);
}

// Slow chain path: one workgroup per listed read. (tid << 8 | k slot) words are gathered into
// LDS (global scratch beyond SLOW_CAP), sorted, and counted per transcript run.
#if SKQ_PART == 0
// the workgroup's LDS for one read of k_chain_slow (also k_general_slow's)
struct ChainSlowLds {
    uint64_t ent[SLOW_CAP];
    uint32_t max[SKQ_MAX_K];
    uint32_t cnt, nc;
    unsigned long long at;
};

// one listed read, by the whole workgroup (uniform r)
__device__ __forceinline__ void chain_slow_read(const ChainParams& p, uint64_t r, ChainSlowLds& L) {
    uint64_t* s_ent = L.ent;
    uint32_t* s_max = L.max;
    uint32_t& s_cnt = L.cnt;
    uint32_t& s_nc = L.nc;
    unsigned long long& s_at = L.at;
    const uint32_t t = threadIdx.x;
    unsigned long long* bump_s = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_S);
    unsigned long long* bump_c = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_C);
    {
        __syncthreads();
        // pass 1: postings count P
        if (t == 0) s_cnt = 0;
        if (t < SKQ_MAX_K) s_max[t] = 0;
        __syncthreads();
        for (uint32_t i = 0; i < p.nk; ++i) {
            if (!p.tabs[i].present || (p.present && !p.present[r * p.nk + i])) continue;
            const uint32_t hc = hash_count(p, r, i);
            uint64_t hstride;
            const uint32_t* hs = hash_list<true>(p, r, i, hc, hstride);
            uint32_t mine = 0;
            for (uint32_t h = t; h < hc; h += WG) {
                const uint32_t* pp;
                uint32_t np;
                if (probe_list(p, p.tabs[i], hs[h * hstride], pp, np)) mine += np;
            }
            if (mine) atomicAdd(&s_cnt, mine);
        }
        __syncthreads();
        const uint32_t P = s_cnt;
        // entries + candidates: LDS when 2P fits, else 2P words of global scratch
        const bool in_lds = 2 * (uint64_t)P <= SLOW_CAP;
        __syncthreads();
        if (t == 0) {
            s_at = 0;
            if (!in_lds) {
                const unsigned long long at = atomicAdd(bump_s, (unsigned long long)(2 * (uint64_t)P + 1));
                if (at + 2 * (uint64_t)P + 1 <= p.scratch_cap) s_at = at;
                else {
                    atomicOr(&p.ctrl[C_ERR2], (uint32_t)E_SCRATCH);
                    s_at = ~0ull;
                }
            }
            s_cnt = 0;
            s_nc = 0;
        }
        __syncthreads();
        if (s_at == ~0ull) {
            if (t == 0) p.cand_cnt[r] = 0;
            return;
        }
        uint64_t* ent = in_lds ? s_ent : p.scratch + s_at;
        // pass 2: gather
        for (uint32_t i = 0; i < p.nk; ++i) {
            if (!p.tabs[i].present || (p.present && !p.present[r * p.nk + i])) continue;
            const uint32_t hc = hash_count(p, r, i);
            uint64_t hstride;
            const uint32_t* hs = hash_list<true>(p, r, i, hc, hstride);
            for (uint32_t h = t; h < hc; h += WG) {
                const uint32_t* pp;
                uint32_t np;
                if (!probe_list(p, p.tabs[i], hs[h * hstride], pp, np)) continue;
                const uint32_t at = atomicAdd(&s_cnt, np);
                for (uint32_t q = 0; q < np; ++q) ent[at + q] = ((uint64_t)pp[q] << 8) | i;
            }
        }
        __syncthreads();
        uint32_t n2 = pow2_at_least(P);
        if (in_lds && n2 <= SLOW_CAP) {
            for (uint32_t x = P + t; x < n2; x += WG) s_ent[x] = ~0ull;
            __syncthreads();
            block_sort(s_ent, n2);
        } else {
            if (t == 0) serial_sort(ent, P);
            __syncthreads();
        }
        // per-transcript runs: the thread owning a run's first word counts it
        for (uint32_t a = t; a < P; a += WG) {
            if (a > 0 && (ent[a] >> 8) == (ent[a - 1] >> 8)) continue;
            uint32_t c[SKQ_MAX_K];
            for (uint32_t i = 0; i < p.nk; ++i) c[i] = 0;
            for (uint32_t b = a; b < P && (ent[b] >> 8) == (ent[a] >> 8); ++b) c[ent[b] & 0xFF]++;
            for (uint32_t i = 0; i < p.nk; ++i) atomicMax(&s_max[i], c[i]);
        }
        __syncthreads();
        double thr[SKQ_MAX_K];
        for (uint32_t i = 0; i < p.nk; ++i) thr[i] = p.fraction * (double)s_max[i];
        uint64_t* cand = ent + P;
        for (uint32_t a = t; a < P; a += WG) {
            if (a > 0 && (ent[a] >> 8) == (ent[a - 1] >> 8)) continue;
            uint32_t c[SKQ_MAX_K];
            for (uint32_t i = 0; i < p.nk; ++i) c[i] = 0;
            for (uint32_t b = a; b < P && (ent[b] >> 8) == (ent[a] >> 8); ++b) c[ent[b] & 0xFF]++;
            bool ok = true;
            uint32_t score = 0;
            for (uint32_t i = 0; i < p.nk; ++i) {  // src/sparse_chaining.cpp:91-101
                if ((double)c[i] < thr[i]) {
                    ok = false;
                    break;
                }
                score += c[i];
            }
            if (ok) cand[atomicAdd(&s_nc, 1u)] = ((uint64_t)(0xFFFFFFFFu - score) << 32) | (uint32_t)(ent[a] >> 8);
        }
        __syncthreads();
        const uint32_t nc = s_nc;
        n2 = pow2_at_least(nc);
        if (in_lds && P + n2 <= SLOW_CAP) {
            for (uint32_t x = nc + t; x < n2; x += WG) cand[x] = ~0ull;
            __syncthreads();
            block_sort(cand, n2);
        } else {
            if (t == 0) serial_sort(cand, nc);
            __syncthreads();
        }
        uint32_t* ct = p.cand_tid + r;
        uint32_t* cs = p.cand_score + r;
        uint64_t stride = p.n;
        if (nc > (uint32_t)CCAP || p.cpack) {  // (packed layout: always a run, behind a [count, 0] pair)
            const uint32_t hd = p.cpack ? 1u : 0u;
            if (t == 0) {
                const unsigned long long at = atomicAdd(bump_c, (unsigned long long)(nc + hd));
                if (at + nc + hd <= p.cand_ext_cap && at < CAND_EXT) {
                    s_at = at;
                    if (p.cpack) {
                        p.cand_ext[2 * at] = nc;
                        p.cand_ext[2 * at + 1] = 0;
                    } else {
                        p.cand_tid[r] = (uint32_t)at;
                    }
                } else {
                    atomicOr(&p.ctrl[C_ERR2], (uint32_t)E_CAND_EXT);
                    s_at = ~0ull;
                }
            }
            __syncthreads();
            if (s_at == ~0ull) {
                if (t == 0) p.cand_cnt[r] = 0;
                return;
            }
            ct = p.cand_ext + 2 * (s_at + hd);
            cs = ct + 1;
            stride = 2;
        }
        for (uint32_t a = t; a < nc; a += WG) {
            const uint32_t tid = (uint32_t)cand[a];
            const uint32_t score = 0xFFFFFFFFu - (uint32_t)(cand[a] >> 32);
            ct[a * stride] = tid;
            cs[a * stride] = score;
            if (p.accumulate && p.slow_totals) {  // the count kernel binned the fast reads' totals
                atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[tid]), 1ull);
                atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[tid]), (unsigned long long)score);
            }
        }
        if (t == 0) p.cand_cnt[r] = p.cpack ? (CAND_EXT | (uint32_t)s_at) : nc;
    }
}

__global__ __launch_bounds__(WG) void k_chain_slow(ChainParams p) {
    __shared__ ChainSlowLds L;
    const uint32_t cnt = min(p.ctrl[p.ovf_word], p.ovf_cap);
    for (uint32_t j = blockIdx.x; j < cnt; j += gridDim.x) chain_slow_read(p, p.ovf2[j], L);
}

// The general slow paths behind k_slow_wave in one launch: each read on its chain list (ovf4),
// re-sketched first when k_slow_wave left its sketch too (status still ST_SLOW1: the reads on
// ovf3, a subset of ovf4), then chained, by one workgroup. Per read this is k_sketch_slow's then
// k_chain_slow's work in their order; a read's chain reads only its own sets, and the packed
// offsets of its wave's other reads come from shares that a concurrent re-sketch keeps
// (hash_list<true>). Saves the second launch of the batch's tail.
// zero_next (or null): the control words of the frame's other half, zeroed for the next batch here,
// so the launch stream needs no reset between two maps (skq_capi.hip Frame::ctrl_mem)
__global__ __launch_bounds__(WG) void k_general_slow(SketchParams sp, ChainParams p, uint32_t* zero_next) {
    if (zero_next && blockIdx.x == 0 && threadIdx.x < C_WORDS) zero_next[threadIdx.x] = 0;
    // one LDS region for both steps (each ends / starts at a barrier): a workgroup needs no more
    // than k_chain_slow's, so the launch's workgroups still fit beside the side stream's (with
    // both regions apart, 50 KB each, it waited for k_bin_packed's workgroups: 71 µs at cfg3)
    __shared__ union {
        SketchSlowLds s;
        ChainSlowLds c;
    } L;
    const uint32_t cnt = min(p.ctrl[p.ovf_word], p.ovf_cap);
    for (uint32_t j = blockIdx.x; j < cnt; j += gridDim.x) {
        const uint64_t r = p.ovf2[j];
        if (sp.status[r] & ST_SLOW1) sketch_slow_read(sp, r, L.s);  // (uniform)
        chain_slow_read(p, r, L.c);
        __syncthreads();  // (the chain's last LDS reads before the next read's sketch writes)
    }
}

// Wave slow path (fused map, wide or compact tables, 1..4 k slots): one 64-lane workgroup per
// read the map kernel listed (ovf2; the ones with status ST_SLOW1 also need their sketch), so the
// common slow reads (17-255 retained hashes per k, or 17-256 distinct transcripts) cost a few
// microseconds in one launch instead of a workgroup-wide sort each. Sketch: the windows in one
// contiguous run per lane (rebuilt from k bases, then rolled), retained values compacted into LDS,
// a bitonic sort and de-duplication, written exactly as k_sketch_slow writes them. Chain: one
// entry gather per retained hash per lane, its transcripts counted per k slot in an LDS table of
// SW_T slots (tid; 8-bit count per k), the filter of src/sparse_chaining.cpp:76-101, a bitonic
// sort of (score desc, tid asc) keys, the candidates and totals written as k_chain_slow writes
// them. Reads beyond these limits go on to the general paths (k_sketch_slow, k_chain_slow) through
// the second-level lists ovf3 (sketch and chain) and ovf4 (chain).
constexpr uint32_t SW_NW = 512;  // windows per (read, k)
constexpr uint32_t SW_H = 255;   // retained hashes per (read, k) (8-bit counts)
constexpr uint32_t SW_T = 256;   // distinct transcripts per read

// ascending bitonic sort of a[0..n2) in LDS (n2 a power of two), by one wave
template <typename T>
__device__ __forceinline__ void wave_lds_sort(T* a, uint32_t n2, uint32_t lane) {
    for (uint32_t k2 = 2; k2 <= n2; k2 <<= 1)
        for (uint32_t j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
            for (uint32_t x = lane; x < n2; x += 64) {
                const uint32_t y = x ^ j2;
                if (y > x) {
                    const T u = a[x], v = a[y];
                    const bool up = (x & k2) == 0;
                    if (up ? (u > v) : (u < v)) {
                        a[x] = v;
                        a[y] = u;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}


template <int NK, bool CMP>
__global__ __launch_bounds__(64) void k_slow_wave(SketchParams p, ChainParams cp, uint32_t* ovf3, uint32_t* ovf4) {
    __shared__ uint32_t s_h[NK][SW_H + 1];
    __shared__ uint32_t s_tid[SW_T], s_c[SW_T];
    __shared__ uint64_t s_key[SW_T];
    __shared__ uint8_t s_seq[SW_NW + 64 + 16];  // the read's bases (len <= SW_NW + min k - 1)
    __shared__ uint32_t s_m[NK], s_flag, s_nc;
    __shared__ unsigned long long s_at;
    __shared__ uint64_t s_rt[NK * 16 + 4];  // the roll terms per k slot, then the seeds (the rolls
                                            // below are chains of dependent lookups: LDS, not global)
    constexpr uint32_t EMPTY = 0xFFFFFFFFu;
    const uint32_t lane = threadIdx.x;
    const uint32_t cnt = min(cp.ctrl[C_OVF2], cp.ovf_cap);
    if (blockIdx.x >= cnt) return;  // (uniform) nothing listed for this workgroup
    unsigned long long* bump_h = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_H);
    unsigned long long* bump_c = reinterpret_cast<unsigned long long*>(cp.ctrl + C_BUMP_C);
    // runs are cut from chunks this workgroup takes from the shared bump counters: one atomic
    // per chunk instead of one per run (tens of thousands of runs per batch at cfg5 serialise on
    // one counter otherwise). (lane 0 only; ~0ull: the region is exhausted, error recorded)
    __shared__ unsigned long long s_hcur, s_hend, s_ccur, s_cend;
    if (lane == 0) {  // first this workgroup's own stretches (past the bump allocators' capacity)
        s_hcur = p.hash_ext_cap + (uint64_t)blockIdx.x * SW_HCH;
        const bool own = blockIdx.x < SW_GRID;
        s_hend = s_hcur + (own ? SW_HCH : 0u);
        s_ccur = cp.cand_ext_cap + (uint64_t)blockIdx.x * SW_CCH;
        s_cend = s_ccur + (own ? SW_CCH : 0u);
    }
    auto take = [](unsigned long long* bump, unsigned long long& cur, unsigned long long& end, uint32_t need,
                   uint32_t chunk, uint64_t cap) -> unsigned long long {
        if (cur + need > end) {
            const uint32_t g = max(need, chunk);
            const unsigned long long at = atomicAdd(bump, (unsigned long long)g);
            if (at + g > cap) return ~0ull;
            cur = at;
            end = at + g;
        }
        const unsigned long long at = cur;
        cur += need;
        return at;
    };
    for (uint32_t e = lane; e < NK * 16 + 4; e += 64) s_rt[e] = p.rolltab[e];
    wave_sync();
    const uint64_t* seed = s_rt + NK * 16;
    const uint64_t n = cp.n;
    for (uint32_t jr = blockIdx.x; jr < cnt; jr += gridDim.x) {
        const uint32_t r = cp.ovf2[jr];
        const uint8_t st0 = p.status[r];
        bool hashed = false;  // (uniform) the read's retained sets are in s_h / s_m
        uint8_t st = st0 & SKQ_STATUS_MASK;
        if (st0 & ST_SLOW1) {
            // ---- sketch (k_sketch_slow's contract)
            uint64_t start, len;
            read_extent(p.offs, p.fixed_len, r, start, len);
            uint32_t mink = p.ks[0];
#pragma unroll
            for (int i = 1; i < NK; ++i) mink = min(mink, p.ks[i]);
            if (len > (uint64_t)SW_NW + mink - 1 || len > (uint64_t)SW_NW + 64) {  // (s_seq's size)
                if (lane == 0) {
                    list_push(p.ctrl, C_OVF3, C_ERR1, ovf3, p.ovf_cap, r, E_OVF1_FULL);
                    list_push(cp.ctrl, C_OVF4, C_ERR2, ovf4, cp.ovf_cap, r, E_OVF2_FULL);
                }
                continue;
            }
            // the bases to LDS first (all of a lane's loads in flight together): the hashing below
            // reads each base up to twice, in dependent steps
            bool bad = false;
            {
                const uint8_t* g = p.reads + start;
                uint8_t c[(SW_NW + 64 + 63) / 64];
#pragma unroll
                for (uint32_t t = 0; t < (SW_NW + 64 + 63) / 64; ++t) {
                    const uint32_t q = lane + 64 * t;
                    c[t] = q < len ? g[q] : (uint8_t)'A';
                }
#pragma unroll
                for (uint32_t t = 0; t < (SW_NW + 64 + 63) / 64; ++t) {
                    const uint32_t q = lane + 64 * t;
                    if (q < len) s_seq[q] = c[t];
                    bad |= !(c[t] == 'A' || c[t] == 'C' || c[t] == 'G' || c[t] == 'T');
                }
            }
            bad = __any(bad);
            wave_sync();
            const uint8_t* sb = s_seq;
            st = bad ? SKQ_READ_INVALID : (len < p.maxk ? SKQ_READ_SHORT : SKQ_READ_OK);
            if (!p.hpack)  // (packed layout: the old count words still give the read's region shares)
                for (uint32_t i = lane; i < p.nk; i += 64) p.hash_cnt[(uint64_t)i * n + r] = 0;
            bool fits = true;
            if (st == SKQ_READ_OK) {
#pragma unroll
                for (int i = 0; i < NK; ++i) {
                    const uint32_t k = p.ks[i];
                    const uint32_t nw = (uint32_t)len - k + 1;
                    const uint32_t seg = (nw + 63) / 64;  // <= 8
                    const uint32_t wa = min(nw, lane * seg), wb = min(nw, wa + seg);
                    uint32_t got[SW_NW / 64];
                    uint32_t keepb = 0;  // bit u: window wa + u is retained
                    if (wa < wb) {
                        const uint64_t* tab = s_rt + i * 16;
                        uint32_t hlo = 0, hhi = 0;
                        for (uint32_t q = 0; q < k; ++q) roll33(hlo, hhi, seed[(sb[wa + q] >> 1) & 3u]);
#pragma unroll
                        for (uint32_t u = 0; u < SW_NW / 64; ++u) {
                            const uint32_t w = wa + u;
                            if (w < wb) {
                                if (u) roll33(hlo, hhi, tab[((sb[w + k - 1] >> 1) & 3u) * 4 + ((sb[w - 1] >> 1) & 3u)]);
                                got[u] = hlo;
                                keepb |= (hlo <= p.threshold ? 1u : 0u) << u;  // src/sketch.cpp:33-35
                            }
                        }
                    }
                    const uint32_t m = __builtin_popcount(keepb);
                    const uint32_t incl = wave_incl_scan(m, lane);
                    const uint32_t tot = __shfl(incl, 63, 64);
                    if (tot > SW_H) {  // uniform: the general path
                        fits = false;
                        break;
                    }
                    {
                        uint32_t at = incl - m;
#pragma unroll
                        for (uint32_t u = 0; u < SW_NW / 64; ++u)
                            if ((keepb >> u) & 1u) s_h[i][at++] = got[u];
                    }
                    const uint32_t n2 = pow2_at_least(max(tot, 1u));
                    for (uint32_t x = tot + lane; x < n2; x += 64) s_h[i][x] = EMPTY;
                    wave_sync();
                    wave_lds_sort(s_h[i], n2, lane);
                    // de-duplicate in place: each chunk of 64 read (with its predecessor) before
                    // any of its compacted values are written
                    uint32_t u_all = 0, prev = EMPTY;
                    for (uint32_t x0 = 0; x0 < tot; x0 += 64) {
                        const uint32_t x = x0 + lane;
                        const uint32_t v = x < tot ? s_h[i][x] : EMPTY;
                        // (the shuffle runs on every lane: a lane it reads from must be active)
                        const uint32_t up = __shfl_up(v, 1, 64);
                        const uint32_t pv = lane ? up : prev;
                        const bool keep = x < tot && (x == 0 || v != pv);
                        prev = __shfl(v, 63, 64);
                        const uint64_t bm = __ballot(keep);
                        const uint32_t at = u_all + __builtin_popcountll(bm & ((1ull << lane) - 1ull));
                        wave_sync();
                        if (keep) s_h[i][at] = v;
                        u_all += __builtin_popcountll(bm);
                        wave_sync();
                    }
                    if (lane == 0) s_m[i] = 0;
                    // out: <= hcap in the padded slots, else a bump-allocated run in hash_ext
                    // (packed layout: always a run, [count, region share, hashes...], marked in hash_cnt)
                    uint32_t* slot = p.hashes + (uint64_t)i * p.hcap * n + r;
                    uint32_t* dst = slot;
                    uint64_t dstride = n;
                    uint32_t s_share = 0;  // (lane 0: the read's region share, kept in its run mark)
                    if (u_all > p.hcap || p.hpack) {
                        const uint32_t need = run_words(u_all + (p.hpack ? 2u : 0u));
                        if (lane == 0) {
                            const unsigned long long at = take(bump_h, s_hcur, s_hend, need, 1024u, p.hash_ext_cap);
                            s_at = at != ~0ull && at + need <= RUN_MAX ? at : ~0ull;
                            if (s_at == ~0ull) atomicOr(&p.ctrl[C_ERR1], (uint32_t)E_HASH_EXT);
                        }
                        wave_sync();
                        if (s_at == ~0ull) continue;  // (error recorded; hash_cnt stays 0)
                        dst = p.hash_ext + s_at + (p.hpack ? 2u : 0u);
                        dstride = 1;
                        if (lane == 0) {
                            if (p.hpack) {
                                s_share = packed_share(p.hash_cnt, p.hash_ext, (uint64_t)i * n + r);
                                p.hash_ext[s_at + 1] = s_share;
                                p.hash_ext[s_at] = u_all;
                            } else {
                                slot[0] = (uint32_t)s_at;
                            }
                        }
                    }
                    for (uint32_t x = lane; x < u_all; x += 64) dst[(uint64_t)x * dstride] = s_h[i][x];
                    if (lane == 0) {
                        p.hash_cnt[(uint64_t)i * n + r] = p.hpack ? run_mark(s_at, s_share) : u_all;
                        s_m[i] = u_all;
                    }
                }
            }
            if (!fits) {  // hashing starts over in k_sketch_slow (status and hash_cnt rewritten there)
                if (lane == 0) {
                    list_push(p.ctrl, C_OVF3, C_ERR1, ovf3, p.ovf_cap, r, E_OVF1_FULL);
                    list_push(cp.ctrl, C_OVF4, C_ERR2, ovf4, cp.ovf_cap, r, E_OVF2_FULL);
                }
                continue;
            }
            if (lane == 0) p.status[r] = st;
            hashed = true;
        }
        if (st != SKQ_READ_OK) {
            if (lane == 0) cp.cand_cnt[r] = 0;
            continue;
        }
        // ---- chain (k_chain_slow's contract)
        if (!hashed) {  // a read the map kernel sketched: its sets are in the padded slots
            bool fits = true;
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const uint32_t hc = hash_count(cp, r, i);
                if (hc > SW_H) fits = false;
                uint64_t hs;
                const uint32_t* hp = hash_list<true>(cp, r, i, hc, hs);
                for (uint32_t x = lane; x < hc && x < SW_H; x += 64) s_h[i][x] = hp[x * hs];
                if (lane == 0) s_m[i] = hc;
            }
            if (!fits) {
                if (lane == 0) list_push(cp.ctrl, C_OVF4, C_ERR2, ovf4, cp.ovf_cap, r, E_OVF2_FULL);
                continue;
            }
        }
        for (uint32_t x = lane; x < SW_T; x += 64) {
            s_tid[x] = EMPTY;
            s_c[x] = 0;
        }
        if (lane == 0) s_flag = 0;
        wave_sync();
        auto ins = [&](uint32_t tid, uint32_t inc) {
            uint32_t sl = (tid * 0x9E3779B1u) >> 24;
            for (uint32_t z = 0; z < SW_T; ++z) {
                const uint32_t old = atomicCAS(&s_tid[sl], EMPTY, tid);
                if (old == EMPTY || old == tid) {
                    atomicAdd(&s_c[sl], inc);
                    return;
                }
                sl = (sl + 1) & (SW_T - 1);
            }
            s_flag = 1;  // more than SW_T transcripts
        };
#pragma unroll
        for (int i = 0; i < NK; ++i) {
            if (!cp.tabs[i].present) continue;
            const uint32_t m = s_m[i], inc = 1u << (8 * i);
            const uint32_t* wd = cp.wdir[i];
            const uint64_t wlen = cp.wdir_len[i];
            for (uint32_t x = lane; x < m; x += 64) {
                const uint32_t h = s_h[i][x];
                uint64_t at;
                bool ok;
                if (CMP) {
                    const uint32_t kh = cmp_key_hash(h, cp.wseed[i]);
                    at = (uint64_t)cmp_slot(kh, cp.wpil[i][cmp_scale(kh, cp.wnb[i])], wlen) * 8;
                    ok = true;
                } else {
                    ok = h < wlen;
                    at = ok ? (uint64_t)h * 8 : 0;
                }
                const uint4 a = *reinterpret_cast<const uint4*>(wd + at);
                const uint4 b = *reinterpret_cast<const uint4*>(wd + at + 4);
                uint32_t nn;
                if (CMP) nn = ok && a.x == h ? a.y >> 22 : 0u;
                else nn = ok ? a.x : 0u;
                constexpr uint32_t TM = CMP ? TID_MASK : 0xFFFFFFFFu;
                const uint32_t t7[7] = {a.y & TM, a.z & TM, a.w & TM, b.x & TM, b.y & TM, b.z & TM, b.w & TM};
#pragma unroll
                for (uint32_t q = 0; q < 7; ++q)
                    if (q < nn) ins(t7[q], inc);
                if (nn > 7) {  // the rest of a longer list
                    const uint32_t lo = CMP ? cmp_long_off(b) : nn & 0x7FFFFFFFu;
                    const uint32_t L = cp.lists[lo];
                    for (uint32_t q = 7; q < L; ++q) ins(cp.lists[lo + 1 + q], inc);
                }
            }
        }
        wave_sync();
        if (s_flag) {
            if (lane == 0) list_push(cp.ctrl, C_OVF4, C_ERR2, ovf4, cp.ovf_cap, r, E_OVF2_FULL);
            continue;
        }
        // per-k maxima (src/sparse_chaining.cpp:76-82), then the filter (:84-101) as the fast path
        uint32_t mx[NK] = {};
        for (uint32_t x = lane; x < SW_T; x += 64)
            if (s_tid[x] != EMPTY) {
#pragma unroll
                for (int i = 0; i < NK; ++i) mx[i] = max(mx[i], (s_c[x] >> (8 * i)) & 0xFFu);
            }
        uint32_t need[NK];
#pragma unroll
        for (int i = 0; i < NK; ++i) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) mx[i] = max(mx[i], (uint32_t)__shfl_xor(mx[i], d, 64));
            const double thr = cp.fraction * (double)mx[i];
            uint32_t ti = 0;
            if (thr > 0.0) ti = thr >= 256.0 ? 256u : (uint32_t)ceil(thr);
            need[i] = ti;
        }
        if (lane == 0) s_nc = 0;
        wave_sync();
        for (uint32_t x0 = 0; x0 < SW_T; x0 += 64) {
            const uint32_t x = x0 + lane;
            const uint32_t tid = s_tid[x], c = s_c[x];
            bool keep = tid != EMPTY;
            uint32_t score = 0;
#pragma unroll
            for (int i = 0; i < NK; ++i) {
                const uint32_t ci = (c >> (8 * i)) & 0xFFu;
                keep &= ci >= need[i];
                score += ci;
            }
            const uint64_t bm = __ballot(keep);
            const uint32_t at = s_nc + __builtin_popcountll(bm & ((1ull << lane) - 1ull));
            // score desc, tid asc (src/sparse_chaining.cpp:108-109, ties normalised)
            const uint64_t key = ((uint64_t)(0xFFFFFFFFu - score) << 32) | tid;
            wave_sync();
            if (keep) s_key[at] = key;
            if (lane == 0) s_nc += __builtin_popcountll(bm);
            wave_sync();
        }
        const uint32_t nc = s_nc;
        const uint32_t n2 = pow2_at_least(max(nc, 1u));
        for (uint32_t x = nc + lane; x < n2; x += 64) s_key[x] = ~0ull;
        wave_sync();
        wave_lds_sort(s_key, n2, lane);
        uint32_t* ct = cp.cand_tid + r;
        uint32_t* cs = cp.cand_score + r;
        uint64_t stride = n;
        if (nc > (uint32_t)CCAP || cp.cpack) {  // (packed layout: always a run, behind a [count, 0] pair)
            const uint32_t hd = cp.cpack ? 1u : 0u;
            if (lane == 0) {
                const unsigned long long at = take(bump_c, s_ccur, s_cend, nc + hd, 128u, cp.cand_ext_cap);
                if (at != ~0ull && at < CAND_EXT) {
                    s_at = at;
                    if (cp.cpack) {
                        cp.cand_ext[2 * at] = nc;
                        cp.cand_ext[2 * at + 1] = 0;
                    } else {
                        cp.cand_tid[r] = (uint32_t)at;
                    }
                } else {
                    atomicOr(&cp.ctrl[C_ERR2], (uint32_t)E_CAND_EXT);
                    s_at = ~0ull;
                }
            }
            wave_sync();
            if (s_at == ~0ull) {
                if (lane == 0) cp.cand_cnt[r] = 0;
                continue;
            }
            ct = cp.cand_ext + 2 * (s_at + hd);
            cs = ct + 1;
            stride = 2;
        }
        for (uint32_t a = lane; a < nc; a += 64) {
            const uint32_t tid = (uint32_t)s_key[a];
            const uint32_t score = 0xFFFFFFFFu - (uint32_t)(s_key[a] >> 32);
            ct[a * stride] = tid;
            cs[a * stride] = score;
            if (cp.accumulate && cp.slow_totals) {  // the map kernel binned the fast reads' totals
                atomicAdd(reinterpret_cast<unsigned long long*>(&cp.tx_reads[tid]), 1ull);
                atomicAdd(reinterpret_cast<unsigned long long*>(&cp.tx_score[tid]), (unsigned long long)score);
            }
        }
        if (lane == 0) cp.cand_cnt[r] = cp.cpack ? (CAND_EXT | (uint32_t)s_at) : nc;
    }
}

// Per-transcript totals without one scattered atomic per candidate (those run at the fabric's
// random-request rate). Pass 1, one workgroup per 256 reads: the workgroup's candidates are
// grouped by transcript bucket (2^bits ids) with LDS counters and a scan and written, packed as
// (tid & (2^bits - 1)) | score << bits, into the workgroup's own region; hdr[b * nW + w] is
// where bucket b starts in region w (b = nb: the region's total). Candidates that do not pack
// (overflow lists, huge scores) are added directly. Pass 2, one workgroup per (chunk of
// regions, bucket): an LDS histogram of the bucket, flushed with one coalesced atomic per
// non-empty bin into the batch's packed sums tx_acc, which k_fold_totals adds into the running
// totals with atomics (commuting with the slow paths' direct adds) and clears.
__global__ __launch_bounds__(WG) void k_bin(ChainParams p, uint32_t bits, uint32_t nb, uint32_t nW, uint32_t* hdr,
                                           uint32_t* region) {
    __shared__ uint32_t s_cnt[WG + 1], s_fill[WG + 1];
    __shared__ __attribute__((aligned(16))) uint32_t s_reg[WG * CCAP];  // the region, staged
    const uint32_t t = threadIdx.x, w = blockIdx.x;
    const uint64_t r = (uint64_t)w * WG + t;
    if (nb == 0) {  // index too large to bin (> 256 buckets of 2^14): every candidate added directly
        const uint32_t cnt = r < p.n ? p.cand_cnt[r] : 0u;
        const bool ext = cnt > (uint32_t)CCAP;
        const uint32_t* e = ext ? p.cand_ext + 2ull * p.cand_tid[r] : nullptr;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t x = ext ? e[2 * j] : p.cand_tid[(uint64_t)j * p.n + r];
            const uint32_t y = ext ? e[2 * j + 1] : p.cand_score[(uint64_t)j * p.n + r];
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[x]), 1ull);
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[x]), (unsigned long long)y);
        }
        return;
    }
    s_cnt[t] = 0;
    s_fill[t] = 0;
    if (t == 0) s_cnt[WG] = 0;
    __syncthreads();
    uint32_t cnt = r < p.n ? p.cand_cnt[r] : 0u;
    if (cnt > (uint32_t)CCAP) {  // overflow list (k_chain_slow): added directly
        const uint32_t* e = p.cand_ext + 2ull * p.cand_tid[r];
        for (uint32_t j = 0; j < cnt; ++j) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[e[2 * j]]), 1ull);
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[e[2 * j]]), (unsigned long long)e[2 * j + 1]);
        }
        cnt = 0;
    }
    uint32_t tid[CCAP], sc[CCAP];
    const uint32_t smax = 1u << (32 - bits);
    // all CCAP slots are loaded (they exist for every read; stale ones are masked), so the loads
    // are in flight together
    const uint64_t rr = r < p.n ? r : 0;
#pragma unroll
    for (int j = 0; j < CCAP; ++j) {
        const uint32_t a = p.cand_tid[(uint64_t)j * p.n + rr], b = p.cand_score[(uint64_t)j * p.n + rr];
        tid[j] = (uint32_t)j < cnt ? a : 0u;
        sc[j] = (uint32_t)j < cnt ? b : 0u;
    }
#pragma unroll
    for (int j = 0; j < CCAP; ++j) {
        if ((uint32_t)j >= cnt) continue;
        if (sc[j] >= smax) {  // does not pack: added directly
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[tid[j]]), 1ull);
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[tid[j]]), (unsigned long long)sc[j]);
            continue;
        }
        atomicAdd(&s_cnt[tid[j] >> bits], 1u);
    }
    __syncthreads();
    if (t < 64) {  // one wave scans the (<= 256) bucket counts, 4 per lane
        uint32_t c4[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = 4 * t + u;
            c4[u] = b < nb ? s_cnt[b] : 0u;
            sum += c4[u];
        }
        const uint32_t incl = wave_incl_scan(sum, t);
        uint32_t run = incl - sum;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = 4 * t + u;
            if (b < nb) {
                hdr[(uint64_t)b * nW + w] = run;
                s_fill[b] = run;  // running position per bucket
            }
            run += c4[u];
        }
        if (t == 63) hdr[(uint64_t)nb * nW + w] = incl;  // the region's total
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < CCAP; ++j) {
        if ((uint32_t)j >= cnt || sc[j] >= smax) continue;
        const uint32_t b = tid[j] >> bits;
        const uint32_t pos = atomicAdd(&s_fill[b], 1u);
        s_reg[pos] = (tid[j] & ((1u << bits) - 1u)) | (sc[j] << bits);
    }
    __syncthreads();
    // the region leaves in 16-B coalesced stores (scattered 4-B stores would each cost a
    // memory request)
    const uint32_t total = s_fill[nb - 1];  // end of the last bucket = entries in the region
    uint4* reg = reinterpret_cast<uint4*>(region + (uint64_t)w * (WG * CCAP));
    const uint4* sr = reinterpret_cast<const uint4*>(s_reg);
    for (uint32_t q = t; q < (total + 3) / 4; q += WG) reg[q] = sr[q];
}

// The fused map's candidates (per-wave packed layout, ChainParams::cpack: tid | score << 22) binned
// for the totals, one workgroup per map workgroup (the same regions and headers k_map1 used to fill
// in its epilogue): the map kernel ends at its last candidate store and this runs after it (on the
// session's side stream for large batches, beside the next batch's map; the candidate buffers
// alternate by batch parity, so that map writes the other pair). A read the slow paths took has
// no share of its wave's region (its count word is 0 or, once they have run, a CAND_EXT mark) and
// adds its totals itself.
// CAPW: the staged region's capacity in words: WG * CCAP (every candidate a workgroup can have),
// or less — a workgroup with more candidates than that adds them all directly (64-bit atomics into
// the running totals) and leaves its region empty. (1,280 words, ~6 KB of LDS, would fit beside
// five k_map1 workgroups on a CU: measured no faster, launch_bin.)
template <uint32_t CAPW, int G>
__global__ __launch_bounds__(WG) void k_bin_packed(ChainParams p, uint32_t bits, uint32_t nb, uint32_t nWg,
                                                   uint32_t* hdr, uint32_t* region) {
    __shared__ uint32_t s_bc[WG + 1];
    __shared__ uint32_t s_tot;
    __shared__ __attribute__((aligned(16))) uint32_t s_reg[CAPW];
    const uint32_t t = threadIdx.x, w = blockIdx.x, lane = t & 63, v = t >> 6;
    s_bc[t] = 0;
    if (t == 0) s_bc[WG] = 0;
    // wave v takes map wave v of each of the G map workgroups w * G .. w * G + G - 1: their packed
    // words [0, tot) (ChainParams::cand_wtot, the map's own count of them), the first 256 of each
    // in one 16-B load per lane, all G loads issued beside the counts, so the kernel waits on one
    // memory round trip (the words past 256 — a region of more than 4 candidates per read — are
    // read again per lane in both passes below). G > 1: one binned region per G map workgroups,
    // whose bucket segments are G times longer for k_bin_sum4
    uint32_t tot[G];
    uint4 x[G];
    const uint32_t* src[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint64_t W = ((uint64_t)w * G + g) * (WG / 64) + v, r0 = W * 64;
        tot[g] = r0 < p.n ? p.cand_wtot[W] : 0u;  // (wave-uniform)
        src[g] = p.cand_tid + (r0 < p.n ? r0 : 0) * CCAP;
        const uint32_t lim = r0 + 64 <= p.n ? 256u : tot[g];  // (a partial last wave: only what it holds)
        x[g] = lane * 4 < lim ? reinterpret_cast<const uint4*>(src[g])[lane] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const uint32_t mask = (1u << bits) - 1u;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint32_t xs[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (lane * 4 + i < tot[g]) atomicAdd(&s_bc[(xs[i] & 0x3FFFFFu) >> bits], 1u);
        for (uint32_t e = 256 + lane; e < tot[g]; e += 64) atomicAdd(&s_bc[(src[g][e] & 0x3FFFFFu) >> bits], 1u);
    }
    __syncthreads();
    if (t < 64) {  // one wave scans the (<= 256) bucket counts, 4 per lane
        uint32_t c4[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = 4 * t + u;
            c4[u] = b < nb ? s_bc[b] : 0u;
            sum += c4[u];
        }
        const uint32_t bi = wave_incl_scan(sum, t);
        const uint32_t all = wave_last(bi);
        const bool fits = all <= CAPW;
        uint32_t run = bi - sum;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t b = 4 * t + u;
            if (b < nb) {
                hdr[(uint64_t)b * nWg + w] = fits ? run : 0u;
                s_bc[b] = run;
            }
            run += c4[u];
        }
        if (t == 63) {
            hdr[(uint64_t)nb * nWg + w] = fits ? bi : 0u;
            s_tot = bi;
        }
    }
    __syncthreads();
    const bool fits = s_tot <= CAPW;  // (uniform)
    auto place = [&](uint32_t xw) {
        const uint32_t tid = xw & 0x3FFFFFu, score = xw >> 22;
        if (fits) {
            const uint32_t pos = atomicAdd(&s_bc[tid >> bits], 1u);
            s_reg[pos] = (tid & mask) | (score << bits);
        } else {  // (more candidates than the staging holds: straight into the totals)
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[tid]), 1ull);
            atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[tid]), (unsigned long long)score);
        }
    };
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint32_t xs[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (lane * 4 + i < tot[g]) place(xs[i]);
        for (uint32_t e = 256 + lane; e < tot[g]; e += 64) place(src[g][e]);
    }
    if (!fits) return;  // (uniform)
    __syncthreads();
    uint4* reg = reinterpret_cast<uint4*>(region + (uint64_t)w * CAPW);
    const uint4* sr = reinterpret_cast<const uint4*>(s_reg);
    for (uint32_t q = t; q < (s_tot + 3) / 4; q += WG) reg[q] = sr[q];
}

// The fused map's packed candidates summed per transcript with no binning pass, for small
// transcript sets (ntx <= TOT_SMALL_TX): workgroup (chunk c, range q) walks a contiguous stretch of
// map waves' packed regions (16-B loads, ChainParams::cand_wtot words each) and adds
// (1 << 40 | score) into u64 LDS bins for the transcripts of its range (2560 between two maps;
// TOT_RANGE_TX beside a running map: 32 KiB of LDS, so it starts as soon as one map workgroup
// retires on a CU, where 80 KiB waited for three), then adds its non-empty bins into the
// packed sums tx_acc with coalesced atomics. The ranges of one chunk re-read it from the L2 (the
// q-th range of chunk c is workgroup c * R + q). For cfg2 (10k transcripts) this replaces
// k_bin_packed + k_bin_sum_g. Slow reads have no share of their wave's region and add their own.
constexpr uint32_t TOT_SMALL_TX = 16384, TOT_RANGE_TX = 4096, TOT_WG = 1024;
__global__ __launch_bounds__(TOT_WG) void k_tot_small(ChainParams p, uint32_t nwaves, uint32_t per, uint32_t nr, uint32_t range) {
    extern __shared__ unsigned long long s_tb[];  // (range bins, then the chunk's region word counts)
    uint32_t* s_tot = reinterpret_cast<uint32_t*>(s_tb + range);
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6, nt = blockDim.x;  // (256 or TOT_WG threads)
    const uint32_t c = blockIdx.x / nr, q = blockIdx.x % nr;
    const uint32_t lo = q * range, hi = min(p.ntx, lo + range);
    const uint32_t w0 = c * per, w1 = min(nwaves, w0 + per);
    for (uint32_t i = t; i < range; i += nt) s_tb[i] = 0;
    for (uint32_t i = t; i < w1 - w0; i += nt) s_tot[i] = p.cand_wtot[w0 + i];  // (every count in one round trip)
    __syncthreads();
    // each wave takes RB map-wave regions a round, their first 256 words (64 x 16 B; a region holds
    // ~200 words at cfg2) loaded together, the next round's loads issued before this round's adds:
    // one exposed memory round trip per workgroup rather than two per region
    constexpr uint32_t RB = 8;
    auto add = [&](uint32_t x) {
        const uint32_t tid = x & 0x3FFFFFu;
        if (tid - lo < hi - lo) atomicAdd(&s_tb[tid - lo], (1ull << 40) | (unsigned long long)(x >> 22));
    };
    // (the loads are unconditional — a region slot always holds 1024 words; words past its count are
    // ignored below — so no branch splits them and the compiler keeps the next round in flight
    // while this round is summed: vmcnt(RB), not vmcnt(0))
    auto issue = [&](uint32_t Wb, uint4 (&x)[RB]) {
#pragma unroll
        for (uint32_t u = 0; u < RB; ++u) {
            const uint32_t W = min(Wb + u, w1 - 1);
            const uint4* src = reinterpret_cast<const uint4*>(p.cand_tid + (uint64_t)W * 64 * CCAP);
            x[u] = src[lane];
        }
    };
    auto consume = [&](uint32_t Wb, const uint4 (&x)[RB]) {
#pragma unroll
        for (uint32_t u = 0; u < RB; ++u) {
            const uint32_t W = Wb + u;
            const uint32_t tot = W < w1 ? s_tot[W - w0] : 0u;
            const uint32_t xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (lane * 4 + i < tot) add(xs[i]);
            const uint4* src = reinterpret_cast<const uint4*>(p.cand_tid + (uint64_t)W * 64 * CCAP);
            for (uint32_t e = lane + 64; e * 4 < tot; e += 64) {  // (rare: a region past 256 words)
                const uint4 y = src[e];
                const uint32_t ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (e * 4 + i < tot) add(ys[i]);
            }
        }
    };
    const uint32_t STEP = (nt / 64) * RB;
    uint32_t Wb = w0 + wv * RB;
    uint4 xa[RB], xb[RB];
    if (Wb < w1) issue(Wb, xa);
    while (Wb < w1) {  // (a round past the chunk's end loads its last region again, unused)
        const uint32_t Wn = Wb + STEP;
        issue(Wn, xb);
        consume(Wb, xa);
        Wb = Wn;
        if (Wb >= w1) break;
        const uint32_t Wm = Wb + STEP;
        issue(Wm, xa);
        consume(Wb, xb);
        Wb = Wm;
    }
    __syncthreads();
    for (uint32_t i = t; i < hi - lo; i += nt) {
        const unsigned long long a = s_tb[i];
        if (a) atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_acc[lo + i]), a);
    }
}

// the workgroup's bins out with atomics into tx_acc: one packed atomic per non-empty bin
// ((reads << 40) | score: a batch holds < 2^24 reads of score <= 2^10), coalesced over the bins;
// k_fold_totals unpacks the batch's sums once
__device__ __forceinline__ void bins_out(const unsigned long long* s_bins, uint32_t bs, uint32_t b, uint32_t ntx,
                                         uint64_t* tx_acc) {
    for (uint32_t i = threadIdx.x; i < bs; i += WG) {
        const unsigned long long a = s_bins[i];
        const uint32_t tx = b * bs + i;
        if (a && tx < ntx) atomicAdd(reinterpret_cast<unsigned long long*>(&tx_acc[tx]), a);
    }
}

__global__ __launch_bounds__(WG) void k_bin_sum(uint64_t* tx_acc, uint32_t ntx, uint32_t bits, uint32_t nb, uint32_t nW,
                                               uint32_t chunk, const uint32_t* hdr, const uint32_t* region,
                                               uint32_t rstride) {
    extern __shared__ unsigned long long s_bins[];
    const uint32_t t = threadIdx.x, b = blockIdx.y;
    const uint32_t bs = 1u << bits;
    for (uint32_t i = t; i < bs; i += WG) s_bins[i] = 0;
    __syncthreads();
    const uint32_t w0 = blockIdx.x * chunk, w1 = min(nW, w0 + chunk);
    // one lane per region (the header loads of WG regions are coalesced); a segment holds ~16-32
    // entries, read as 16-B words (a lane's load is one line-request for 4 entries, not 1: the
    // texture addresser works per lane-request), 4 in flight, and the next region's header is
    // read ahead. (Two regions' segments in flight per lane measured 31 % slower: 0.093 against
    // 0.071 ms per 10M reads, profiles/r5_totals_kernels_ab.log.)
    constexpr int U = 4;
    uint32_t w = w0 + t;
    uint32_t s0 = 0, s1 = 0;
    if (w < w1) {
        s0 = hdr[(uint64_t)b * nW + w];
        s1 = hdr[(uint64_t)(b + 1) * nW + w];
    }
    while (w < w1) {
        const uint32_t* reg = region + (uint64_t)w * rstride;
        const uint32_t wn = w + WG;
        uint32_t n0 = 0, n1 = 0;
        if (wn < w1) {
            n0 = hdr[(uint64_t)b * nW + wn];
            n1 = hdr[(uint64_t)(b + 1) * nW + wn];
        }
        const uint4* reg4 = reinterpret_cast<const uint4*>(reg);  // (regions are 16-B aligned)
        for (uint32_t q = s0 & ~3u; q < s1; q += 4 * U) {
            uint4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = reg4[min(q / 4 + u, (s1 - 1) / 4)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t j = q + 4 * u + i;
                    if (j >= s0 && j < s1)
                        atomicAdd(&s_bins[xs[i] & (bs - 1u)], (1ull << 40) | (unsigned long long)(xs[i] >> bits));
                }
            }
        }
        w = wn;
        s0 = n0;
        s1 = n1;
    }
    __syncthreads();
    bins_out(s_bins, bs, b, ntx, tx_acc);
}

// k_bin_sum for few, long bucket segments (small transcript sets: a region's segment of a bucket
// holds hundreds of entries): a group of GS lanes per region reads its segment coalesced, U
// loads per lane in flight, instead of one lane walking it (the one-lane walk is a chain of
// dependent round trips: 57 us for 1M reads against 10k transcripts)
template <int GS>
__global__ __launch_bounds__(WG) void k_bin_sum_g(uint64_t* tx_acc, uint32_t ntx, uint32_t bits, uint32_t nW,
                                                  uint32_t chunk, const uint32_t* hdr, const uint32_t* region,
                                                  uint32_t rstride) {
    extern __shared__ unsigned long long s_bins[];
    const uint32_t t = threadIdx.x, b = blockIdx.y;
    const uint32_t bs = 1u << bits;
    for (uint32_t i = t; i < bs; i += WG) s_bins[i] = 0;
    __syncthreads();
    const uint32_t w0 = blockIdx.x * chunk, w1 = min(nW, w0 + chunk);
    const uint32_t g = t / GS, gl = t % GS;
    constexpr int U = 8;
    for (uint32_t w = w0 + g; w < w1; w += WG / GS) {
        const uint32_t* reg = region + (uint64_t)w * rstride;
        const uint32_t s0 = hdr[(uint64_t)b * nW + w], s1 = hdr[(uint64_t)(b + 1) * nW + w];
        for (uint32_t q = s0 + gl; q < s1; q += GS * U) {
            uint32_t x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = reg[min(q + u * GS, s1 - 1)];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (q + u * GS < s1) atomicAdd(&s_bins[x[u] & (bs - 1u)], (1ull << 40) | (unsigned long long)(x[u] >> bits));
        }
    }
    __syncthreads();
    bins_out(s_bins, bs, b, ntx, tx_acc);
}

// k_bin_sum over k_bin_packed's grouped regions (G map workgroups each: a bucket's segment holds
// ~65 entries at cfg3): a group of GS lanes per region reads its segment as 16-B words, U per lane
// in flight (GS * U * 4 entries a round)
template <int GS>
__global__ __launch_bounds__(WG) void k_bin_sum4(uint64_t* tx_acc, uint32_t ntx, uint32_t bits, uint32_t nW,
                                                 uint32_t chunk, const uint32_t* hdr, const uint32_t* region,
                                                 uint32_t rstride) {
    extern __shared__ unsigned long long s_bins[];
    const uint32_t t = threadIdx.x, b = blockIdx.y;
    const uint32_t bs = 1u << bits;
    for (uint32_t i = t; i < bs; i += WG) s_bins[i] = 0;
    __syncthreads();
    const uint32_t w0 = blockIdx.x * chunk, w1 = min(nW, w0 + chunk);
    const uint32_t g = t / GS, gl = t % GS;
    constexpr int U = 4;
    for (uint32_t w = w0 + g; w < w1; w += WG / GS) {
        const uint32_t s0 = hdr[(uint64_t)b * nW + w], s1 = hdr[(uint64_t)(b + 1) * nW + w];
        const uint4* reg4 = reinterpret_cast<const uint4*>(region + (uint64_t)w * rstride);  // (16-B aligned)
        for (uint32_t q = (s0 & ~3u) + 4 * gl; q < s1; q += 4 * GS * U) {
            uint4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = reg4[min((q + 4 * GS * u) / 4, (s1 - 1) / 4)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t j = q + 4 * GS * u + i;
                    if (j >= s0 && j < s1)
                        atomicAdd(&s_bins[xs[i] & (bs - 1u)], (1ull << 40) | (unsigned long long)(xs[i] >> bits));
                }
            }
        }
    }
    __syncthreads();
    bins_out(s_bins, bs, b, ntx, tx_acc);
}

__global__ __launch_bounds__(WG) void k_fold_totals(uint64_t* acc, uint64_t* reads, uint64_t* score, uint32_t ntx) {
    for (uint32_t t = blockIdx.x * WG + threadIdx.x; t < ntx; t += gridDim.x * WG) {
        const uint64_t a = acc[t];
        if (a) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&reads[t]), (unsigned long long)(a >> 40));
            atomicAdd(reinterpret_cast<unsigned long long*>(&score[t]), (unsigned long long)(a & ((1ull << 40) - 1)));
            acc[t] = 0;
        }
    }
}
#endif  // SKQ_PART == 0


// ---------------------------------------------------------------------------------------------
// launchers

#if SKQ_PART == 0
static bool use_count3(const ChainParams& p) { return p.ntx <= (1u << 22); }

bool count_bins(const ChainParams& p) { return use_count3(p) && p.nk <= (uint32_t)NK_FAST && p.bin_nb > 0; }

int launch_sketch(const SketchParams& p, void* stream) {
    if (p.n == 0) return 0;
    const dim3 grid((unsigned)((p.n + WG - 1) / WG));
    const size_t lds = sketch_lds_bytes(p.nk, p.tile_chunks, p.hcap, p.nthash != 0);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (lds > 160 * 1024) return -1;
    auto go = [&](auto kern) {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        launch_timed(kern, grid, dim3(WG), lds, s, p);
    };
    switch (p.hcap * 2 + (p.nthash ? 1 : 0)) {
    case 32: go(k_sketch<16, false>); break;
    case 64: go(k_sketch<32, false>); break;
    case 128: go(k_sketch<64, false>); break;
    case 33: go(k_sketch<16, true>); break;
    case 65: go(k_sketch<32, true>); break;
    case 129: go(k_sketch<64, true>); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_sketch_slow(const SketchParams& p, void* stream, unsigned grid) {
    if (p.n == 0) return 0;
    hipLaunchKernelGGL(k_sketch_slow, dim3(grid), dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_probe(const ChainParams& p, void* stream) {
    if (p.n == 0) return 0;
    const dim3 grid((unsigned)((p.n + WG - 1) / WG));
    launch_timed(k_probe, grid, dim3(WG), chain_lds_bytes(p.nk), reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_count(const ChainParams& p, void* stream) {
    if (p.n == 0) return 0;
    const dim3 grid((unsigned)((p.n + WG - 1) / WG));
    // k_count3 (32-bit sort keys) unless transcript ids need more than 22 bits
    if (use_count3(p)) {
        const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        auto go = [&](auto mode) {
            constexpr int M = decltype(mode)::value;
            switch (p.nk) {
            case 1: launch_timed(k_count3<1, M>, grid, dim3(WG), 0, st, p); break;
            case 2: launch_timed(k_count3<2, M>, grid, dim3(WG), 0, st, p); break;
            case 3: launch_timed(k_count3<3, M>, grid, dim3(WG), 0, st, p); break;
            case 4: launch_timed(k_count3<4, M>, grid, dim3(WG), 0, st, p); break;
            default: launch_timed(k_route_slow, grid, dim3(WG), 0, st, p); break;
            }
        };
        // wide tables, 2..4 k slots: the entry-parallel count
        if ((p.wide == 1 || p.wide == 3) && p.nk >= 2 && p.nk <= (uint32_t)NK_FAST && p.status && !p.present &&
            !p.hash_offs) {
            const bool cmp = p.wide == 3;
            switch (p.nk) {
            case 2:
                if (cmp) launch_timed(k_countw<2, true>, grid, dim3(WG), 0, st, p);
                else launch_timed(k_countw<2, false>, grid, dim3(WG), 0, st, p);
                break;
            case 3:
                if (cmp) launch_timed(k_countw<3, true>, grid, dim3(WG), 0, st, p);
                else launch_timed(k_countw<3, false>, grid, dim3(WG), 0, st, p);
                break;
            default:
                if (cmp) launch_timed(k_countw<4, true>, grid, dim3(WG), 0, st, p);
                else launch_timed(k_countw<4, false>, grid, dim3(WG), 0, st, p);
                break;
            }
            return hipGetLastError() == hipSuccess ? 0 : -2;
        }
        if (p.wide == 1) go(std::integral_constant<int, 1>{});
        else if (p.wide == 3) go(std::integral_constant<int, 3>{});
        else go(std::integral_constant<int, 0>{});
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    switch (p.nk) {
    case 1: launch_timed(k_count<1>, grid, dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p); break;
    case 2: launch_timed(k_count<2>, grid, dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p); break;
    case 3: launch_timed(k_count<3>, grid, dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p); break;
    case 4: launch_timed(k_count<4>, grid, dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p); break;
    default: launch_timed(k_route_slow, grid, dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_slow_wave(const SketchParams& p, const ChainParams& cp, uint32_t* ovf3, uint32_t* ovf4, void* stream) {
    if (cp.n == 0) return 0;
    if (cp.wide != 1 && cp.wide != 3) return -4;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // a 64-lane workgroup per listed read, grid-stride (the list length is on the device); 16
    // per CU fit (LDS ~9 KB, < 100 VGPRs)
    // (a small batch's few slow reads need fewer workgroups: an empty list still dispatches all;
    // at cfg3 a quarter or an eighth of the grid measured 0.5-1 % slower, profiles/r6_slow_wave_grid_ab.log)
    const dim3 grid((unsigned)std::min<uint64_t>(SW_GRID, std::max<uint64_t>(256, cp.n / 2048))), blk(64);
    const bool cmp = cp.wide == 3;
    switch (cp.nk) {
    case 1:
        if (cmp) hipLaunchKernelGGL((k_slow_wave<1, true>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        else hipLaunchKernelGGL((k_slow_wave<1, false>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        break;
    case 2:
        if (cmp) hipLaunchKernelGGL((k_slow_wave<2, true>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        else hipLaunchKernelGGL((k_slow_wave<2, false>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        break;
    case 3:
        if (cmp) hipLaunchKernelGGL((k_slow_wave<3, true>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        else hipLaunchKernelGGL((k_slow_wave<3, false>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        break;
    case 4:
        if (cmp) hipLaunchKernelGGL((k_slow_wave<4, true>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        else hipLaunchKernelGGL((k_slow_wave<4, false>), grid, blk, 0, st, p, cp, ovf3, ovf4);
        break;
    default: return -4;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_chain_slow(const ChainParams& p, void* stream, unsigned grid) {
    if (p.n == 0) return 0;
    hipLaunchKernelGGL(k_chain_slow, dim3(grid), dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_general_slow(const SketchParams& sp, const ChainParams& p, void* stream, unsigned grid, uint32_t* zero_next) {
    if (p.n == 0) return 0;
    hipLaunchKernelGGL(k_general_slow, dim3(grid), dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), sp, p, zero_next);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// wide entry for key keys[j]: [n, t0..t6] (n <= 7) or [0x80000000 | list offset, t0..t6]
__global__ void k_wdir_scatter(uint32_t* wdir, const uint32_t* keys, const uint32_t* vals, const uint32_t* lists,
                               uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t off = vals[j];
    const uint32_t len = lists[off];
    uint32_t e[8];
    e[0] = len <= 7 ? len : (0x80000000u | off);
#pragma unroll
    for (int q = 0; q < 7; ++q) e[q + 1] = (uint32_t)q < len ? lists[off + 1 + q] : 0u;
    uint4* d = reinterpret_cast<uint4*>(wdir + (uint64_t)keys[j] * 8);
    d[0] = make_uint4(e[0], e[1], e[2], e[3]);
    d[1] = make_uint4(e[4], e[5], e[6], e[7]);
}

__global__ void k_dir_scatter(uint32_t* dir, const uint32_t* keys, const uint32_t* vals, uint64_t n) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x)
        dir[keys[j]] = vals[j];
}

int launch_dir_scatter(uint32_t* dir, const uint32_t* keys, const uint32_t* vals, uint64_t n, void* stream) {
    if (n == 0) return 0;
    const unsigned grid = (unsigned)std::min<uint64_t>((n + WG - 1) / WG, 4096);
    hipLaunchKernelGGL(k_dir_scatter, dim3(grid), dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), dir, keys, vals, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif  // SKQ_PART == 0





#if SKQ_PART == 0
int launch_wdir_scatter(uint32_t* wdir, const uint32_t* keys, const uint32_t* vals, const uint32_t* lists,
                        uint64_t n, void* stream) {
    if (n == 0) return 0;
    const unsigned grid = (unsigned)((n + WG - 1) / WG);
    hipLaunchKernelGGL(k_wdir_scatter, dim3(grid), dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), wdir, keys,
                       vals, lists, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_fold_totals(uint64_t* acc, uint64_t* reads, uint64_t* score, uint32_t ntx, void* stream) {
    if (ntx == 0) return 0;
    const unsigned grid = (unsigned)std::min<uint32_t>((ntx + WG - 1) / WG, 1024);
    hipLaunchKernelGGL(k_fold_totals, dim3(grid), dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), acc, reads,
                       score, ntx);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_bin(const ChainParams& p, int binned, void* stream, bool beside_map) {
    if (p.n == 0) return 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint32_t nW = (uint32_t)((p.n + WG - 1) / WG);
    const uint32_t bits = p.bin_bits, nb = p.bin_nb;
    uint32_t* hdr = p.bin_hdr;
    const uint32_t* region = p.bin_region;
    if (nb > (uint32_t)WG) return -1;
    if (!binned && p.cpack && p.ntx <= TOT_SMALL_TX && p.cand_wtot) {  // (small transcript sets: no binning)
        const uint32_t nwaves = (uint32_t)((p.n + 63) / 64);
        // between maps: 1024-thread workgroups, 64 chunks of the batch's map waves, ranges of <= 5120
        // ids (40 KiB of bins: two ranges at cfg2's 10k). Swept at cfg2 (profiles/r6_tot_small_sweep.log):
        // 64 chunks x 5000 ids 13.9 us, x 2560 16.2, x 10000 19+; 128 chunks (twice the flush atomics)
        // 17-20 us; 256-thread workgroups 19-26 us (one wave per SIMD: each wave waits on its own loads)
        const uint32_t nr0 = (p.ntx + 5119) / 5120;
        const uint32_t range = beside_map ? TOT_RANGE_TX : (p.ntx + nr0 - 1) / nr0;
        const uint32_t chunks = 64;
        const uint32_t nr = (p.ntx + range - 1) / range;
        const uint32_t per = std::min<uint32_t>(1024, std::max<uint32_t>(16, (nwaves + chunks - 1) / chunks));
        const uint32_t nc = (nwaves + per - 1) / per;
        const size_t lds = (size_t)range * 8 + (size_t)per * 4;
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_tot_small), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds);
        hipLaunchKernelGGL(k_tot_small, dim3(nc * nr), dim3(beside_map ? WG : TOT_WG), lds, st, p, nwaves, per, nr, range);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    // the fused map's packed candidates: one binned region per four map workgroups (k_bin_packed<4096,
    // 4>), summed by k_bin_sum4 — against one per map workgroup, cfg3 9.50 -> 9.95 G reads/s on one
    // box; two, three or eight per region, unstaged stores and 2^10-2^11-id buckets measured slower,
    // the forms small enough in LDS to run beside five map workgroups per CU too: their overlap
    // slows the map more than it saves (profiles/r6_bin_group_ab.log)
    const bool grouped = !binned && p.cpack && nb > 4;
    const uint32_t nWb = grouped ? (nW + 3) / 4 : nW;  // (binned regions)
    const uint32_t rstride = WG * CCAP;                 // (words per binned region)
    if (!binned) {
        if (grouped)
            hipLaunchKernelGGL((k_bin_packed<WG * CCAP, 4>), dim3(nWb), dim3(WG), 0, st, p, bits, nb, nWb, p.bin_hdr,
                               p.bin_region);
        else if (p.cpack && nb)
            hipLaunchKernelGGL((k_bin_packed<WG * CCAP, 1>), dim3(nW), dim3(WG), 0, st, p, bits, nb, nW, p.bin_hdr,
                               p.bin_region);
        else
            hipLaunchKernelGGL(k_bin, dim3(nW), dim3(WG), 0, st, p, bits, nb, nW, p.bin_hdr, p.bin_region);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    if (nb == 0) return 0;
    // chunks * nb ~ 512 workgroups, 1024 for many buckets (their bins are 32 KiB: four workgroups
    // per CU; profiles/r5_totals_sweep.log)
    const uint32_t wgs = nb >= 16 ? 1024 : 512;
    const uint32_t chunks = std::max<uint32_t>(1, std::min<uint32_t>(nWb, wgs / nb));
    const uint32_t chunk = (nWb + chunks - 1) / chunks;
    const size_t lds = (size_t)8 << bits;
    if (grouped) {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_sum4<4>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_bin_sum4<4>, dim3((nWb + chunk - 1) / chunk, nb), dim3(WG), lds, st, p.tx_acc, p.ntx,
                           bits, nWb, chunk, hdr, region, rstride);
    } else if (nb <= 4) {  // few buckets: long segments per region, a 16-lane group walks each
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_sum_g<16>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_bin_sum_g<16>, dim3((nW + chunk - 1) / chunk, nb), dim3(WG), lds, st, p.tx_acc, p.ntx,
                           bits, nW, chunk, hdr, region, (uint32_t)(WG * CCAP));
    } else {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_sum), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds);
        hipLaunchKernelGGL(k_bin_sum, dim3((nW + chunk - 1) / chunk, nb), dim3(WG), lds, st, p.tx_acc, p.ntx, bits,
                           nb, nW, chunk, hdr, region, (uint32_t)(WG * CCAP));
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
#endif  // SKQ_PART == 0


}  // namespace skq
