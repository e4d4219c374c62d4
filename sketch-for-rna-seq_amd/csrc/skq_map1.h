// skq_map1.h — k_map1, the fused quant kernel (sketch + index probe + chain + emit), for the
// two map translation units (skq_map1.hip: one k; skq_map1_pass.hip: the multi-k passes). It
// follows skq_kernels.hip (the device helpers it uses), which each of them includes first.
#pragma once

namespace skq {

// k_map1 LDS: static, at LDS address 0, the HCAP + 2 raw rows (Map1Static: row 0 the sink of
// windows past the capacity, then the retained windows from the last row down, so a row's LDS
// address is the hashing loop's own counter) and the roll terms; dynamic, per wave max(staged
// codes, one pass of the entry list: MAP_P hashes and their owning lanes)
// (the per-chunk bad bits sit in the wave's columns of the last raw row, dead until hashing starts)
// (MAP_P: 8 per read; at 384 — the mean of cfg3's ~6.0 distinct hashes per read x 64 — half of
// the waves listed their hashes in two passes, the second one a dependent reload and gather
// round; profiles/r3_map1_writes.log)
constexpr uint32_t MAP_P = 512;
// threads per k_map1 workgroup (one k): 64 (one wave: a workgroup's LDS is released when ITS wave
// ends) or WG (four waves; the default)
#ifndef SKQ_MAP_WG
#define SKQ_MAP_WG 256
#endif
constexpr int MAP_MW = SKQ_MAP_WG;
// threads per workgroup of the multi-k passes (k_map1 PASS, k_mapk): one wave, whose LDS is
// released when it ends (cfg5 4.6 % faster than four-wave workgroups; one k: 3.8 % slower,
// profiles/r5_wg64_ab.log)
#ifndef SKQ_PASS_WG
#define SKQ_PASS_WG 64
#endif
constexpr int PASS_MW = SKQ_PASS_WG;
// A wave's packed output (lane-ordered runs: this lane's words from its exclusive offset `off`
// of the wave's `tot`, word j present when has(j), valued val(j)) to 16-B aligned g through the
// wave's LDS region in chunks of MAP1_OUT_CH words, each written back as 16-B coalesced stores: a
// store of 64 lanes then touches 8 lines, where one store per word rank touched up to 64 (the
// texture addresser works per line: the chained tables' coalesced loads showed it, round 4)
constexpr uint32_t MAP1_OUT_CH = 640;  // (2560 B: below the per-read flags)
#ifndef SKQ_OUT_LDS
#define SKQ_OUT_LDS 0  // (1: through LDS; measured: wide 3 % slower, chained the same, profiles/r4_out_lds_ab.log)
#endif
// (MONO: has(j) implies has(j - 1) in every lane, so the words stop at the wave's longest run)
template <int N, bool MONO = false, typename Has, typename Val>
__device__ __forceinline__ void wave_out_packed(uint32_t* g, uint32_t off, uint32_t tot, uint32_t* s_buf, uint32_t lane,
                                                Has has, Val val) {
    if (!SKQ_OUT_LDS) {
        uint32_t e = off;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (MONO && !__any(has(j))) break;  // (uniform)
            if (has(j)) g[e++] = val(j);
        }
        return;
    }
    for (uint32_t c0 = 0; c0 < tot; c0 += MAP1_OUT_CH) {  // (uniform)
        uint32_t e = off;
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (has(j)) {
                if (e - c0 < MAP1_OUT_CH) s_buf[e - c0] = val(j);
                ++e;
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nq = (min(MAP1_OUT_CH, tot - c0) + 3) / 4;
        uint4* g4 = reinterpret_cast<uint4*>(g + c0);
        const uint4* s4 = reinterpret_cast<const uint4*>(s_buf);
        for (uint32_t q = lane; q < nq; q += 64) g4[q] = s4[q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// The hashing loop's slot counter is the LDS byte address of the lane's next raw-row store (the
// raw rows sit at LDS address 0, Map1Static). A lane past row 0 moves it below 0: the plain subtract
// wraps it past the LDS allocation, and the hardware drops a DS store there (tools/micro/lds_oob,
// profiles/r5_lds_oob.log). That holds ONLY for DS stores (address_space(3), 32-bit addresses):
// through a generic or global pointer such an address faults, as round 5's k_sketch_server did
// with a pointer formed below an LDS array. So the counter is only ever used through
// lds_slot_store, whose pointer is the 32-bit LDS kind (the static_assert), and the debug build
// (make debuglds: -DSKQ_DEBUG_LDS, tests/test_debug_lds_gpu.py) clamps it at 0 instead — lane 0's
// sink slot, which nothing reads; a read past its capacity still counts HCAP + 1 windows and goes slow.
#ifndef SKQ_DEBUG_LDS
#define SKQ_DEBUG_LDS 0
#endif
typedef __attribute__((address_space(3))) uint32_t lds_u32;
#if defined(__HIP_DEVICE_COMPILE__)
static_assert(sizeof(lds_u32*) == 4, "the slot counter is a 32-bit LDS (DS) address, never a generic pointer");
#endif
__device__ __forceinline__ void lds_slot_store(uint32_t addr, uint32_t v) { *(lds_u32*)(size_t)addr = v; }
__device__ __forceinline__ uint32_t lds_slot_next(uint32_t d, uint32_t adv) {
#if SKQ_DEBUG_LDS
    return __builtin_elementwise_sub_sat(d, adv);
#else
    return d - adv;  // (may wrap below LDS address 0: see above)
#endif
}

template <int HCAP, int MW = WG>
struct Map1Static {
    uint32_t raw[(HCAP + 2) * MW];  // (first: at LDS address 0, the kernel's only static LDS)
    uint2 tab[16 + 4];              // the roll terms, then the seeds
#if SKQ_HASH_PAIR
    uint2 tb[16];                   // the roll terms with bit 32 in bit 0 of .y (hashing loop, below)
#endif
};
// the per-read overflow flags' place in the wave's region: after the list — hashes, then owning
// lanes (u8; compact tables: u32 slot | lane << 26) (tab: 0 wide, 2 compact, 3 chained over
// wide, 4 chained over compact). (Round 3 measured 6 workgroups per CU against 5 with the list packed
// tighter: no change, profiles/r3_ingest_sweep.log.)
inline size_t map1_flag_at(int tab, uint32_t hcap) {
    if (tab == 2 || tab == 4) return (size_t)MAP_P * 8;
    return ((size_t)MAP_P * 5 + 15) & ~(size_t)15;
}
inline size_t map1_wave_bytes(uint32_t wc, int tab, uint32_t hcap) {
    const size_t a = sketch_codes_bytes(wc);
    const size_t b = map1_flag_at(tab, hcap) + 64 * 4;
    const size_t c = (size_t)(WG + 1) * 4;
    const size_t m = a > b ? a : b;
    return ((m > c ? m : c) + 15) & ~(size_t)15;
}

// sets p.map_wave_bytes / p.map_flag_at; returns the launch's dynamic LDS bytes (mw: threads per
// workgroup; the raw rows are static)
inline size_t map1_layout(SketchParams& p, int tab, uint32_t hcap, uint32_t mw = WG) {
    p.map_wave_bytes = (uint32_t)map1_wave_bytes(p.tile_chunks, tab, hcap);
    p.map_flag_at = (uint32_t)map1_flag_at(tab, hcap);
    return (mw / 64) * (size_t)p.map_wave_bytes;
}

// Fused map kernel (quant mode, one k slot, wide tables): k_sketch's staging and hashing, then
// the retained hashes go straight from registers to the pair-cooperative wide-table count
// (wide_chunk), the filter and the candidates (k_bin_packed bins them for the totals after it). The count tables
// overlay LDS the hashing no longer needs: the transcript table the raw slots ([slot][WG], this
// lane's own), the parked list the wave's staged codes (all of the wave's lanes have left the
// hashing loop before any counts). Reads k_sketch would hand to the slow path are listed for
// both slow paths (k_sketch_slow, then k_chain_slow). No early exits: pairs gather together.
// development phase clocks (ChainParams::stamps): 8 u64 per wave, written by lane 0
#define MAP1_STAMP(i)                                                                           \
    do {                                                                                        \
        if (cp.stamps && lane == 0)                                                             \
            cp.stamps[((uint64_t)blockIdx.x * (MW / 64) + wv) * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
    } while (0)

// TAB: 0 = wide tables, 2 = compact tables, 3 = chained tables over wide ones, 4 = chained tables at the
// compact tables' slots (over compact ones). PASS: one k slot (p.kslot) of a
// multi-k map: the entries of the read's count table at that k that meet that k's need go out to
// cp.ktab / cp.kcnt with the need (a transcript short of one k slot's need fails the multi-k
// filter whatever the other k slots hold), with no candidates or binning; a read any pass lists
// for the slow path is listed once (pflag), and a read an earlier pass found sketch-slow is
// skipped. FINAL (the last k slot's pass): the earlier passes' entries are merged in registers with
// this pass's table (matched only, when this k slot filters), then filtered, ordered, written and
// binned as in the one-k map.
// (the kernel's only static LDS, one instance for every body a kernel inlines: k_mapk runs several)
template <int HCAP, int MW>
__device__ __forceinline__ Map1Static<HCAP, MW>& map1_static() {
    __shared__ __attribute__((aligned(16))) Map1Static<HCAP, MW> s_st;
    return s_st;
}

// the work of one k slot ks over the workgroup's reads (k_map1: one launch per k slot; k_mapk: the
// k slots one after another in one launch)
// (FINAL: a constant in the k_map1 instantiations, which fold it; k_mapk passes it at run time, so
// its loop over the k slots holds one copy of the body's code)
template <int HCAP, int MB, int TAB, bool PASS, int MW>
__device__ __forceinline__ void map1_body(const SketchParams& p, const ChainParams& cp, const uint32_t ks, const bool FINAL) {
    static_assert(MW == WG || MW == 64 || MW == 128, "a workgroup of 256 threads (4 waves), of two or of one");
    // TAB 4: chained entries at the compact tables' slots (one per present key, not per possible
    // key: 0.6 GB at cfg3 instead of 27.5 GB), the misses through the compact entries
    constexpr bool CMP = TAB == 2 || TAB == 4, CHN = TAB == 3 || TAB == 4, CCH = TAB == 4;
    static_assert(!CHN || HCAP <= 32, "hit bits");
    static_assert(!CCH || SKQ_CHN_COALESCED, "compact chained entries: the coalesced hand-over (word 28)");
    static_assert(HCAP >= TS && HCAP >= CCAP, "the raw rows hold the count tables and the binned region");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int tid = threadIdx.x;
    // (opaque to the optimiser: k_mapk's loop over k slots would otherwise hoist every
    // thread-derived address out of the loop and keep them live across the whole body)
    asm volatile("" : "+v"(tid));
    const uint32_t lane = tid & 63, wv = tid >> 6;
    MAP1_STAMP(0);
    const uint32_t wc = p.tile_chunks;  // chunks per wave
    const size_t wave_bytes = p.map_wave_bytes;
    // (static LDS: the raw rows' and the roll terms' addresses fold into the instructions' offsets)
    Map1Static<HCAP, MW>& s_st = map1_static<HCAP, MW>();
    uint2* s_tab = s_st.tab;
    const uint2* s_seed = s_tab + 16;
    unsigned char* s_wave = smem + wv * wave_bytes;
    uint32_t* s_codes = reinterpret_cast<uint32_t*>(s_wave);
    // raw rows: row 0 the sink, retained window i of the read (position order) in row HCAP + 1 - i;
    // after the hashing, rows 1..TS hold the count tables (s_rows)
    uint32_t* s_raw = s_st.raw;
    uint32_t* s_rows = s_raw + MW;
    uint64_t* s_badw = reinterpret_cast<uint64_t*>(s_raw + (HCAP + 1) * MW + wv * 64);  // (the wave's columns, last row)
    for (uint32_t e = tid; e < 16 + 4; e += MW) {  // k slot ks's roll terms, then the seeds
        const uint64_t v = e < 16 ? p.rolltab[ks * 16 + e] : p.rolltab[p.nk * 16 + (e - 16)];
        s_tab[e] = make_uint2((uint32_t)v, (uint32_t)(v >> 32) << 31);
    }
#if SKQ_HASH_PAIR
    // the roll terms again, bit 32 in bit 0 (the hashing loop folds it into the next window's XOR)
    if (tid < 16) {
        const uint64_t v = p.rolltab[ks * 16 + tid];
        s_st.tb[tid] = make_uint2((uint32_t)v, (uint32_t)(v >> 32) & 1u);
    }
#endif
    __syncthreads();

    const uint64_t r0 = (uint64_t)blockIdx.x * MW + wv * 64;  // this wave's first read
    const uint32_t nr = r0 < p.n ? (uint32_t)min((uint64_t)64, p.n - r0) : 0u;  // wave-uniform
    const uintptr_t base = reinterpret_cast<uintptr_t>(p.reads);
    const uintptr_t abase = base & ~(uintptr_t)15;
    const uint64_t delta = base - abase;
    uint64_t c0 = 0;
    uint32_t nch = 0;
    if (nr) {
        uint64_t s0, l0, sl, ll;
        read_extent(p.offs, p.fixed_len, r0, s0, l0);
        read_extent(p.offs, p.fixed_len, r0 + nr - 1, sl, ll);
        c0 = (s0 + delta) >> 4;
        const uint64_t c1 = (sl + ll + delta + 15) >> 4;
        nch = (uint32_t)min((uint64_t)wc, c1 - c0);
        const uint4* src = reinterpret_cast<const uint4*>(p.reads - delta) + c0;
        constexpr uint32_t SU = 10;
        // multi-k passes (SketchParams::stash): the first stores the wave's staged image, the
        // later ones stage from it (38 B per 150-bp read instead of the 150 B of bases)
        uint32_t* sw = PASS && p.stash ? p.stash + (r0 >> 6) * p.stash_stride : nullptr;
        const uint32_t sbad = (wc + 1) & ~1u;  // (the bad bits' first word)
        if (PASS && sw && ks > 0) {
            for (uint32_t cb = lane; cb < nch; cb += SU * 64) {
                uint32_t x[SU];
#pragma unroll
                for (uint32_t u = 0; u < SU; ++u) x[u] = __builtin_nontemporal_load(sw + min(cb + u * 64, nch - 1));
#pragma unroll
                for (uint32_t u = 0; u < SU; ++u)
                    if (cb + u * 64 < nch) s_codes[cb + u * 64] = x[u];
            }
            if (lane < (nch + 63) / 64)
                s_badw[lane] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(sw + sbad) + lane);
        }
        for (uint32_t cb = lane; cb < nch && !(PASS && sw && ks > 0) && !(cp.ablate & 16u); cb += SU * 64) {
            uint4 vv[SU];
#pragma unroll
            for (uint32_t u = 0; u < SU; ++u) {
                // (non-temporal: the streamed bases do not evict the entries' lines; +2 %)
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + min(cb + u * 64, nch - 1)));
                vv[u] = make_uint4(x.x, x.y, x.z, x.w);
            }
#pragma unroll
            for (uint32_t u = 0; u < SU; ++u) {
                const uint32_t c = cb + u * 64;
                const uint4 v = vv[u];
                const uint32_t cs = c < nch ? c : wc + 1;
                const uint32_t ta = (v.x >> 1) & 0x03030303u, tb = (v.y >> 1) & 0x03030303u;
                const uint32_t tc = (v.z >> 1) & 0x03030303u, td = (v.w >> 1) & 0x03030303u;
                constexpr uint32_t W4 = 0x40100401u;
                const uint32_t code = __builtin_amdgcn_udot4(ta, W4, 0u, false) |
                                      (__builtin_amdgcn_udot4(tb, W4, 0u, false) << 8) |
                                      (__builtin_amdgcn_udot4(tc, W4, 0u, false) << 16) |
                                      (__builtin_amdgcn_udot4(td, W4, 0u, false) << 24);
                constexpr uint32_t GTCA = 0x47544341u;
                const uint32_t x = (__builtin_amdgcn_perm(0u, GTCA, ta) ^ v.x) | (__builtin_amdgcn_perm(0u, GTCA, tb) ^ v.y) |
                                   (__builtin_amdgcn_perm(0u, GTCA, tc) ^ v.z) | (__builtin_amdgcn_perm(0u, GTCA, td) ^ v.w);
                s_codes[cs] = code;
                const uint64_t wbits = __ballot(x != 0);
                if (lane == 0 && c < nch) s_badw[c >> 6] = wbits;
                if (PASS && sw && c < nch) {  // (first pass: the image for the later ones)
                    __builtin_nontemporal_store(code, sw + c);
                    if (lane == 0) __builtin_nontemporal_store(wbits, reinterpret_cast<uint64_t*>(sw + sbad) + (c >> 6));
                }
            }
        }
        if (lane == 0) s_codes[nch] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    MAP1_STAMP(1);

    const bool live = lane < nr;
    const uint64_t r = live ? r0 + lane : 0;
    uint64_t start = 0, len = 0;
    if (live) read_extent(p.offs, p.fixed_len, r, start, len);
    const uint64_t q0 = start + delta - c0 * 16;
    bool slow = live && (len > (uint64_t)LFAST || q0 + len > (uint64_t)nch * 16);
    uint8_t st = SKQ_READ_OK;
    if (live && !slow) {
        // is_valid_sequence (src/data_io.cpp:17-34), as in k_sketch
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

    // pass mode, after the first pass: listed already (pf_prev), sketch-slow already (sk_prev)
    const uint8_t pf_prev = (PASS && ks > 0 && live) ? p.pflag[r] : (uint8_t)0;
    const bool sk_prev = PASS && ks > 0 && live && (p.status[r] & ST_SLOW1);
    uint32_t v[HCAP];
#pragma unroll
    for (int j = 0; j < HCAP; ++j) v[j] = 0xFFFFFFFFu;
    uint64_t keepm = 0;  // bit j: v[j] is a distinct retained hash
    uint32_t nraw_out = 0;  // retained windows in the raw rows (position order), fast reads
    const bool hashing = live && !slow && !sk_prev && st == SKQ_READ_OK;
    // chained tables: the read's first retained window (position order) is its query; its entry is
    // requested as soon as the hashing loop is done, so the sort and the hash writes below run
    // while it is in flight
    // (the request is issued by every lane outside any divergent branch — lanes without a query
    // read entry 0 and drop it — so no copy at a branch join waits for it)
    uint32_t cq = 0;
    bool has_q = false;
    // (clang vectors, not uint4: copies of the HIP vector struct kept this array in scratch)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 ce[CHN ? (SKQ_CHN_COALESCED ? 8 : 7) : 1];
    uint32_t nraw = 0;  // retained windows (position order) in the raw rows
    if (hashing) {
        const uint32_t T = p.threshold;
        const uint32_t L = (uint32_t)len;
        const uint32_t k = p.ks[ks];
        auto codes16 = [&](uint32_t q) -> uint32_t {
            const uint32_t d = q >> 4;
            return __builtin_amdgcn_alignbit(s_codes[d + 1], s_codes[d], (q & 15) * 2);
        };
        // first window (NtHash::init): the seeds of 16 bases read before their serial rolls
        uint32_t hlo = 0, hhi = 0;
        for (uint32_t b = 0; b < k; b += 16) {
            const uint32_t w = codes16((uint32_t)q0 + b);
            uint2 e[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) e[j] = s_seed[(w >> (2 * j)) & 3u];
            if (b + 16 <= k) {  // (uniform)
#pragma unroll
                for (int j = 0; j < 16; ++j) roll33b(hlo, hhi, e[j]);
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (b + j < k) roll33b(hlo, hhi, e[j]);
            }
        }
        s_raw[(HCAP + 1) * MW + tid] = hlo;
        const uint32_t nw = L - k + 1;
        const uint32_t qin = (uint32_t)q0 + k, qout = (uint32_t)q0;
        // windows 1..nw-1, 16 per block (in-base at w + k - 1, out-base at w - 1). A window's roll
        // term sits at byte (in << 5 | out << 3) of s_tab: with A the in-bases' 2-bit codes
        // shifted up by 2 and B the out-bases', the nibbles of ce = A:B (even windows) and
        // co = B:A (odd windows) hold (in, out) pairs, so a term's offset is one shift and one
        // mask. Every window's value is stored at the lane's write row, which a retained window
        // (src/sketch.cpp:33-35) moves down a row: retained window i in row HCAP + 1 - i, row 1 the
        // (HCAP + 1)-th (the read then goes slow), row 0 the sink of any past it. The lane's slot is
        // kept as its LDS offset d from the raw rows (at LDS address 0: the offset is the store's
        // address), moved by a saturating subtract, so no compare or clamp sits in the loop: a lane
        // past row 0 lands at offset 0, lane 0's sink slot, which nothing reads (lds_slot_next). For T < 2^31 the
        // test h <= T is bit 31 of ~((T - h) | h). Every operation in the loop but the rotate is a
        // full-rate VALU form (tools/micro/valu_mix: compares, min/max and the three-operand
        // integer forms issue at half rate).
        const uint32_t rbase = (uint32_t)(size_t)(lds_u32*)s_raw;  // (0: Map1Static is the only static LDS)
        constexpr uint32_t ROW = (uint32_t)MW * 4u;
        constexpr uint32_t ROW_SH = MW == 256 ? 21u : MW == 128 ? 22u : 23u;  // (2^31 >> ROW_SH == ROW)
        static_assert((0x80000000u >> ROW_SH) == ROW, "row stride");
        const uint32_t d0 = (uint32_t)tid * 4u + (uint32_t)(HCAP + 1) * ROW;
        uint32_t d = d0 - (hlo <= T ? ROW : 0u);
#if SKQ_HASH_PAIR
        // Windows 1..nw-1 in blocks of 16, two VALU operations per roll. With x_w the 33-bit lane
        // of window w (lo_w its low 32 bits) and t_w its roll term (in, out bases), the roll
        // x_w = rot33(x_{w-1}) ^ t_w gives bit 32 of x_{w-1} as (lo_{w-2} >> 31) ^ bit 32 of
        // t_{w-1}, so
        //     lo_w = alignbit(lo_{w-1}, lo_{w-2}, 31) ^ lo(t_w) ^ bit32(t_{w-1}),
        // one funnel shift and one three-way XOR (v_bitop3), bit 32 of each term kept in bit 0 of
        // its table entry's second word. Window 1's "previous" word is window 0's high lane (hhi,
        // bit 31) and its previous term none. The terms stay a 16-entry table read at the (in,
        // out) nibble's offset: 64 lanes hit at most 16 distinct 8-B entries, so a read is a
        // broadcast, never a bank conflict (a 256-entry table of pair terms, one XOR fewer, measured
        // 3 % slower: random reads of 1 KB conflict). The nibbles: ex (even windows) and ox (odd)
        // from the in- and out-base codes, each offset one byte select of four masked words. The
        // slot counter moves by a plain subtract: a lane past row 0 stores below LDS address 0,
        // which wraps past the allocation, and such stores are dropped (tools/micro/lds_oob,
        // profiles/r5_lds_oob.log).
        uint32_t lprev = hhi, yprev = 0;
        const uint32_t* pa = s_codes + (qin >> 4);
        const uint32_t* pb = s_codes + (qout >> 4);
        const uint32_t sa = (qin & 15u) * 2u, sb = (qout & 15u) * 2u;
        const unsigned char* tbb = reinterpret_cast<const unsigned char*>(s_st.tb);
        auto bfi = [](uint32_t m, uint32_t x, uint32_t y) {  // (x & m) | (y & ~m), one v_bfi_b32
            uint32_t r;
            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(y));
            return r;
        };
        auto block = [&](uint32_t bi, uint32_t jn, auto full, auto small) {
            const uint32_t A = __builtin_amdgcn_alignbit(pa[bi + 1], pa[bi], sa);
            const uint32_t B = __builtin_amdgcn_alignbit(pb[bi + 1], pb[bi], sb);
            // nibble m of ex = (in << 2 | out) of window 2m, of ox of window 2m + 1
            const uint32_t ex = bfi(0xCCCCCCCCu, A << 2, B);
            const uint32_t ox = bfi(0xCCCCCCCCu, A, B >> 2);
            // byte b of word c: window 4b + c's nibble times 8 (its term's offset)
            const uint32_t wq[4] = {(ex << 3) & 0x78787878u, (ox << 3) & 0x78787878u, (ex >> 1) & 0x78787878u,
                                    (ox >> 1) & 0x78787878u};
            uint2 e[16];
            static_for<16>([&](auto jc) {
                constexpr int j = decltype(jc)::value, b = j >> 2;
                const uint32_t x = wq[j & 3];
                uint32_t o;
                if constexpr (b == 0) {
                    o = x & 0xFFu;
                } else if constexpr (b == 1) {
                    asm("v_mov_b32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(o) : "v"(x));
                } else if constexpr (b == 2) {
                    asm("v_mov_b32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(o) : "v"(x));
                } else {
                    o = x >> 24;
                }
                e[j] = *reinterpret_cast<const uint2*>(tbb + o);
            });
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t h = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(hlo, lprev, 31), e[j].x, yprev, 0x96);
                lprev = hlo;
                hlo = h;
                yprev = e[j].y;
                lds_slot_store(rbase + d, h);
                uint32_t adv = decltype(small)::value ? (uint32_t)__builtin_amdgcn_bitop3_b32(T - h, h, 0x80000000u, 0x02) >> ROW_SH
                                                      : (h <= T ? ROW : 0u);
                if (!decltype(full)::value) adv &= (uint32_t)((int)(j - (int)jn) >> 31);  // (windows past the read)
                d = lds_slot_next(d, adv);
            }
        };
        uint32_t w0 = 1, bi = 0;
        if (T < 0x80000000u) {  // (uniform)
            for (; w0 + 16 <= nw && !(cp.ablate & 32u); w0 += 16, ++bi) block(bi, 16u, std::true_type{}, std::true_type{});
            if (w0 < nw && !(cp.ablate & 32u)) block(bi, nw - w0, std::false_type{}, std::true_type{});
        } else {
            for (; w0 + 16 <= nw; w0 += 16, ++bi) block(bi, 16u, std::true_type{}, std::false_type{});
            if (w0 < nw) block(bi, nw - w0, std::false_type{}, std::false_type{});
        }
#else
        const unsigned char* tabb = reinterpret_cast<const unsigned char*>(s_tab);
        auto block = [&](uint32_t w0, uint32_t jn, auto full, auto small) {
            const uint32_t A = codes16(qin + w0 - 1), B = codes16(qout + w0 - 1);
            const uint32_t A2 = A << 2;
            const uint32_t ce = (A2 & 0xCCCCCCCCu) | (B & 0x33333333u);
            const uint32_t co = (A2 & 0x33333333u) | (B & 0xCCCCCCCCu);
            uint32_t off[16];
#if SKQ_HASH_SDWA
            // the 15 offsets as bytes of four masked words (window 4b + c in byte b of word c),
            // each taken by one byte-select move instead of a shift and a mask
            const uint32_t wq[4] = {(ce << 3) & 0x78787878u, (co << 1) & 0x78787878u, (ce >> 1) & 0x78787878u,
                                    (co >> 3) & 0x78787878u};
            static_for<15>([&](auto jc) {
                constexpr int j = decltype(jc)::value, b = j >> 2;
                const uint32_t x = wq[j & 3];
                uint32_t r;
                if constexpr (b == 0) {
                    r = x & 0xFFu;
                } else if constexpr (b == 1) {
                    asm("v_mov_b32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(r) : "v"(x));
                } else if constexpr (b == 2) {
                    asm("v_mov_b32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2" : "=v"(r) : "v"(x));
                } else {
                    r = x >> 24;
                }
                off[j] = r;
            });
#else
            off[0] = (ce << 3) & 0x78u;
            off[1] = (co << 1) & 0x78u;
#pragma unroll
            for (int j = 2; j < 15; ++j) off[j] = ((j & 1 ? co : ce) >> (2 * j - 3)) & 0x78u;
#endif
            off[15] = ((A >> 30) << 5) | ((B >> 30) << 3);
            uint2 e[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) e[j] = *reinterpret_cast<const uint2*>(tabb + off[j]);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                roll33b(hlo, hhi, e[j]);
                lds_slot_store(rbase + d, hlo);
                // (small: ~((T - h) | h) & 2^31 as one bitop3, then the shift down to ROW)
                uint32_t adv = decltype(small)::value ? (uint32_t)__builtin_amdgcn_bitop3_b32(T - hlo, hlo, 0x80000000u, 0x02) >> ROW_SH
                                                      : (hlo <= T ? ROW : 0u);
                if (!decltype(full)::value) adv &= (uint32_t)((int)(j - (int)jn) >> 31);  // (windows past the read)
                d = __builtin_elementwise_sub_sat(d, adv);
            }
        };
        uint32_t w0 = 1;
        if (T < 0x80000000u) {  // (uniform)
            for (; w0 + 16 <= nw && !(cp.ablate & 32u); w0 += 16) block(w0, 16u, std::true_type{}, std::true_type{});
            if (w0 < nw && !(cp.ablate & 32u)) block(w0, nw - w0, std::false_type{}, std::true_type{});
        } else {
            for (; w0 + 16 <= nw; w0 += 16) block(w0, 16u, std::true_type{}, std::false_type{});
            if (w0 < nw) block(w0, nw - w0, std::false_type{}, std::false_type{});
        }
#endif
        nraw = (d0 - d) / ROW;  // (> HCAP: more than HCAP retained; exact, d0 - d < 2^32)
    }
    uint32_t qslot = 0;  // the query's entry (TAB 4: its compact slot, whose entry names its key)
    if constexpr (CHN) {
        cq = s_raw[(HCAP + 1) * MW + tid];  // (the first retained window)
        has_q = hashing && nraw && nraw <= HCAP && cq < cp.chain_len[ks];  // (TAB 4 too: past the last key)
        qslot = cq;
        if constexpr (CCH) {  // the bucket's pilot (an L2-resident array), then the slot
            const uint32_t qh = cmp_key_hash(cq, cp.wseed[ks]);
            qslot = has_q ? cmp_slot(qh, cp.wpil[ks][cmp_scale(qh, cp.wnb[ks])], cp.wdir_len[ks]) : 0u;
        }
#if SKQ_CHN_COALESCED
        // eight lanes read one entry, a 16-B piece each, eight entries per load: a load touches 8
        // lines, not 64 (the texture addresser, busy ~75 % of k_map1's time, works per line), and
        // the pieces reach their owners through LDS in the chain step below. The wave's region is
        // free here: the hashing loop is done with the staged codes.
        {
            uint32_t* s_q = reinterpret_cast<uint32_t*>(s_wave);
            s_q[lane] = has_q ? qslot : 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const u32x4* tab = reinterpret_cast<const u32x4*>(cp.chain[ks]) + (lane & 7u);
#pragma unroll
            for (int u = 0; u < 8; ++u) ce[u] = tab[(uint64_t)s_q[8 * u + (lane >> 3)] * 8];
        }
#else
        // words 0-27 of the entry (28-31 unused), one lane per entry
        const u32x4* ent = reinterpret_cast<const u32x4*>(cp.chain[ks]) + (has_q ? (uint64_t)qslot * 8 : 0ull);
#pragma unroll
        for (int u = 0; u < 7; ++u) ce[u] = ent[u];
#endif
        has_q = hashing && nraw && nraw <= HCAP;  // (a query past the table: no such key)
    }
    if (hashing) {
        if (nraw > HCAP) {
            slow = true;
        } else {
            nraw_out = nraw;
#pragma unroll
            for (int j = 0; j < HCAP; ++j) v[j] = (uint32_t)j < nraw ? s_raw[(HCAP + 1 - j) * MW + tid] : 0xFFFFFFFFu;
            sort_prefix<HCAP>(v, nraw);
            uint32_t* out = p.hashes + (uint64_t)ks * p.hcap * p.n + r;
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < HCAP; ++j) {
                const bool keep = (uint32_t)j < nraw && (j == 0 || v[j] != v[j - 1]);
                if (keep) {
                    if (!p.hpack) out[(uint64_t)m * p.n] = v[j];
                    ++m;
                    keepm |= 1ull << j;
                }
            }
            p.hash_cnt[(uint64_t)ks * p.n + r] = m;
        }
    }
    // packed layout (uniform): the wave's sets one after another in lane order, from the wave's
    // region — whole 64-B lines, where the padded rows leave most lines partly written (the
    // kernel's write requests share the fabric's request budget with its gathers)
    uint32_t hoff = 0;  // (packed) this read's first hash in the wave's region of k slot ks
    if (p.hpack && !(cp.ablate & 8u)) {
        const uint32_t mw = (uint32_t)__builtin_popcountll(keepm);
        const uint32_t incl = wave_incl_scan(mw, lane);
        hoff = incl - mw;
        // (the wave's region: the staged codes are dead, the chain step's loads issued)
        wave_out_packed<HCAP>(p.hashes + (uint64_t)ks * p.hcap * p.n + r0 * p.hcap, hoff, wave_last(incl),
                              reinterpret_cast<uint32_t*>(s_wave), lane, [&](int j) { return ((keepm >> j) & 1ull) != 0; },
                              [&](int j) { return v[j]; });
    }
    if (live && !sk_prev) {
        if (slow) {
            st = ST_SLOW1;
            if (p.hpack) p.hash_cnt[(uint64_t)ks * p.n + r] = 0;  // (none packed: the slow path marks its run)
            if (!pf_prev) {
                list_push(p.ctrl, C_OVF1, C_ERR1, p.ovf1, p.ovf_cap, (uint32_t)r, E_OVF1_FULL);
                list_push(cp.ctrl, C_OVF2, C_ERR2, cp.ovf2, cp.ovf_cap, (uint32_t)r, E_OVF2_FULL);
            }
        } else if (st != SKQ_READ_OK) {
            p.hash_cnt[(uint64_t)ks * p.n + r] = 0;
        }
        p.status[r] = st;
        // (a later skq_chain on these results reads it; pass mode: listed for the slow path)
        if (!PASS || ks == 0 || slow) p.pflag[r] = slow ? 1 : 0;
    } else if (live && p.hpack) {  // (pass mode, slow since an earlier pass: no share of this region)
        p.hash_cnt[(uint64_t)ks * p.n + r] = 0;
    }
    MAP1_STAMP(2);
    // every lane of the wave has left the hashing loop: the staged codes become the parked lists
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- count, entry-parallel: the wave's retained hashes are listed in LDS (hash, owning
    // lane), in passes of MAP_P; lane pairs take them round-robin (each pair gathers one 32-B
    // wide entry, the even lane inserts its head tids t0..t2, the odd lane t3..t6) into the
    // owning read's transcript table with LDS atomics, so the work follows the tids the wave
    // really has rather than its longest read. Table of read (lane) o: column o of this wave in
    // the raw region, slot s at s * WG, (tid << 8 | count) or EMPTY; slot TS: overflow flag.
    // (pass mode: a k slot the index has no table for is sketched but not counted,
    // src/sparse_chaining.cpp:51-53)
    const bool act = hashing && !slow && (!PASS || cp.tabs[ks].present);
    const uint64_t keepm_all = keepm;  // the read's distinct retained hashes (as written out)
    constexpr uint32_t EMPTY = 0xFFFFFFFFu;
#pragma unroll
    for (int sl = 0; sl < TS; ++sl) s_rows[sl * MW + tid] = EMPTY;
    uint32_t* s_flag = reinterpret_cast<uint32_t*>(s_wave + p.map_flag_at);  // per read: > TS transcripts
    s_flag[lane] = 0;
    uint32_t* s_h = reinterpret_cast<uint32_t*>(s_wave);
    uint8_t* s_own = reinterpret_cast<uint8_t*>(s_wave) + MAP_P * 4;
    uint32_t* s_x = reinterpret_cast<uint32_t*>(s_wave + MAP_P * 4);  // compact: slot | lane << 26
    uint32_t* colbase = s_rows + wv * 64;
    const uint32_t* wd = cp.wdir[ks];
    const uint64_t wlen = cp.wdir_len[ks];
    const uint16_t* cpil = cp.wpil[ks];
    const uint32_t cnb = cp.wnb[ks], cseed = cp.wseed[ks];
    const bool odd = lane & 1u;
    // slot sl of read (lane) o sits in column (o + sl) & 63 of row sl: the slots of one read
    // fall in distinct LDS banks (the lane pairs of one round mostly insert into the same read)
    // an insert whose home slot holds another tid probes on from the next slot (rare: not unrolled)
    auto ains_probe = [&](uint32_t x, uint32_t o, uint32_t c = 1u) {
        uint32_t sl = Counter<1, WG>::slot_of(x);
#pragma unroll 1
        for (int z = 1; z < TS; ++z) {
            sl = (sl + 1) & (TS - 1);
            uint32_t* a = colbase + sl * MW + ((o + sl) & 63u);
            const uint32_t old = atomicCAS(a, EMPTY, (x << 8) | c);
            if (old == EMPTY) return;
            if ((old >> 8) == x) {
                atomicAdd(a, c);
                return;
            }
        }
        atomicOr(s_flag + o, 1u);  // more than TS distinct transcripts
    };
    auto ains = [&](uint32_t x, uint32_t o) {
        const uint32_t sl = Counter<1, WG>::slot_of(x);
        uint32_t* a = colbase + sl * MW + ((o + sl) & 63u);
        const uint32_t old = atomicCAS(a, EMPTY, (x << 8) | 1u);
        if (old == EMPTY) return;
        if ((old >> 8) == x) atomicAdd(a, 1u);
        else ains_probe(x, o);
    };
    if constexpr (CHN) {
        // chained tables, one request per read (ChainParams::chain, layout skq_internal.h CHN_*):
        // the lane matches its own retained hashes (v, registers) against the records of its
        // query's entry (ce, requested after the hashing loop), counts each of the entry's ids as
        // the matched records whose list holds it (a popcount over the id's record set), and inserts
        // those into its own count table (no other lane writes it before the entry list below).
        // What no record holds goes through the entry list as before. An entry with no records (no
        // such key, or a query past the table) settles the query itself: no postings.
#if SKQ_CHN_COALESCED
        // the loads' pieces to their owners, 16 entries (2 loads) a round through the wave's region:
        // piece p of entry e at (e * 9 + p) * 16 (the pad: an owner's reads 144 B apart fall in
        // distinct banks); the owners of a round read their entry's words 0-27 (TAB 4: 0-31, word 28
        // naming the slot's key)
        constexpr int NP = CCH ? 8 : 7;
        u32x4 cw[NP];
        {
            u32x4* s_tr = reinterpret_cast<u32x4*>(s_wave);
            const uint32_t g = lane >> 3, pc = lane & 7u, el = lane & 15u;
            // (static_for: a rolled loop would index ce at run time, i.e. through scratch)
            static_for<4>([&](auto rdc) {
                constexpr int rd = decltype(rdc)::value;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                s_tr[g * 9 + pc] = ce[2 * rd];
                s_tr[(8 + g) * 9 + pc] = ce[2 * rd + 1];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if ((lane >> 4) == (uint32_t)rd)
#pragma unroll
                    for (int q = 0; q < NP; ++q) cw[q] = s_tr[el * 9 + q];
            });
        }
#else
        const u32x4* cw = ce;
#endif
        uint32_t w[28];
        // (else the lane read entry 0 and drops it; TAB 4: a query that is no key of the index
        // lands on another key's slot, or an empty one: nothing of it is used)
        bool inb = has_q && cq < cp.chain_len[ks];
        if constexpr (CCH) inb = inb && (cw[7].x ^ CHN_KEY_LIMIT) == cq;
#pragma unroll
        for (int u = 0; u < 7; ++u) {
            w[4 * u] = inb ? cw[u].x : 0u;
            w[4 * u + 1] = inb ? cw[u].y : 0u;
            w[4 * u + 2] = inb ? cw[u].z : 0u;
            w[4 * u + 3] = inb ? cw[u].w : 0u;
        }
        const bool absent = has_q && w[CHN_W_KEY] == 0u;
        uint32_t kh[CHN_KEYS];
#pragma unroll
        for (int i = 0; i < (int)CHN_KEYS; ++i) kh[i] = w[CHN_W_KEY + i] ^ CHN_KEY_LIMIT;  // (unused: 0x0FFFFFFF)
        kh[0] = absent ? cq : kh[0];
        bool hk[CHN_KEYS];
#pragma unroll
        for (int i = 0; i < (int)CHN_KEYS; ++i) hk[i] = false;
        uint32_t hitv = 0;  // bit j: v[j] is a record's key
#pragma unroll
        for (int j = 0; j < HCAP; ++j) {
            if (!__any((uint32_t)j < nraw_out)) break;  // (uniform: the wave's longest set)
            bool hj = false;
#pragma unroll
            for (int i = 0; i < (int)CHN_KEYS; ++i) {
                const bool e = v[j] == kh[i];
                hk[i] = hk[i] || e;
                hj = hj || e;
            }
            hitv |= hj ? (1u << j) : 0u;
        }
        // the matched records as a set; an id's count is the number of them whose list holds it
        uint32_t hm = 0;
#pragma unroll
        for (int i = 0; i < (int)CHN_KEYS; ++i) hm |= hk[i] ? 1u << i : 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the entry's ids with their counts into this read's table: every first attempt (a CAS at
        // the id's home slot) in flight together; the ids are distinct, so an occupied home slot
        // holds another id and the insert probes on
        uint32_t olds[CHN_TIDS], xs[CHN_TIDS], cs[CHN_TIDS];
#pragma unroll
        for (int q = 0; q < (int)CHN_TIDS; ++q) {
            cs[q] = (uint32_t)__builtin_popcount(hm & (w[CHN_W_SET + q / 2] >> (16 * (q & 1))));
            xs[q] = w[CHN_W_TID + q];
            const uint32_t sl = Counter<1, WG>::slot_of(xs[q]);
            olds[q] = cs[q] ? atomicCAS(colbase + sl * MW + ((lane + sl) & 63u), EMPTY, (xs[q] << 8) | cs[q]) : EMPTY;
        }
#pragma unroll
        for (int q = 0; q < (int)CHN_TIDS; ++q)
            if (olds[q] != EMPTY) ains_probe(xs[q], lane, cs[q]);
        keepm &= ~(uint64_t)hitv;
    }
    // the wave's entry list: every retained hash not counted above
    const uint64_t keep0 = keepm_all;
    const uint32_t m = act ? (uint32_t)__builtin_popcountll(keepm) : 0u;
    const uint32_t incl = wave_incl_scan(m, lane);
    const uint32_t off = incl - m;
    const uint32_t M = wave_last(incl);
    {
    // the first pass's list, straight from the sorted registers (v dies here)
    {
        uint32_t rank = 0;
#pragma unroll
        for (int j = 0; j < HCAP; ++j) {
            const bool kj = (keepm >> j) & 1ull;
            const uint32_t e = off + rank;
            if (kj && e < MAP_P) {
                s_h[e] = v[j];
                if (CMP) s_x[e] = lane << 26;
                else s_own[e] = (uint8_t)lane;
            }
            rank += kj ? 1u : 0u;
        }
    }
    for (uint32_t pb = 0; pb < ((cp.ablate & 2u) ? 0u : M); pb += MAP_P) {  // wave-uniform
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (pb) {  // (rare: more than MAP_P hashes in the wave) this lane's hashes, as written above
            // (the d-th listed hash is the d-th still in keepm; its place among the read's written
            // hashes is its rank in keep0, which differs once the chain step counted some)
            uint32_t d = 0, rank = 0;
#pragma unroll
            for (int j = 0; j < HCAP; ++j) {
                if (!((keep0 >> j) & 1ull)) continue;
                if ((keepm >> j) & 1ull) {
                    const uint32_t e = off + d;
                    if (e >= pb && e < pb + MAP_P) {
                        s_h[e - pb] = p.hpack ? p.hashes[(uint64_t)ks * p.hcap * p.n + (r - lane) * p.hcap + hoff + rank]
                                              : p.hashes[((uint64_t)ks * p.hcap + rank) * p.n + r];
                        if (CMP) s_x[e - pb] = lane << 26;
                        else s_own[e - pb] = (uint8_t)lane;
                    }
                    ++d;
                }
                ++rank;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t ne = min(M - pb, (uint32_t)MAP_P);
        if constexpr (CMP) {
            // compact tables: every listed hash's slot, one lane per entry: the bucket's pilot
            // (an L2-resident array; all of the lane's pilot loads in flight together), then the
            // slot, so the lane pairs below gather without a dependent load or any hashing
            constexpr int SB = (MAP_P + 63) / 64;
            uint32_t kh[SB], pv[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const uint32_t e = lane + 64 * q;
                kh[q] = cmp_key_hash(s_h[e < ne ? e : 0], cseed);
                pv[q] = e < ne ? cpil[cmp_scale(kh[q], cnb)] : 0u;
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const uint32_t e = lane + 64 * q;
                if (e < ne) s_x[e] |= cmp_slot(kh[q], pv[q], wlen);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        constexpr int R = MB;  // rounds of 32 entries in flight together
        // lane pair q walks entries [q * S, (q + 1) * S): the 32 entries of one round lie S apart,
        // mostly in different reads' count tables (fewer LDS atomics on one address)
        const uint32_t S = (ne + 31) >> 5;
        for (uint32_t e0 = 0; e0 < S; e0 += R) {
            uint4 w[R];
            uint32_t own[R], hk[R];
            bool ok[R];
            // rounds this pass really has (uniform): behind the chained tables a wave lists ~30
            // hashes, one round, and the other three would only issue predicated-off inserts
            // (chained: 1 % faster; wide tables, whose passes have all four: 2 % slower with the
            // guard, so they keep the fixed rounds: profiles/r4_list_rounds_sdwa_ab.log)
            const uint32_t nu = (SKQ_LIST_NU && CHN) ? min((uint32_t)R, S - e0) : (uint32_t)R;
            if constexpr (CMP) {
                // one entry each, at the slot listed with the hash
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if ((uint32_t)u >= nu) break;
                    const uint32_t e = (lane >> 1) * S + e0 + u;
                    ok[u] = e0 + u < S && e < ne;
                    const uint32_t ee = ok[u] ? e : 0;
                    hk[u] = s_h[ee];
                    const uint32_t x = s_x[ee];
                    own[u] = x >> 26;
                    w[u] = *reinterpret_cast<const uint4*>(wd + (uint64_t)(x & 0x3FFFFFFu) * 8 + (odd ? 4u : 0u));
                }
            } else {
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if ((uint32_t)u >= nu) break;
                    const uint32_t e = (lane >> 1) * S + e0 + u;
                    const bool in = e0 + u < S && e < ne;
                    hk[u] = s_h[in ? e : 0];
                    own[u] = s_own[in ? e : 0];
                    ok[u] = in && hk[u] < wlen;
                    w[u] = *reinterpret_cast<const uint4*>(wd + (ok[u] ? (uint64_t)hk[u] << 3 : 0ull) + (odd ? 4u : 0u));
                }
            }
            constexpr uint32_t TM = CMP ? TID_MASK : 0xFFFFFFFFu;
            // the inserts of each entry: the four first attempts (a CAS at each tid's home slot)
            // are issued before any result is looked at, one LDS round trip; a tid already there
            // gets a non-returning add, and only a slot held by another tid sends the insert on
            // to the probing loop
#pragma unroll
            for (int u = 0; u < R; ++u) {
                if ((uint32_t)u >= nu) break;
                // tids in the entry, pair-uniform (> 7: the list continues at lists[offset];
                // wide: [0x80000000 | offset]); compact: the even lane's half holds key and F
                const uint32_t mine = CMP ? (w[u].x == hk[u] ? w[u].y >> 22 : 0u) : w[u].x;
                const uint32_t sw = pair_swap(mine);
                const uint32_t n = ok[u] ? (odd ? sw : mine) : 0u;
                const uint32_t qb = odd ? 3u : 0u;
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
                    olds[q] = vs[q] ? atomicCAS(colbase + sl * MW + ((own[u] + sl) & 63u), EMPTY, (xs[q] << 8) | 1u)
                                    : EMPTY;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t x = xs[q], sl = Counter<1, WG>::slot_of(x), o = olds[q];
                    if (o == EMPTY) continue;
                    if ((o >> 8) == x) atomicAdd(colbase + sl * MW + ((own[u] + sl) & 63u), 1u);
                    else ains_probe(x, own[u]);
                }
                // lists longer than 7 (rare): the lane holding the offset (wide: even, compact:
                // odd) inserts the rest of the list
                const bool tl = n > 7 && (CMP ? odd : !odd);
                if (__any(tl) && tl) {
                    const uint32_t lo = CMP ? cmp_long_off(w[u]) : n & 0x7FFFFFFFu;
                    const uint32_t len = cp.lists[lo];
                    for (uint32_t q = 7; q < len; ++q) ains(cp.lists[lo + 1 + q], own[u]);
                }
            }
        }
    }
    }  // (the entry list)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    MAP1_STAMP(3);
    uint32_t key[TS];
    uint32_t nc = 0;
    // the need at one k slot from its largest count (src/sparse_chaining.cpp:93: c >= fraction * max
    // as the integer c >= ceil(fraction * max); 256: none passes; 0: all pass)
    auto need_of = [&](uint32_t mx) -> uint32_t {
        const double thr = cp.fraction * (double)mx;
        return thr > 0.0 ? (thr >= 256.0 ? 256u : (uint32_t)ceil(thr)) : 0u;
    };
    if constexpr (PASS) {
        bool listed = pf_prev != 0;  // listed for the slow path by this or an earlier pass
        uint8_t* kneed = cp.kcnt + (uint64_t)p.nk * cp.n;
        uint32_t kev[TS];  // (a pass before the last) the entries meeting this k slot's need, or EMPTY
        uint32_t km = 0;
#pragma unroll
        for (int sl = 0; sl < TS; ++sl) kev[sl] = EMPTY;
        if (act) {
            if (s_flag[lane] != 0) {  // more than TS transcripts at this k: the slow chain path
                if (!listed) list_push(cp.ctrl, C_OVF2, C_ERR2, cp.ovf2, cp.ovf_cap, (uint32_t)r, E_OVF2_FULL);
                p.pflag[r] = 1;
                listed = true;
                if (!FINAL) cp.kcnt[(uint64_t)ks * cp.n + r] = 0;
            } else if (!FINAL) {  // the entries meeting this k slot's need, front-packed, and the need
                uint32_t mx = 0;
#pragma unroll
                for (int sl = 0; sl < TS; ++sl) {
                    kev[sl] = colbase[sl * MW + ((lane + sl) & 63u)];
                    mx = max(mx, kev[sl] != EMPTY ? kev[sl] & 0xFFu : 0u);
                }
                const uint32_t need = need_of(mx);
#pragma unroll
                for (int sl = 0; sl < TS; ++sl) {
                    if (kev[sl] != EMPTY && (kev[sl] & 0xFFu) < need) kev[sl] = EMPTY;
                    if (kev[sl] != EMPTY) {
                        if (!cp.hpack) cp.ktab[((uint64_t)ks * TS + km) * cp.n + r] = kev[sl];
                        ++km;
                    }
                }
                cp.kcnt[(uint64_t)ks * cp.n + r] = (uint8_t)km;
                kneed[(uint64_t)ks * cp.n + r] = (uint8_t)min(need, 255u);
            }
        } else if (live && !FINAL) {  // (a k slot the index lacks does not filter)
            cp.kcnt[(uint64_t)ks * cp.n + r] = 0;
            kneed[(uint64_t)ks * cp.n + r] = 0;
        }
        if (!FINAL && cp.hpack) {  // (uniform) packed: the wave's kept entries in lane order
            const uint32_t incl = wave_incl_scan(km, lane);
            wave_out_packed<TS>(cp.ktab + (uint64_t)ks * TS * cp.n + r0 * TS, incl - km, wave_last(incl),
                                reinterpret_cast<uint32_t*>(s_wave), lane, [&](int sl) { return kev[sl] != EMPTY; },
                                [&](int sl) { return kev[sl]; });
        }
        // (last pass, packed) where each earlier pass's entries of this read start in its region
        uint32_t koff[NK_FAST - 1] = {};
        if (FINAL && cp.hpack) {  // (uniform)
#pragma unroll
            for (int i = 0; i < NK_FAST - 1; ++i)
                if ((uint32_t)i < ks) {
                    const uint32_t c = live ? cp.kcnt[(uint64_t)i * cp.n + r] : 0u;
                    koff[i] = wave_incl_scan(c, lane) - c;
                }
        }
        if (FINAL) {
            // the transcripts over the k slots, in registers: slot s holds tid ut[s] (EMPTY: free)
            // and its 8-bit counts per k slot uc[s]; this pass's table as it lies (its slots), then
            // the earlier passes' entries matched by tid — or, when this k slot does not filter
            // (need 0), placed in a free slot (src/sparse_chaining.cpp:55-73)
            const bool merge = hashing && !slow && !listed;
            if (merge) {
                // this pass's table (in LDS, the lane's own column): its need, and which slots meet it
                uint32_t mxf = 0, thisok = 0;
                {
                    uint32_t ev[TS];
#pragma unroll
                    for (int sl = 0; sl < TS; ++sl) {
                        ev[sl] = colbase[sl * MW + ((lane + sl) & 63u)];
                        mxf = max(mxf, ev[sl] != EMPTY ? ev[sl] & 0xFFu : 0u);
                    }
                    const uint32_t nf = need_of(mxf);
#pragma unroll
                    for (int sl = 0; sl < TS; ++sl)
                        thisok |= ev[sl] != EMPTY && (ev[sl] & 0xFFu) >= nf ? 1u << sl : 0u;
                }
                const uint32_t needf = need_of(mxf);
                const bool inter = needf > 0;  // only this k slot's transcripts can pass
                if (!inter) thisok = 0xFFFFu;  // (this k slot does not filter: any slot, also one filled below)
                bool full = false;
                // the earlier passes' entry counts and needs, then their entries 8 per k slot at a
                // time, all of a batch's loads in flight together
                const uint8_t* kneed = cp.kcnt + (uint64_t)p.nk * cp.n;
                uint32_t mk[NK_FAST - 1], nd[NK_FAST - 1], nfilt = 0;
#pragma unroll
                for (int i = 0; i < NK_FAST - 1; ++i) {
                    mk[i] = (uint32_t)i < ks ? cp.kcnt[(uint64_t)i * cp.n + r] : 0u;
                    nd[i] = (uint32_t)i < ks ? kneed[(uint64_t)i * cp.n + r] : 0u;
                    nfilt += nd[i] > 0 ? 1u : 0u;
                }
                // each earlier entry (its pass's count, meeting that pass's need) found in this
                // pass's table by its own probe sequence (home slot, then on) and added into the
                // entry there: the count field gathers the counts over the k slots (<= 4 x 32), bits
                // 30-31 count the filtering k slots that hold the transcript (ids < 2^22: free bits).
                // Where this k slot does not filter (need 0) a transcript it lacks takes the first
                // free slot on its probe path (src/sparse_chaining.cpp:55-73). The lane's column is
                // its own: plain loads and stores. (Round 4 compared every entry with all 16 slots in
                // registers: the same time within 0.3 %, 18 KB more code; profiles/r5_merge_ab.log.)
                for (uint32_t j0 = 0; j0 < ((cp.ablate & 64u) ? 0u : (uint32_t)TS); j0 += 8) {  // (64: pricing)
                    bool more = false;
#pragma unroll
                    for (int i = 0; i < NK_FAST - 1; ++i) more |= j0 < mk[i];
                    if (!__any(more)) break;
                    uint32_t eb[NK_FAST - 1][8];
#pragma unroll
                    for (int i = 0; i < NK_FAST - 1; ++i)
#pragma unroll
                        for (int u = 0; u < 8; ++u)
                            eb[i][u] = j0 + u < mk[i]
                                           ? (cp.hpack ? cp.ktab[(uint64_t)i * TS * cp.n + (r - lane) * TS + koff[i] + j0 + u]
                                                       : cp.ktab[((uint64_t)i * TS + j0 + u) * cp.n + r])
                                           : EMPTY;
#pragma unroll
                    for (int i = 0; i < NK_FAST - 1; ++i)
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t e = eb[i][u];
                        if (e == EMPTY) continue;
                        const uint32_t x = e >> 8, add = (e & 0xFFu) + (nd[i] > 0 ? 1u << 30 : 0u);
                        uint32_t sl = Counter<1, WG>::slot_of(x);
                        bool done = false;
#pragma unroll 1
                        for (int z = 0; z < TS && !done; ++z) {
                            uint32_t* a = colbase + sl * MW + ((lane + sl) & 63u);
                            const uint32_t v = *a;
                            if (v == EMPTY) {
                                if (!inter) *a = (x << 8) + add;
                                done = true;
                            } else if (((v >> 8) & TID_MASK) == x) {
                                *a = v + add;
                                done = true;
                            }
                            sl = (sl + 1) & (TS - 1);
                        }
                        full |= !done && !inter;
                    }
                }
                if (full) {  // more than TS transcripts over the k slots
                    list_push(cp.ctrl, C_OVF2, C_ERR2, cp.ovf2, cp.ovf_cap, (uint32_t)r, E_OVF2_FULL);
                    p.pflag[r] = 1;
                    cp.cand_cnt[r] = 0;
                } else {
                    // filter at every k slot (src/sparse_chaining.cpp:76-101), as Counter::finish: this
                    // one's need from its table (thisok), the earlier ones' as their passes applied them
                    // (their entries met them: a transcript passes where every filtering earlier k
                    // slot holds it); score = the counts' sum (src/sparse_chaining.cpp:100). (Counts
                    // <= 32 here, so a need past 255 passes nothing.)
                    const bool nonef = needf > 255u;
#pragma unroll
                    for (int sl = 0; sl < TS; ++sl) {
                        const uint32_t v = colbase[sl * MW + ((lane + sl) & 63u)];
                        const bool ok = v != EMPTY && ((thisok >> sl) & 1u) && (v >> 30) == nfilt && !nonef;
                        // score desc, tid asc (src/sparse_chaining.cpp:108-109, ties normalised)
                        key[sl] = ok ? ((1023u - (v & 0xFFu)) << 22) | ((v >> 8) & TID_MASK) : ~0u;
                    }
                    bitonic_sort<TS>(key);
                    uint32_t* ct = cp.cand_tid + r;
                    uint32_t* cs = cp.cand_score + r;
#pragma unroll
                    for (int d = 0; d < TS; ++d) {
                        if (key[d] != ~0u) {
                            if (!cp.cpack) {
                                ct[(uint64_t)d * cp.n] = key[d] & 0x3FFFFFu;
                                cs[(uint64_t)d * cp.n] = 1023u - (key[d] >> 22);
                            }
                            ++nc;
                        }
                    }
                    cp.cand_cnt[r] = nc;
                }
            } else if (live && !sk_prev) {  // (sk_prev: k_slow_wave writes them)
                cp.cand_cnt[r] = 0;
            }
            if (cp.cpack) {  // (uniform) packed: the wave's candidates in lane order, tid | score << 22
                const uint32_t incl = wave_incl_scan(nc, lane);
                if (lane == 63 && cp.cand_wtot && nr) cp.cand_wtot[r0 >> 6] = incl;  // (k_bin_packed)
                wave_out_packed<TS, true>(cp.cand_tid + r0 * CCAP, incl - nc, wave_last(incl),
                                    reinterpret_cast<uint32_t*>(s_wave), lane, [&](int d) { return (uint32_t)d < nc; },
                                    [&](int d) { return (key[d] & 0x3FFFFFu) | ((1023u - (key[d] >> 22)) << 22); });
            }
        }
    } else {
        if (act && !(cp.ablate & 4u)) {
            if (s_flag[lane] == 0) {
                // filter and order (src/sparse_chaining.cpp:76-110), as Counter::finish
                uint32_t ev[TS];
                uint32_t mx = 0;
#pragma unroll
                for (int sl = 0; sl < TS; ++sl) {
                    ev[sl] = colbase[sl * MW + ((lane + sl) & 63u)];
                    mx = max(mx, ev[sl] != EMPTY ? ev[sl] & 0xFFu : 0u);
                }
                const double thr = cp.fraction * (double)mx;
                uint32_t need = 0;
                if (thr > 0.0) need = thr >= 256.0 ? 256u : (uint32_t)ceil(thr);
#pragma unroll
                for (int sl = 0; sl < TS; ++sl) {
                    const uint32_t cnt = ev[sl] & 0xFFu;
                    key[sl] = (ev[sl] != EMPTY && cnt >= need) ? ((1023u - cnt) << 22) | (ev[sl] >> 8) : ~0u;
                }
                bitonic_sort<TS>(key);
                uint32_t* ct = cp.cand_tid + r;
                uint32_t* cs = cp.cand_score + r;
#pragma unroll
                for (int d = 0; d < TS; ++d) {
                    if (!__any(key[d] != ~0u)) break;  // (uniform: sorted, the kept keys come first)
                    if (key[d] != ~0u) {
                        if (!cp.cpack) {
                            ct[(uint64_t)d * cp.n] = key[d] & 0x3FFFFFu;
                            cs[(uint64_t)d * cp.n] = 1023u - (key[d] >> 22);
                        }
                        ++nc;
                    }
                }
                cp.cand_cnt[r] = nc;
            } else {
                list_push(cp.ctrl, C_OVF2, C_ERR2, cp.ovf2, cp.ovf_cap, (uint32_t)r, E_OVF2_FULL);
                cp.cand_cnt[r] = 0;
            }
        } else if (live) {
            cp.cand_cnt[r] = 0;
        }
        if (cp.cpack) {  // (uniform) packed: the wave's candidates in lane order, tid | score << 22
            const uint32_t incl = wave_incl_scan(nc, lane);
            if (lane == 63 && cp.cand_wtot && nr) cp.cand_wtot[r0 >> 6] = incl;  // (k_bin_packed)
            // (the wave's region: the entry list and the per-read flags are dead)
            wave_out_packed<TS, true>(cp.cand_tid + r0 * CCAP, incl - nc, wave_last(incl), reinterpret_cast<uint32_t*>(s_wave),
                                lane, [&](int d) { return (uint32_t)d < nc; },
                                [&](int d) { return (key[d] & 0x3FFFFFu) | ((1023u - (key[d] >> 22)) << 22); });
        }
    }
    MAP1_STAMP(4);
}

// (SKQ_MAP1_WPE / SKQ_PASS_WPE: the waves per SIMD the compiler budgets registers for, one-k map /
// multi-k passes. 5 (96 VGPRs): the passes over chained tables otherwise take 99-108 VGPRs, 4 waves;
// at 5 they spill 4-20 VGPRs to scratch and run 5 % faster at cfg5 (tools/abbench.py,
// profiles/r6_wpe5_ab.log); the one-k map fits 5 unforced)
#ifndef SKQ_MAP1_WPE
#define SKQ_MAP1_WPE 5
#endif
#ifndef SKQ_PASS_WPE
#define SKQ_PASS_WPE 5
#endif
template <int HCAP, int MB, int TAB, bool PASS = false, bool FINAL = false, int MW = WG>
__global__ __launch_bounds__(MW) __attribute__((amdgpu_waves_per_eu(PASS ? SKQ_PASS_WPE : SKQ_MAP1_WPE))) void k_map1(SketchParams p, ChainParams cp) {
    static_assert(PASS || !FINAL, "the final pass is a pass");
    map1_body<HCAP, MB, TAB, PASS, MW>(p, cp, PASS ? p.kslot : 0u, FINAL);
}

// Multi-k map in ONE launch: each workgroup runs the k slots' passes over its own reads one after
// another (the same work as the k_map1 pass launches, each k slot with the same capacity HCAP and
// table kind TAB). A pass's per-read results (pflag, status, ktab / kcnt, the staged image of the
// bases) are read back by the same workgroup's waves in the next pass, through the CU's cache, and
// the launches' tails are paid once. The barrier between passes: every wave is done with the roll
// terms and its LDS region before the next pass rewrites them, and the pass's global stores are
// complete (workgroup-scope release / acquire).
// (its registers: 128 at 4 waves per SIMD, k_map1's ~100 for 5 plus the loop's; SKQ_MAPK_WPE=5
// caps them at 96 with ~30 spilled, a development A/B)
#ifndef SKQ_MAPK_WPE
#define SKQ_MAPK_WPE 4
#endif
template <int HCAP, int MB, int TAB, int MW = WG>
__global__ __launch_bounds__(MW) __attribute__((amdgpu_waves_per_eu(SKQ_MAPK_WPE))) void k_mapk(SketchParams p, ChainParams cp) {
#pragma unroll 1
    for (uint32_t ks = 0; ks < p.nk; ++ks) {
        if (ks) __syncthreads();
        map1_body<HCAP, MB, TAB, true, MW>(p, cp, ks, ks + 1 == p.nk);
    }
}

}  // namespace skq
