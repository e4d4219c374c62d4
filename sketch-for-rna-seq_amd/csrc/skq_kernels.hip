// skq_kernels.hip — gfx950 kernels for the FracMinHash sketch + sparse-chain hot path.
//
//   k_sketch       reads (ASCII) -> per (read, k) sorted set of retained 32-bit ntHash values.
//                  Restates createSketch_FracMinhash_direct (reference src/sketch.cpp:24-39) and
//                  the read filters of process_fastq_single_pass (src/main.cpp:132-138).
//                  One workgroup = 256 reads. The workgroup's byte span is staged once into LDS
//                  with coalesced 16-B loads, converted to 2-bit codes + an invalid-base mask;
//                  each lane then rolls the 33-bit ntHash lane over its own read.
//   k_chain        per read: probe every retained hash in the device index, count per
//                  (transcript, k), per-k max, keep transcripts with count >= fraction*max at
//                  every k, score = sum of counts, sort (score desc, tid asc). Restates
//                  sparse_chain (src/sparse_chaining.cpp:42-111). One lane per read; the count
//                  table lives in registers (16 transcripts x packed 8-bit counts).
//   *_slow         exact fallbacks for what the fast kernels do not bound (reads > 256 bp, more
//                  than HCAP retained hashes, more than 16 distinct transcripts, > 4 k slots).
//                  They run over device-side work lists with a fixed grid: no host round trip.
#include <hip/hip_runtime.h>

#include "skq_internal.h"

namespace skq {

// ---------------------------------------------------------------------------------------------
// small helpers

template <typename T>
__device__ __forceinline__ void cswap(T& a, T& b) {
    T lo = a < b ? a : b;
    T hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// ascending bitonic sort of a register array (fully unrolled: every index is a constant)
template <int N, typename T>
__device__ __forceinline__ void bitonic_sort(T (&a)[N]) {
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

// ---------------------------------------------------------------------------------------------
// K1: sketch

size_t sketch_lds_bytes(uint32_t nk, uint32_t tile_chunks, uint32_t hcap) {
    size_t b = (size_t)nk * 32 * 8;                         // roll tables
    b += (size_t)tile_chunks * 4;                           // 2-bit codes
    b += ((size_t)tile_chunks * 2 + 15) & ~(size_t)15;      // invalid-base masks
    b += (size_t)hcap * WG * 4;                             // raw retained hashes
    return b;
}

template <int HCAP>
__global__ __launch_bounds__(WG) void k_sketch(SketchParams p) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* s_tab = reinterpret_cast<uint64_t*>(smem);
    uint32_t* s_codes = reinterpret_cast<uint32_t*>(smem + (size_t)p.nk * 32 * 8);
    uint16_t* s_bad = reinterpret_cast<uint16_t*>(s_codes + p.tile_chunks);
    uint32_t* s_raw = reinterpret_cast<uint32_t*>(
        reinterpret_cast<unsigned char*>(s_bad) + ((((size_t)p.tile_chunks * 2) + 15) & ~(size_t)15));

    const int tid = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * WG;
    const uint32_t nr = (uint32_t)min((uint64_t)WG, p.n - r0);

    // workgroup byte span, in 16-byte chunks of the aligned-down base pointer
    const uintptr_t base = reinterpret_cast<uintptr_t>(p.reads);
    const uintptr_t abase = base & ~(uintptr_t)15;
    const uint64_t delta = base - abase;
    uint64_t s0, l0, sl, ll;
    read_extent(p.offs, p.fixed_len, r0, s0, l0);
    read_extent(p.offs, p.fixed_len, r0 + nr - 1, sl, ll);
    const uint64_t c0 = (s0 + delta) >> 4;
    const uint64_t c1 = (sl + ll + delta + 15) >> 4;
    const uint32_t nch = (uint32_t)min((uint64_t)p.tile_chunks, c1 - c0);

    for (uint32_t c = tid; c < nch; c += WG) {
        const uint4 v = *reinterpret_cast<const uint4*>(abase + (c0 + c) * 16);
        uint32_t a, b, cc, d, ba, bb, bc, bd;
        encode4(v.x, a, ba);
        encode4(v.y, b, bb);
        encode4(v.z, cc, bc);
        encode4(v.w, d, bd);
        s_codes[c] = a | (b << 8) | (cc << 16) | (d << 24);
        s_bad[c] = (uint16_t)(ba | (bb << 4) | (bc << 8) | (bd << 12));
    }
    for (uint32_t e = tid; e < p.nk * 32; e += WG) s_tab[e] = p.rolltab[e];
    __syncthreads();

    if ((uint32_t)tid >= nr) return;
    const uint64_t r = r0 + tid;
    uint64_t start, len;
    read_extent(p.offs, p.fixed_len, r, start, len);
    const uint64_t q0 = start + delta - c0 * 16;  // tile position of this read's first base

    bool slow = len > (uint64_t)LFAST || q0 + len > (uint64_t)nch * 16;
    uint8_t st = SKQ_READ_OK;
    if (!slow) {
        // is_valid_sequence (src/data_io.cpp:17-34): every byte uppercase A/C/G/T
        bool bad = false;
        if (len) {
            const uint64_t last = q0 + len - 1;
            for (uint64_t c = q0 >> 4; c <= (last >> 4); ++c) {
                uint32_t m = s_bad[c];
                const uint32_t lo = (c == (q0 >> 4)) ? (uint32_t)(q0 & 15) : 0u;
                const uint32_t hi = (c == (last >> 4)) ? (uint32_t)(last & 15) : 15u;
                m &= ((2u << hi) - 1u) & ~((1u << lo) - 1u);
                bad |= m != 0;
            }
        }
        if (bad) st = SKQ_READ_INVALID;
        else if (len < p.maxk) st = SKQ_READ_SHORT;  // src/main.cpp:136-138
    }

    if (!slow && st == SKQ_READ_OK) {
        const uint32_t T = p.threshold;
        for (uint32_t i = 0; i < p.nk && !slow; ++i) {
            const uint32_t k = p.ks[i];
            const uint64_t* tab = s_tab + i * 32;
            uint32_t hlo = 0, hhi = 0, nraw = 0;
            // h <- rot33(h) ^ seed(in) ^ rot33^k(seed(out)); the first k steps have no out base,
            // which builds the first window's hash from zero (NtHash::init).
            for (uint32_t pos = 0; pos < (uint32_t)len; ++pos) {
                const uint64_t qi = q0 + pos;
                const uint32_t cin = (s_codes[qi >> 4] >> ((qi & 15) * 2)) & 3u;
                uint32_t cout = 4u;
                if (pos >= k) {
                    const uint64_t qo = qi - k;
                    cout = (s_codes[qo >> 4] >> ((qo & 15) * 2)) & 3u;
                }
                const uint64_t e = tab[cin * 8 + cout];
                const uint32_t nlo = (hlo << 1) | hhi;
                hhi = (hlo >> 31) ^ (uint32_t)(e >> 32);
                hlo = nlo ^ (uint32_t)e;
                if (pos + 1 >= k && hlo <= T) {  // src/sketch.cpp:33-35
                    if (nraw < HCAP) s_raw[nraw * WG + tid] = hlo;
                    ++nraw;
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
            bitonic_sort<HCAP>(v);
            uint32_t* out = p.hashes + (r * p.nk + i) * p.hcap;
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < HCAP; ++j) {
                const bool keep = (uint32_t)j < nraw && (j == 0 || v[j] != v[j - 1]);
                if (keep) out[m++] = v[j];
            }
            p.hash_cnt[r * p.nk + i] = m;
        }
    }
    if (slow) {
        st = ST_SLOW1;
        list_push(p.ctrl, C_OVF1, C_ERR1, p.ovf1, p.ovf_cap, (uint32_t)r, E_OVF1_FULL);
    } else if (st != SKQ_READ_OK) {
        for (uint32_t i = 0; i < p.nk; ++i) p.hash_cnt[r * p.nk + i] = 0;
    }
    p.status[r] = st;
}

// Slow sketch path: one lane per listed read, straight from global memory. Retained hashes go
// to a bump-allocated region sized by the read's window count, then are sorted in place.
__global__ __launch_bounds__(64) void k_sketch_slow(SketchParams p) {
    const uint32_t cnt = min(p.ctrl[C_OVF1], p.ovf_cap);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
        const uint64_t r = p.ovf1[j];
        uint64_t start, len;
        read_extent(p.offs, p.fixed_len, r, start, len);
        const uint8_t* s = p.reads + start;
        bool bad = false;
        for (uint64_t q = 0; q < len && !bad; ++q) {
            const uint8_t c = s[q];
            bad = !(c == 'A' || c == 'C' || c == 'G' || c == 'T');
        }
        uint8_t st = bad ? SKQ_READ_INVALID : (len < p.maxk ? SKQ_READ_SHORT : SKQ_READ_OK);
        for (uint32_t i = 0; i < p.nk; ++i) p.hash_cnt[r * p.nk + i] = 0;
        if (st == SKQ_READ_OK) {
            for (uint32_t i = 0; i < p.nk; ++i) {
                const uint32_t k = p.ks[i];
                const uint64_t nw = len - k + 1;
                unsigned long long* bump = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_H);
                const uint64_t at = atomicAdd(bump, (unsigned long long)nw);
                if (at + nw > p.hash_ext_cap) {
                    atomicOr(&p.ctrl[C_ERR1], (uint32_t)E_HASH_EXT);
                    break;
                }
                uint32_t* ext = p.hash_ext + at;
                const uint64_t* tab = p.rolltab + i * 32;
                uint32_t hlo = 0, hhi = 0;
                uint64_t m = 0;
                for (uint64_t pos = 0; pos < len; ++pos) {
                    const uint32_t cin = (s[pos] >> 1) & 3u;
                    const uint32_t cout = pos >= k ? ((s[pos - k] >> 1) & 3u) : 4u;
                    const uint64_t e = tab[cin * 8 + cout];
                    const uint32_t nlo = (hlo << 1) | hhi;
                    hhi = (hlo >> 31) ^ (uint32_t)(e >> 32);
                    hlo = nlo ^ (uint32_t)e;
                    if (pos + 1 >= k && hlo <= p.threshold) ext[m++] = hlo;
                }
                // shell sort (Ciura gaps) + unique, in place
                const uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
                for (int g = 0; g < 8; ++g) {
                    const uint64_t gap = gaps[g];
                    for (uint64_t a = gap; a < m; ++a) {
                        const uint32_t x = ext[a];
                        uint64_t b = a;
                        while (b >= gap && ext[b - gap] > x) {
                            ext[b] = ext[b - gap];
                            b -= gap;
                        }
                        ext[b] = x;
                    }
                }
                uint64_t u = 0;
                for (uint64_t a = 0; a < m; ++a)
                    if (a == 0 || ext[a] != ext[u - 1]) ext[u++] = ext[a];
                uint32_t* slot = p.hashes + (r * p.nk + i) * p.hcap;
                if (u <= p.hcap) {
                    for (uint64_t a = 0; a < u; ++a) slot[a] = ext[a];
                } else {
                    slot[0] = (uint32_t)at;
                }
                p.hash_cnt[r * p.nk + i] = (uint32_t)u;
            }
        }
        p.status[r] = st;
    }
}

// ---------------------------------------------------------------------------------------------
// K2: chain

__device__ __forceinline__ const uint32_t* hash_list(const ChainParams& p, uint64_t r, uint32_t i,
                                                     uint32_t cnt) {
    if (p.hash_offs) return p.hashes + p.hash_offs[r * p.nk + i];
    const uint32_t* slot = p.hashes + (r * p.nk + i) * p.hcap;
    return cnt <= p.hcap ? slot : p.hash_ext + slot[0];
}

// returns the postings offset of `key` in table t, or ~0u on a miss
__device__ __forceinline__ uint32_t probe(const uint64_t* slots, const DevTable& t, uint32_t key) {
    const uint64_t mask = (1ull << t.log2cap) - 1;
    uint64_t s = (uint32_t)(key * HASH_MUL) >> (32 - t.log2cap);
    for (;;) {
        const uint64_t v = slots[t.slot_base + s];
        if (v == EMPTY_SLOT) return ~0u;
        if ((uint32_t)(v >> 32) == key) return (uint32_t)v;
        s = (s + 1) & mask;
    }
}

__global__ __launch_bounds__(WG) void k_chain(ChainParams p) {
    const uint64_t r = (uint64_t)blockIdx.x * WG + threadIdx.x;
    if (r >= p.n) return;
    if (p.status && (p.status[r] & SKQ_STATUS_MASK) != SKQ_READ_OK) {
        p.cand_cnt[r] = 0;
        return;
    }
    uint32_t tids[DCAP], cnts[DCAP];
#pragma unroll
    for (int d = 0; d < DCAP; ++d) {
        tids[d] = 0xFFFFFFFFu;
        cnts[d] = 0;
    }
    uint32_t nd = 0;
    bool slow = p.nk > (uint32_t)NK_FAST;

    for (uint32_t i = 0; i < p.nk && !slow; ++i) {
        const DevTable t = p.tabs[i];
        if (!t.present) continue;
        if (p.present && !p.present[r * p.nk + i]) continue;
        const uint32_t cnt = p.hash_cnt[r * p.nk + i];
        if (cnt > (uint32_t)HFAST) {
            slow = true;
            break;
        }
        const uint32_t* hs = hash_list(p, r, i, cnt);
        const uint32_t inc = 1u << (8 * i);
        for (uint32_t j0 = 0; j0 < cnt && !slow; j0 += 4) {
            // issue up to 4 independent probes, then their postings headers
            uint32_t off[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) off[u] = (j0 + u < cnt) ? probe(p.slots, t, hs[j0 + u]) : ~0u;
            uint4 head[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                head[u] = off[u] != ~0u ? *reinterpret_cast<const uint4*>(p.post + off[u])
                                        : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t np = head[u].x;
                for (uint32_t e = 0; e < np; ++e) {
                    const uint32_t x = e == 0 ? head[u].y : e == 1 ? head[u].z : e == 2 ? head[u].w
                                                                                         : p.post[off[u] + 1 + e];
                    bool found = false;
#pragma unroll
                    for (int d = 0; d < DCAP; ++d) {
                        const bool hit = tids[d] == x;
                        cnts[d] += hit ? inc : 0u;
                        found |= hit;
                    }
                    if (!found) {
                        if (nd == (uint32_t)DCAP) {
                            slow = true;
                            break;
                        }
#pragma unroll
                        for (int d = 0; d < DCAP; ++d) {
                            if ((uint32_t)d == nd) {
                                tids[d] = x;
                                cnts[d] = inc;
                            }
                        }
                        ++nd;
                    }
                }
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
    // (counts here are <= HFAST, so a threshold clamped to 255 rejects the same transcripts; a
    // NaN or non-positive threshold accepts everything, as `c < thr` is then false.)
    uint32_t need = 0;  // packed per-k ceil thresholds
    for (uint32_t i = 0; i < p.nk; ++i) {
        uint32_t m = 0;
#pragma unroll
        for (int d = 0; d < DCAP; ++d) m = max(m, (cnts[d] >> (8 * i)) & 0xFFu);
        const double thr = p.fraction * (double)m;
        uint32_t ti = 0;
        if (thr > 0.0) ti = thr >= 255.0 ? 255u : (uint32_t)ceil(thr);
        need |= ti << (8 * i);
    }
    uint64_t key[DCAP];
#pragma unroll
    for (int d = 0; d < DCAP; ++d) {
        bool ok = (uint32_t)d < nd;
        uint32_t score = 0;
        for (uint32_t i = 0; i < p.nk; ++i) {
            const uint32_t c = (cnts[d] >> (8 * i)) & 0xFFu;
            ok &= c >= ((need >> (8 * i)) & 0xFFu);
            score += c;
        }
        // sort key: score desc, tid asc (src/sparse_chaining.cpp:108-109, ties normalised)
        key[d] = ok ? (((uint64_t)(0xFFFFFFFFu - score) << 32) | tids[d]) : ~0ull;
    }
    bitonic_sort<DCAP>(key);
    uint32_t nc = 0;
    uint32_t* ct = p.cand_tid + r * CCAP;
    uint32_t* cs = p.cand_score + r * CCAP;
#pragma unroll
    for (int d = 0; d < DCAP; ++d) {
        if (key[d] != ~0ull) {
            const uint32_t tid = (uint32_t)key[d];
            const uint32_t score = 0xFFFFFFFFu - (uint32_t)(key[d] >> 32);
            ct[d] = tid;
            cs[d] = score;
            ++nc;
            if (p.accumulate) {
                atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[tid]), 1ull);
                atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[tid]), (unsigned long long)score);
            }
        }
    }
    p.cand_cnt[r] = nc;
}

// Slow chain path: one lane per listed read. Postings are gathered into a bump-allocated
// scratch of (tid << 3 | k slot) words, sorted, run-length counted.
__device__ void shell_sort_u64(uint64_t* a, uint64_t m) {
    const uint32_t gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
    for (int g = 0; g < 8; ++g) {
        const uint64_t gap = gaps[g];
        for (uint64_t x = gap; x < m; ++x) {
            const uint64_t v = a[x];
            uint64_t b = x;
            while (b >= gap && a[b - gap] > v) {
                a[b] = a[b - gap];
                b -= gap;
            }
            a[b] = v;
        }
    }
}

__global__ __launch_bounds__(64) void k_chain_slow(ChainParams p) {
    const uint32_t cnt = min(p.ctrl[C_OVF2], p.ovf_cap);
    unsigned long long* bump_s = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_S);
    unsigned long long* bump_c = reinterpret_cast<unsigned long long*>(p.ctrl + C_BUMP_C);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
        const uint64_t r = p.ovf2[j];
        // pass 1: size
        uint64_t P = 0;
        for (uint32_t i = 0; i < p.nk; ++i) {
            if (!p.tabs[i].present || (p.present && !p.present[r * p.nk + i])) continue;
            const uint32_t hc = p.hash_cnt[r * p.nk + i];
            const uint32_t* hs = hash_list(p, r, i, hc);
            for (uint32_t h = 0; h < hc; ++h) {
                const uint32_t off = probe(p.slots, p.tabs[i], hs[h]);
                if (off != ~0u) P += p.post[off];
            }
        }
        const uint64_t need = 2 * P + 1;
        const uint64_t at = atomicAdd(bump_s, (unsigned long long)need);
        if (at + need > p.scratch_cap) {
            atomicOr(&p.ctrl[C_ERR2], (uint32_t)E_SCRATCH);
            p.cand_cnt[r] = 0;
            continue;
        }
        uint64_t* ent = p.scratch + at;
        uint64_t* cand = ent + P;
        uint64_t e = 0;
        for (uint32_t i = 0; i < p.nk; ++i) {
            if (!p.tabs[i].present || (p.present && !p.present[r * p.nk + i])) continue;
            const uint32_t hc = p.hash_cnt[r * p.nk + i];
            const uint32_t* hs = hash_list(p, r, i, hc);
            for (uint32_t h = 0; h < hc; ++h) {
                const uint32_t off = probe(p.slots, p.tabs[i], hs[h]);
                if (off == ~0u) continue;
                const uint32_t np = p.post[off];
                for (uint32_t q = 0; q < np; ++q) ent[e++] = ((uint64_t)p.post[off + 1 + q] << 8) | i;
            }
        }
        shell_sort_u64(ent, P);
        uint32_t maxc[SKQ_MAX_K];
        for (uint32_t i = 0; i < p.nk; ++i) maxc[i] = 0;
        for (uint64_t a = 0; a < P;) {
            uint64_t b = a;
            const uint64_t t = ent[a] >> 8;
            uint32_t c[SKQ_MAX_K];
            for (uint32_t i = 0; i < p.nk; ++i) c[i] = 0;
            while (b < P && (ent[b] >> 8) == t) c[ent[b++] & 0xFF]++;
            for (uint32_t i = 0; i < p.nk; ++i) maxc[i] = max(maxc[i], c[i]);
            a = b;
        }
        double thr[SKQ_MAX_K];
        for (uint32_t i = 0; i < p.nk; ++i) thr[i] = p.fraction * (double)maxc[i];
        uint64_t nc = 0;
        for (uint64_t a = 0; a < P;) {
            uint64_t b = a;
            const uint64_t t = ent[a] >> 8;
            uint32_t c[SKQ_MAX_K];
            for (uint32_t i = 0; i < p.nk; ++i) c[i] = 0;
            while (b < P && (ent[b] >> 8) == t) c[ent[b++] & 0xFF]++;
            bool ok = true;
            uint32_t score = 0;
            for (uint32_t i = 0; i < p.nk; ++i) {
                if ((double)c[i] < thr[i]) { ok = false; break; }
                score += c[i];
            }
            if (ok) cand[nc++] = ((uint64_t)(0xFFFFFFFFu - score) << 32) | (uint32_t)t;
            a = b;
        }
        shell_sort_u64(cand, nc);
        uint32_t* ct;
        uint32_t* cs;
        uint64_t stride = 1;
        if (nc <= (uint64_t)CCAP) {
            ct = p.cand_tid + r * CCAP;
            cs = p.cand_score + r * CCAP;
        } else {
            const uint64_t cat = atomicAdd(bump_c, (unsigned long long)nc);
            if (cat + nc > p.cand_ext_cap) {
                atomicOr(&p.ctrl[C_ERR2], (uint32_t)E_CAND_EXT);
                p.cand_cnt[r] = 0;
                continue;
            }
            p.cand_tid[r * CCAP] = (uint32_t)cat;
            ct = p.cand_ext + 2 * cat;
            cs = ct + 1;
            stride = 2;
        }
        for (uint64_t a = 0; a < nc; ++a) {
            const uint32_t tid = (uint32_t)cand[a];
            const uint32_t score = 0xFFFFFFFFu - (uint32_t)(cand[a] >> 32);
            ct[a * stride] = tid;
            cs[a * stride] = score;
            if (p.accumulate) {
                atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_reads[tid]), 1ull);
                atomicAdd(reinterpret_cast<unsigned long long*>(&p.tx_score[tid]), (unsigned long long)score);
            }
        }
        p.cand_cnt[r] = (uint32_t)nc;
    }
}

// ---------------------------------------------------------------------------------------------
// launchers

int launch_sketch(const SketchParams& p, void* stream) {
    if (p.n == 0) return 0;
    const dim3 grid((unsigned)((p.n + WG - 1) / WG));
    const size_t lds = sketch_lds_bytes(p.nk, p.tile_chunks, p.hcap);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (lds > 160 * 1024) return -1;
    auto go = [&](auto kern) {
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, grid, dim3(WG), lds, s, p);
    };
    switch (p.hcap) {
    case 16: go(k_sketch<16>); break;
    case 32: go(k_sketch<32>); break;
    case 64: go(k_sketch<64>); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_sketch_slow(const SketchParams& p, void* stream) {
    if (p.n == 0) return 0;
    hipLaunchKernelGGL(k_sketch_slow, dim3(256), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_chain(const ChainParams& p, void* stream) {
    if (p.n == 0) return 0;
    const dim3 grid((unsigned)((p.n + WG - 1) / WG));
    hipLaunchKernelGGL(k_chain, grid, dim3(WG), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_chain_slow(const ChainParams& p, void* stream) {
    if (p.n == 0) return 0;
    hipLaunchKernelGGL(k_chain_slow, dim3(256), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace skq
