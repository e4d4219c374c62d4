// skq_em.hip — EM and read assignment on the GPU: estimate_isoform_abundance_em and
// assign_reads_to_isoforms (src/isoform_assignment.cpp:9-97) over the reads' candidate lists
// that sparse_chain produced.
//
// Reads are appended as they are chained, straight from a session's device results
// (skq_em_add_session) or from host CSR arrays (skq_em_add); skq_em_select then drops the reads
// the reference never sees (invalid, short, earlier duplicates of an id). Before the first round
// the kept reads are laid out once, on the device:
//   * reads with at least one candidate, ordered by their first (best) candidate with a stable
//     radix sort, so the reads of one gene sit together; read-major CSR roff / rtid / rsc;
//   * the same entries transcript-major: toff[t], tent = (score, position), positions ascending
//     within a transcript (stable sort by transcript over the read-major order).
// One EM round:
//   k_em_den    lane per read: den = sum of pi[t] * score over its candidates, in list order;
//               w = 1 / den where den > 1e-10 (src/isoform_assignment.cpp:31-44), else 0
//   k_em_sum    16 lanes per transcript: post[t] = sum over its entries of (pi[t] * score) * w,
//               each lane in entry order, then a fixed xor tree: the same sums on every run
//   (several GPUs: the caller all-reduces post here; skq/dist.py)
//   k_em_mstep  pi[t] = (post[t] + (double)(0.01f / R)) + (double)0.01f (:54-59) and
//               |new - old| per workgroup; k_em_change adds the partials in a fixed order
// Assignment (:70-97) is the same pair of passes with w = den where den > 0 and the share
// (pi[t] * score) / den, and marks every transcript that received a share.
// The gathers of pi (ntx doubles) hit L2; the position-sorted layout keeps k_em_sum's gathers of
// w local, so a round streams the candidate lists twice (~16 B per candidate).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <hipcub/hipcub.hpp>
#include <string>
#include <vector>

#include "skq_internal.h"

namespace {

constexpr int EWG = 256;
constexpr int TPT = 16;  // lanes per transcript in k_em_sum

int efail(int code, const std::string& msg) {
    skq::set_error(code, msg.c_str());
    return code;
}

#define EHIP(expr)                                                                     \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) return efail(-3, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct EDeviceGuard {
    int prev = -1;
    explicit EDeviceGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~EDeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <typename T>
struct Buf {
    T* p = nullptr;
    uint64_t cap = 0;
    ~Buf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // grows to at least n elements keeping the first `keep` (device to device); the old block
    // is freed only after the device has drained (work in flight may still use it)
    hipError_t reserve(uint64_t n, uint64_t keep = 0) {
        if (n <= cap) return hipSuccess;
        const uint64_t nc = std::max<uint64_t>(n, cap + cap / 2);
        if (p) {
            const hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) return e;
        }
        T* q = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&q), std::max<uint64_t>(nc, 1) * sizeof(T));
        if (e != hipSuccess) return e;
        if (keep && p) {
            e = hipMemcpy(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice);
            if (e != hipSuccess) {
                (void)hipFree(q);
                return e;
            }
        }
        release();
        p = q;
        cap = nc;
        return hipSuccess;
    }
};

inline unsigned blocks(uint64_t n, unsigned wg) { return (unsigned)std::max<uint64_t>(1, (n + wg - 1) / wg); }
inline int key_bits(uint32_t maxkey) { return std::max(1, 32 - __builtin_clz(maxkey | 1u)); }

// ---- appending ----------------------------------------------------------------------------------

// session results -> counts of a batch (padded rows with ext overflow, or the packed layout's
// runs: cand_cnt = 0x80000000 | pair offset of [count, 0], skq.h)
__global__ void k_em_cnt(uint64_t n, uint32_t packed, const uint32_t* cand_cnt, const uint32_t* cand_ext,
                         uint64_t* cnt) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) {
        const uint32_t c = cand_cnt[r];
        cnt[r] = packed && (c & 0x80000000u) ? cand_ext[2ull * (c & 0x7FFFFFFFu)] : c;
    }
    if (r == n) cnt[n] = 0;
}

// copies read r's candidates to tid[offs[r]..], score[offs[r]..] (offs absolute); packed layout:
// a wave (64 consecutive reads from a multiple of 64: EWG is) scans its counts for the offsets
__global__ void k_em_gather(uint64_t n, uint32_t ccap, uint32_t packed, const uint32_t* cand_cnt,
                            const uint32_t* cand_tid, const uint32_t* cand_score, const uint32_t* cand_ext,
                            const uint64_t* offs, uint32_t* tid, uint32_t* score) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (packed) {
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t c = r < n ? cand_cnt[r] : 0u;
        const bool run = (c & 0x80000000u) != 0;
        const uint32_t m = run ? 0u : c;
        uint32_t incl = m;  // inclusive scan over the wave
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (r >= n) return;
        const uint64_t o = offs[r];
        if (run) {
            const uint32_t* e = cand_ext + 2ull * (c & 0x7FFFFFFFu);
            const uint32_t k = e[0];
            for (uint32_t j = 0; j < k; ++j) {
                tid[o + j] = e[2 * (j + 1)];
                score[o + j] = e[2 * (j + 1) + 1];
            }
        } else {
            const uint32_t* w = cand_tid + (r - lane) * ccap + (incl - m);
            for (uint32_t j = 0; j < m; ++j) {
                tid[o + j] = w[j] & 0x3FFFFFu;
                score[o + j] = w[j] >> 22;
            }
        }
        return;
    }
    if (r >= n) return;
    const uint32_t c = cand_cnt[r];
    const uint64_t o = offs[r];
    if (c <= ccap) {
        for (uint32_t j = 0; j < c; ++j) {
            tid[o + j] = cand_tid[(uint64_t)j * n + r];
            score[o + j] = cand_score[(uint64_t)j * n + r];
        }
    } else {
        const uint32_t* e = cand_ext + 2ull * cand_tid[r];
        for (uint32_t j = 0; j < c; ++j) {
            tid[o + j] = e[2 * j];
            score[o + j] = e[2 * j + 1];
        }
    }
}

__global__ void k_em_shift(uint64_t n, uint64_t* offs, uint64_t base) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r <= n) offs[r] += base;
}

// ---- layout -------------------------------------------------------------------------------------

// sort key of read r: its first candidate, or ntx (sorted last, left out) for reads without
// candidates and reads not kept; cnt[0] += kept reads with candidates
__global__ void k_em_keys(uint64_t n, const uint64_t* offs, const uint32_t* tid, const uint8_t* keep, uint32_t ntx,
                          uint32_t* key, uint32_t* val, uint32_t* cnt) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool in = false;
    if (r < n) {
        const uint64_t a = offs[r], b = offs[r + 1];
        in = b > a && (!keep || keep[r]);
        key[r] = in ? min(tid[a], ntx - 1) : ntx;
        val[r] = (uint32_t)r;
    }
    const uint64_t bal = __ballot(in);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(cnt, (uint32_t)__builtin_popcountll(bal));
}

__global__ void k_em_len(uint32_t m, const uint32_t* order, const uint64_t* offs, uint64_t* len) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < m) {
        const uint32_t r = order[p];
        len[p] = offs[r + 1] - offs[r];
    } else if (p == m) {
        len[m] = 0;
    }
}

// read-major copy in sorted order, the transcript-major sort input and per-transcript counts;
// err |= 1 for a transcript id out of range
__global__ void k_em_copy(uint32_t m, const uint32_t* order, const uint64_t* offs, const uint32_t* tid,
                          const uint32_t* score, const uint64_t* roff, uint32_t ntx, uint32_t* rtid, uint32_t* rsc,
                          uint32_t* tkey, uint64_t* tval, uint32_t* tcnt, uint32_t* err) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m) return;
    const uint32_t r = order[p];
    const uint64_t a = offs[r], b = offs[r + 1], o = roff[p];
    for (uint64_t j = 0; j < b - a; ++j) {
        uint32_t t = tid[a + j];
        const uint32_t s = score[a + j];
        if (t >= ntx) {
            atomicOr(err, 1u);
            t = 0;
        }
        rtid[o + j] = t;
        rsc[o + j] = s;
        tkey[o + j] = t;
        tval[o + j] = ((uint64_t)p << 32) | s;
        atomicAdd(&tcnt[t], 1u);
    }
}

__global__ void k_em_widen(uint32_t n, const uint32_t* c, uint64_t* w) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) w[t] = c[t];
    if (t == n) w[n] = 0;
}

// ---- rounds -------------------------------------------------------------------------------------

__global__ __launch_bounds__(EWG) void k_em_fill(uint32_t n, double v, double* x) {
    const uint32_t t = blockIdx.x * EWG + threadIdx.x;
    if (t < n) x[t] = v;
}

template <bool ASSIGN>
__global__ __launch_bounds__(EWG) void k_em_den(uint32_t m, const uint64_t* roff, const uint32_t* rtid,
                                                const uint32_t* rsc, const double* pi, double* w) {
    const uint32_t p = blockIdx.x * EWG + threadIdx.x;
    if (p >= m) return;
    double den = 0.0;
    for (uint64_t c = roff[p], e = roff[p + 1]; c < e; ++c) den += pi[rtid[c]] * (double)rsc[c];
    if (ASSIGN) w[p] = den > 0.0 ? den : 0.0;       // total_probability > 0.0 (:89)
    else w[p] = den > 1e-10 ? 1.0 / den : 0.0;      // denominator > epsilon (:43-44)
}

template <bool ASSIGN>
__global__ __launch_bounds__(EWG) void k_em_sum(uint32_t ntx, const uint64_t* toff, const uint2* tent,
                                                const double* pi, const double* w, double* post, uint8_t* assigned) {
    const uint32_t g = (blockIdx.x * EWG + threadIdx.x) / TPT, j = threadIdx.x % TPT;
    const bool live = g < ntx;
    double acc = 0.0;
    bool any = false;
    if (live) {
        const double pt = pi[g];
        for (uint64_t i = toff[g] + j, e = toff[g + 1]; i < e; i += TPT) {
            const uint2 q = tent[i];  // x = score, y = read position
            const double wp = w[q.y];
            if (wp != 0.0) {
                const double num = pt * (double)q.x;
                acc += ASSIGN ? num / wp : num * wp;
                any = true;
            }
        }
    }
#pragma unroll
    for (int o = TPT / 2; o; o >>= 1) acc += __shfl_xor(acc, o, TPT);
    const uint64_t bal = __ballot(any);
    const uint32_t lane = threadIdx.x & 63u;
    if (live && j == 0) {
        post[g] = acc;
        if (ASSIGN) assigned[g] = ((bal >> (lane & ~(uint32_t)(TPT - 1))) & ((1ull << TPT) - 1)) ? 1 : 0;
    }
}

__global__ __launch_bounds__(EWG) void k_em_mstep(uint32_t ntx, double* pi, const double* post, double a, double b,
                                                  double* partial) {
    __shared__ double s[EWG];
    const uint32_t t = blockIdx.x * EWG + threadIdx.x;
    double d = 0.0;
    if (t < ntx) {
        const double np = (post[t] + a) + b;
        d = fabs(np - pi[t]);
        pi[t] = np;
    }
    s[threadIdx.x] = d;
    __syncthreads();
#pragma unroll
    for (int o = EWG / 2; o; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(EWG) void k_em_change(uint32_t nb, const double* partial, double* out) {
    __shared__ double s[EWG];
    double d = 0.0;
    for (uint32_t i = threadIdx.x; i < nb; i += EWG) d += partial[i];
    s[threadIdx.x] = d;
    __syncthreads();
#pragma unroll
    for (int o = EWG / 2; o; o >>= 1) {
        if ((int)threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = s[0];
}

}  // namespace

struct skq_em_set {
    int device = 0;
    uint32_t ntx = 0;
    // appended reads (raw, in arrival order): offs[n + 1], tid / score [offs[n]]
    uint64_t n = 0;
    Buf<uint64_t> offs;
    Buf<uint32_t> tid, score;
    Buf<uint8_t> keep;
    bool selected = false;
    uint64_t R = 0;  // reads the reference's EM sees (kept, with or without candidates)
    // layout (built on first use)
    bool built = false;
    uint32_t m = 0;  // kept reads with candidates
    uint64_t nc = 0;
    Buf<uint64_t> roff, toff;
    Buf<uint32_t> rtid, rsc;
    Buf<uint64_t> tent;
    // round state
    Buf<double> w, pi, post, partial, change;
    Buf<uint8_t> assigned;
    Buf<unsigned char> tmp;  // hipcub
};

namespace {

template <typename F>
int cub_call(skq_em_set* em, F&& f) {
    size_t bytes = 0;
    EHIP(f(nullptr, bytes));
    EHIP(em->tmp.reserve(bytes + 1));
    size_t b = em->tmp.cap;
    EHIP(f(em->tmp.p, b));
    return 0;
}

int build(skq_em_set* em, hipStream_t st) {
    if (em->built) return 0;
    EDeviceGuard g(em->device);
    const uint64_t n = em->n;
    if (!em->selected) em->R = n;
    if (n >= 0x7FFFFFF0ull) return efail(-1, "more than 2^31 reads in one EM set");
    EHIP(em->offs.reserve(n + 1, n + 1));
    if (n == 0) EHIP(hipMemsetAsync(em->offs.p, 0, 8, st));
    Buf<uint32_t> k0, k1, v0, v1, cnt;
    EHIP(k0.reserve(n + 1));
    EHIP(k1.reserve(n + 1));
    EHIP(v0.reserve(n + 1));
    EHIP(v1.reserve(n + 1));
    EHIP(cnt.reserve(2));
    EHIP(hipMemsetAsync(cnt.p, 0, 8, st));
    k_em_keys<<<blocks(n, EWG), EWG, 0, st>>>(n, em->offs.p, em->tid.p, em->selected ? em->keep.p : nullptr,
                                              em->ntx, k0.p, v0.p, cnt.p);
    EHIP(hipGetLastError());
    if (n) {
        const int bits = key_bits(em->ntx);
        if (int rc = cub_call(em, [&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, k0.p, k1.p, v0.p, v1.p, (int)n, 0, bits, st);
            }))
            return rc;
    }
    uint32_t m = 0;
    EHIP(hipMemcpyAsync(&m, cnt.p, 4, hipMemcpyDeviceToHost, st));
    EHIP(hipStreamSynchronize(st));
    em->m = m;
    Buf<uint64_t> len;
    EHIP(len.reserve((uint64_t)m + 1));
    EHIP(em->roff.reserve((uint64_t)m + 1));
    k_em_len<<<blocks((uint64_t)m + 1, EWG), EWG, 0, st>>>(m, v1.p, em->offs.p, len.p);
    EHIP(hipGetLastError());
    if (int rc = cub_call(em, [&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveSum(t, b, len.p, em->roff.p, (int)(m + 1), st);
        }))
        return rc;
    uint64_t nc = 0;
    EHIP(hipMemcpyAsync(&nc, em->roff.p + m, 8, hipMemcpyDeviceToHost, st));
    EHIP(hipStreamSynchronize(st));
    if (nc >= 0x7FFFFFF0ull) return efail(-1, "more than 2^31 candidates in one EM set");
    em->nc = nc;
    len.release();
    k0.release();
    k1.release();
    v0.release();
    Buf<uint32_t> tkey, tkey2, tcnt;
    Buf<uint64_t> tval;
    EHIP(em->rtid.reserve(nc + 1));
    EHIP(em->rsc.reserve(nc + 1));
    EHIP(em->tent.reserve(nc + 1));
    EHIP(tkey.reserve(nc + 1));
    EHIP(tkey2.reserve(nc + 1));
    EHIP(tval.reserve(nc + 1));
    EHIP(tcnt.reserve((uint64_t)em->ntx + 1));
    EHIP(em->toff.reserve((uint64_t)em->ntx + 1));
    EHIP(hipMemsetAsync(tcnt.p, 0, ((uint64_t)em->ntx + 1) * 4, st));
    EHIP(hipMemsetAsync(cnt.p, 0, 4, st));
    k_em_copy<<<blocks(m, EWG), EWG, 0, st>>>(m, v1.p, em->offs.p, em->tid.p, em->score.p, em->roff.p, em->ntx,
                                              em->rtid.p, em->rsc.p, tkey.p, tval.p, tcnt.p, cnt.p);
    EHIP(hipGetLastError());
    if (nc) {
        const int bits = key_bits(em->ntx - 1);
        if (int rc = cub_call(em, [&](void* t, size_t& b) {
                return hipcub::DeviceRadixSort::SortPairs(t, b, tkey.p, tkey2.p, tval.p, em->tent.p, (int)nc, 0, bits,
                                                          st);
            }))
            return rc;
    }
    Buf<uint64_t> tcnt64;
    EHIP(tcnt64.reserve((uint64_t)em->ntx + 1));
    k_em_widen<<<blocks((uint64_t)em->ntx + 1, EWG), EWG, 0, st>>>(em->ntx, tcnt.p, tcnt64.p);
    EHIP(hipGetLastError());
    if (int rc = cub_call(em, [&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveSum(t, b, tcnt64.p, em->toff.p, (int)(em->ntx + 1), st);
        }))
        return rc;
    uint32_t err = 0;
    EHIP(hipMemcpyAsync(&err, cnt.p, 4, hipMemcpyDeviceToHost, st));
    EHIP(hipStreamSynchronize(st));
    if (err) return efail(-1, "candidate transcript id out of range");
    const uint64_t nt = em->ntx;
    EHIP(em->w.reserve((uint64_t)m + 1));
    EHIP(em->pi.reserve(nt));
    EHIP(em->post.reserve(nt));
    EHIP(em->partial.reserve(blocks(nt, EWG)));
    EHIP(em->change.reserve(1));
    EHIP(em->assigned.reserve(nt));
    em->built = true;
    return 0;
}

int estep(skq_em_set* em, const double* pi, double* post, bool assign, uint8_t* assigned, hipStream_t st) {
    if (int rc = build(em, st)) return rc;
    EDeviceGuard g(em->device);
    if (assign) k_em_den<true><<<blocks(em->m, EWG), EWG, 0, st>>>(em->m, em->roff.p, em->rtid.p, em->rsc.p, pi, em->w.p);
    else k_em_den<false><<<blocks(em->m, EWG), EWG, 0, st>>>(em->m, em->roff.p, em->rtid.p, em->rsc.p, pi, em->w.p);
    EHIP(hipGetLastError());
    const uint64_t lanes = (uint64_t)em->ntx * TPT;
    const uint2* te = reinterpret_cast<const uint2*>(em->tent.p);
    if (assign)
        k_em_sum<true><<<blocks(lanes, EWG), EWG, 0, st>>>(em->ntx, em->toff.p, te, pi, em->w.p, post, assigned);
    else k_em_sum<false><<<blocks(lanes, EWG), EWG, 0, st>>>(em->ntx, em->toff.p, te, pi, em->w.p, post, nullptr);
    EHIP(hipGetLastError());
    return 0;
}

}  // namespace

extern "C" {

int skq_em_create(int device, uint32_t ntx, skq_em_set** out) {
    if (!out) return efail(-1, "null argument");
    if (ntx == 0) return efail(-1, "EM needs at least one transcript");
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return efail(-2, "no such device");
    skq_em_set* em = new skq_em_set;
    em->device = device;
    em->ntx = ntx;
    *out = em;
    return 0;
}

int skq_em_free(skq_em_set* em) {
    if (!em) return 0;
    EDeviceGuard g(em->device);
    delete em;
    return 0;
}

static int append_prepare(skq_em_set* em, uint64_t n) {
    if (em->built || em->selected) return efail(-1, "EM set already selected or in use: no more reads");
    EHIP(em->offs.reserve(em->n + n + 1, em->n + (em->n ? 1 : 0)));
    if (em->n == 0) EHIP(hipMemset(em->offs.p, 0, 8));
    return 0;
}

int skq_em_add(skq_em_set* em, uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
               const uint32_t* cand_score) {
    if (!em || (nreads && !cand_offs)) return efail(-1, "null argument");
    if (nreads == 0) return 0;
    EDeviceGuard g(em->device);
    const uint64_t c0 = cand_offs[0], nc = cand_offs[nreads] - c0;
    if (nc && (!cand_tid || !cand_score)) return efail(-1, "null argument");
    if (int rc = append_prepare(em, nreads)) return rc;
    uint64_t base = 0;
    if (em->n) EHIP(hipMemcpy(&base, em->offs.p + em->n, 8, hipMemcpyDeviceToHost));
    std::vector<uint64_t> o(nreads);
    for (uint64_t r = 0; r < nreads; ++r) o[r] = base + (cand_offs[r + 1] - c0);
    EHIP(em->tid.reserve(base + nc, base));
    EHIP(em->score.reserve(base + nc, base));
    EHIP(hipMemcpy(em->offs.p + em->n + 1, o.data(), nreads * 8, hipMemcpyHostToDevice));
    if (nc) {
        EHIP(hipMemcpy(em->tid.p + base, cand_tid + c0, nc * 4, hipMemcpyHostToDevice));
        EHIP(hipMemcpy(em->score.p + base, cand_score + c0, nc * 4, hipMemcpyHostToDevice));
    }
    em->n += nreads;
    return 0;
}

int skq_em_add_session(skq_em_set* em, skq_session* s, void* stream) {
    if (!em || !s) return efail(-1, "null argument");
    skq_results res{};
    if (int rc = skq::session_results(s, &res, false)) return rc;
    if (skq::session_device(s) != em->device) return efail(-1, "session and EM set on different devices");
    if (res.ntx != em->ntx) return efail(-1, "session index and EM set disagree on the transcript count");
    const uint64_t n = res.n_reads;
    if (n == 0) return 0;
    EDeviceGuard g(em->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (int rc = append_prepare(em, n)) return rc;
    uint64_t base = 0;
    if (em->n) EHIP(hipMemcpy(&base, em->offs.p + em->n, 8, hipMemcpyDeviceToHost));
    Buf<uint64_t> cnt;
    EHIP(cnt.reserve(n + 1));
    k_em_cnt<<<blocks(n + 1, EWG), EWG, 0, st>>>(n, res.cand_layout, res.cand_cnt, res.cand_ext, cnt.p);
    EHIP(hipGetLastError());
    uint64_t* dst = em->offs.p + em->n;  // exclusive sum of n + 1 counts over [n .. n + n]
    if (int rc = cub_call(em, [&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveSum(t, b, cnt.p, dst, (int)(n + 1), st);
        }))
        return rc;
    k_em_shift<<<blocks(n + 1, EWG), EWG, 0, st>>>(n, dst, base);
    EHIP(hipGetLastError());
    uint64_t end = 0;
    EHIP(hipMemcpyAsync(&end, dst + n, 8, hipMemcpyDeviceToHost, st));
    EHIP(hipStreamSynchronize(st));
    EHIP(em->tid.reserve(end + 1, base));
    EHIP(em->score.reserve(end + 1, base));
    static_assert(EWG % 64 == 0, "k_em_gather's packed scan: whole waves of aligned reads");
    k_em_gather<<<blocks(n, EWG), EWG, 0, st>>>(n, res.ccap, res.cand_layout, res.cand_cnt, res.cand_tid,
                                                res.cand_score, res.cand_ext, dst, em->tid.p, em->score.p);
    EHIP(hipGetLastError());
    EHIP(hipStreamSynchronize(st));
    em->n += n;
    return 0;
}

uint64_t skq_em_size(const skq_em_set* em) { return em ? em->n : 0; }

int skq_em_select(skq_em_set* em, const uint8_t* keep) {
    if (!em || (em->n && !keep)) return efail(-1, "null argument");
    if (em->built || em->selected) return efail(-1, "EM set already selected or in use");
    EDeviceGuard g(em->device);
    uint64_t R = 0;
    for (uint64_t r = 0; r < em->n; ++r) R += keep[r] ? 1 : 0;
    EHIP(em->keep.reserve(em->n + 1));
    if (em->n) EHIP(hipMemcpy(em->keep.p, keep, em->n, hipMemcpyHostToDevice));
    em->R = R;
    em->selected = true;
    return 0;
}

uint64_t skq_em_reads(const skq_em_set* em) { return !em ? 0 : em->selected ? em->R : em->n; }

int skq_em_init(skq_em_set* em, double* d_pi, void* stream) {
    if (!em || !d_pi) return efail(-1, "null argument");
    EDeviceGuard g(em->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    k_em_fill<<<blocks(em->ntx, EWG), EWG, 0, st>>>(em->ntx, 1.0 / em->ntx, d_pi);  // uniform start (:17-20)
    EHIP(hipGetLastError());
    return 0;
}

int skq_em_estep(skq_em_set* em, const double* d_pi, double* d_post, void* stream) {
    if (!em || !d_pi || !d_post) return efail(-1, "null argument");
    return estep(em, d_pi, d_post, false, nullptr, reinterpret_cast<hipStream_t>(stream));
}

int skq_em_mstep(skq_em_set* em, double* d_pi, const double* d_post, uint64_t total_reads, double* change, void* stream) {
    if (!em || !d_pi || !d_post) return efail(-1, "null argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (int rc = build(em, st)) return rc;
    EDeviceGuard g(em->device);
    // the pseudocount is a float (:54-57): (posterior + 0.01f / R) + 0.01f
    const float pc = 0.01f;
    const double a = (double)(pc / (float)total_reads), b = (double)pc;  // (R = 0: inf, as the reference)
    const unsigned nb = blocks(em->ntx, EWG);
    k_em_mstep<<<nb, EWG, 0, st>>>(em->ntx, d_pi, d_post, a, b, em->partial.p);
    EHIP(hipGetLastError());
    k_em_change<<<1, EWG, 0, st>>>(nb, em->partial.p, em->change.p);
    EHIP(hipGetLastError());
    if (change) {
        EHIP(hipMemcpyAsync(change, em->change.p, 8, hipMemcpyDeviceToHost, st));
        EHIP(hipStreamSynchronize(st));
    }
    return 0;
}

int skq_em_run(skq_em_set* em, int max_iterations, double convergence, double* pi, int* iterations) {
    if (!em) return efail(-1, "null argument");
    hipStream_t st = nullptr;
    if (int rc = build(em, st)) return rc;
    EDeviceGuard g(em->device);
    if (int rc = skq_em_init(em, em->pi.p, st)) return rc;
    int it = 0;
    for (; it < max_iterations; ++it) {
        double change = 0.0;
        if (int rc = skq_em_estep(em, em->pi.p, em->post.p, st)) return rc;
        if (int rc = skq_em_mstep(em, em->pi.p, em->post.p, skq_em_reads(em), &change, st)) return rc;
        if (change < convergence) {  // (:62-64)
            ++it;
            break;
        }
    }
    if (pi) EHIP(hipMemcpy(pi, em->pi.p, (uint64_t)em->ntx * 8, hipMemcpyDeviceToHost));
    if (iterations) *iterations = it;
    return 0;
}

int skq_em_assign(skq_em_set* em, const double* d_pi, double* d_counts, uint8_t* d_assigned, void* stream) {
    if (!em || !d_pi || !d_counts || !d_assigned) return efail(-1, "null argument");
    return estep(em, d_pi, d_counts, true, d_assigned, reinterpret_cast<hipStream_t>(stream));
}

int skq_em_assign_host(skq_em_set* em, const double* pi, double* counts, uint8_t* assigned) {
    if (!em || !counts || !assigned) return efail(-1, "null argument");
    hipStream_t st = nullptr;
    if (int rc = build(em, st)) return rc;
    EDeviceGuard g(em->device);
    if (pi) EHIP(hipMemcpy(em->pi.p, pi, (uint64_t)em->ntx * 8, hipMemcpyHostToDevice));
    if (int rc = estep(em, em->pi.p, em->post.p, true, em->assigned.p, st)) return rc;
    EHIP(hipMemcpy(counts, em->post.p, (uint64_t)em->ntx * 8, hipMemcpyDeviceToHost));
    EHIP(hipMemcpy(assigned, em->assigned.p, em->ntx, hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"
