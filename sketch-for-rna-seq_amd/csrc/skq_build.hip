// skq_build.hip — the index side on the GPU: build_and_save_index's per-transcript sketches and
// build_kmer_to_transcript_map (reference src/main.cpp:66-85, src/sketch.cpp:51-74), the same
// tables skq_tables_build makes on host threads (skq_tables.cpp), bit for bit.
//
// Per distinct k, one workgroup of 64 lanes per transcript, each lane a chunk of 64 windows:
// the lane rolls ntHash's 33-bit lane from its chunk's first base (windows holding a byte outside
// ACGTUacgtu are skipped, as ntHash skips them; lowercase hashes like uppercase), counts the
// windows at or below the threshold, reserves room for them with one atomic per wave, then rolls
// again and writes (hash << 32 | transcript) words. A radix sort of the words gives the
// inverted index in key order; duplicates (a hash seen twice in one transcript) fall out when
// the CSR is formed on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>
#include <string>
#include <vector>

#include "skq_host.h"
#include "skq_internal.h"

namespace {

constexpr uint32_t CHUNK = 64;  // windows per lane

int bfail(int code, const std::string& msg) {
    skq::set_error(code, msg.c_str());
    return code;
}

#define BHIP(expr)                                                                     \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) return bfail(-3, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
struct DBuf {
    T* p = nullptr;
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(uint64_t n) {
        if (p) (void)hipFree(p);
        p = nullptr;
        return hipMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(n, 1) * sizeof(T));
    }
};

// byte -> 2-bit code (A/a 0, C/c 1, T/t/U/u 2, G/g 3), 4 = a byte ntHash skips
__device__ __forceinline__ uint32_t code_of(uint8_t b) {
    switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'T': case 't': case 'U': case 'u': return 2;
    case 'G': case 'g': return 3;
    default: return 4;
    }
}

// windows [w0, w0 + CHUNK) of sequence s (length len) at k: calls f(hash) for each retained one
template <typename F>
__device__ __forceinline__ void roll_chunk(const uint8_t* s, uint64_t len, uint32_t k, uint64_t w0, uint32_t thr,
                                           const uint64_t (&seed)[4], const uint64_t (&rk)[4], F&& f) {
    uint64_t h = 0;
    uint32_t run = 0;  // valid bases ending at p, counted from w0
    const uint64_t pend = min(len, w0 + CHUNK + k - 1);
    for (uint64_t p = w0; p < pend; ++p) {
        const uint32_t c = code_of(s[p]);
        if (c == 4) {
            run = 0;
            h = 0;
            continue;
        }
        ++run;
        h = ((h << 1) | (h >> 32)) & skq::M33;
        h ^= seed[c];
        if (run > k) h ^= rk[code_of(s[p - k])];
        if (run >= k && (uint32_t)h <= thr) f((uint32_t)h);
    }
}

__global__ __launch_bounds__(64) void k_tx_sketch(const uint8_t* seqs, const uint64_t* offs, uint32_t ntx,
                                                  uint32_t k, uint32_t maxk, uint32_t thr, uint64_t* words,
                                                  uint64_t cap, unsigned long long* used) {
    const uint32_t t = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const uint64_t a = offs[t], len = offs[t + 1] - a;
    if (len < maxk) return;  // shorter than some k: not indexed (src/main.cpp:66-75); block-uniform
    const uint8_t* s = seqs + a;
    uint64_t seed[4], rk[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        seed[c] = skq::SEED33[c];
        const uint32_t d = k % 33;  // rot33 (skq_internal.h), on the device
        rk[c] = d ? (((skq::SEED33[c] << d) | (skq::SEED33[c] >> (33 - d))) & skq::M33) : skq::SEED33[c];
    }
    const uint64_t nw = len - k + 1;
    const uint64_t nch = (nw + CHUNK - 1) / CHUNK;
    for (uint64_t c0 = 0; c0 < nch; c0 += 64) {  // block-uniform
        const uint64_t ch = c0 + lane;
        uint32_t n = 0;
        if (ch < nch) roll_chunk(s, len, k, ch * CHUNK, thr, seed, rk, [&](uint32_t) { ++n; });
        // one reservation per wave
        uint32_t incl = n;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t v = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += v;
        }
        const uint32_t tot = __shfl(incl, 63, 64);
        unsigned long long base = 0;
        if (lane == 63 && tot) base = atomicAdd(used, (unsigned long long)tot);
        base = __shfl(base, 63, 64);
        uint64_t at = base + incl - n;
        if (ch < nch && n)
            roll_chunk(s, len, k, ch * CHUNK, thr, seed, rk, [&](uint32_t h) {
                if (at < cap) words[at] = ((uint64_t)h << 32) | t;
                ++at;
            });
    }
}

}  // namespace

extern "C" int skq_tables_build_gpu(int device, uint32_t ntx, const uint8_t* seqs, const uint64_t* offs, uint32_t nk,
                                    const uint32_t* ks, uint32_t threshold, skq_tables** out) {
    if (!out || (ntx && (!seqs || !offs)) || (nk && !ks)) return bfail(-1, "null argument");
    *out = nullptr;
    if (nk == 0 || nk > SKQ_MAX_K) return bfail(-1, "k list must hold 1..SKQ_MAX_K entries");
    std::vector<uint32_t> dk;  // distinct ks, first-seen order (as skq_tables_build)
    uint32_t maxk = 0;
    for (uint32_t i = 0; i < nk; ++i) {
        if (ks[i] == 0) return bfail(-1, "k must be greater than 0");
        maxk = std::max(maxk, ks[i]);
        if (std::find(dk.begin(), dk.end(), ks[i]) == dk.end()) dk.push_back(ks[i]);
    }
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return bfail(-2, "no such device");
    int prev = -1;
    (void)hipGetDevice(&prev);
    BHIP(hipSetDevice(device));
    struct Restore {
        int d;
        ~Restore() {
            if (d >= 0) (void)hipSetDevice(d);
        }
    } restore{prev};
    const uint64_t nbytes = ntx ? offs[ntx] : 0;
    uint64_t windows = 0;
    for (uint32_t t = 0; t < ntx; ++t) {
        const uint64_t len = offs[t + 1] - offs[t];
        if (len >= maxk) windows += len;
    }
    if (ntx >= (1u << 31)) return bfail(-1, "too many transcripts");
    DBuf<uint8_t> d_seq;
    DBuf<uint64_t> d_offs, words, sorted;
    DBuf<unsigned long long> used;
    DBuf<unsigned char> tmp;
    BHIP(d_seq.alloc(nbytes + 1));
    BHIP(d_offs.alloc((uint64_t)ntx + 1));
    BHIP(used.alloc(1));
    if (nbytes) BHIP(hipMemcpy(d_seq.p, seqs, nbytes, hipMemcpyHostToDevice));
    BHIP(hipMemcpy(d_offs.p, offs, ((uint64_t)ntx + 1) * 8, hipMemcpyHostToDevice));
    // room for ~6.25 % of the windows (5 % are retained on average at the reference's 0.05); a
    // transcriptome that retains more is re-run with the exact count
    uint64_t cap = windows / 16 + (1u << 20);
    std::vector<std::vector<uint64_t>> tabs(dk.size());
    for (size_t d = 0; d < dk.size(); ++d) {
        unsigned long long n = 0;
        for (int attempt = 0; attempt < 2; ++attempt) {
            BHIP(words.alloc(cap));
            BHIP(hipMemset(used.p, 0, 8));
            if (ntx) {
                hipLaunchKernelGGL(k_tx_sketch, dim3(ntx), dim3(64), 0, nullptr, d_seq.p, d_offs.p, ntx, dk[d], maxk,
                                   threshold, words.p, cap, used.p);
                BHIP(hipGetLastError());
            }
            BHIP(hipMemcpy(&n, used.p, 8, hipMemcpyDeviceToHost));
            if (n <= cap) break;
            cap = n;
        }
        if (n >= 0x7FFFFFFFull) return bfail(-1, "too many retained hashes for one sort");
        BHIP(sorted.alloc(n));
        size_t tb = 0;
        BHIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, words.p, sorted.p, (int)n, 0, 64, nullptr));
        BHIP(tmp.alloc(tb + 1));
        BHIP(hipcub::DeviceRadixSort::SortKeys(tmp.p, tb, words.p, sorted.p, (int)n, 0, 64, nullptr));
        tabs[d].resize(n);
        if (n) BHIP(hipMemcpy(tabs[d].data(), sorted.p, n * 8, hipMemcpyDeviceToHost));
    }
    return skq::tables_from_words((uint32_t)dk.size(), dk.data(), tabs.data(), out);
}
