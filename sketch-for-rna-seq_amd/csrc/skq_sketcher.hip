// skq_sketcher.hip — one sequence per call, for the reference's per-sequence call sites
// (src/main.cpp:79 index side, :143-144 read side: createSketch_FracMinhash_direct once per
// sequence per k, through the C++ drop-in include/dropin/sketch.h).
//
// A call cannot amortise a launch, so it is built to cost one: the caller's bytes go into pinned
// host memory the device maps, one kernel (one workgroup) stages them into LDS with 16-B loads
// over the link, rolls ntHash over the windows (skq_sketch_seqs semantics: windows holding a byte
// outside ACGTUacgtu are skipped, lowercase hashes like uppercase, U like T) and appends the
// retained hashes to mapped pinned memory, then the count last (after a system-scope fence); the
// host spins on that word instead of a stream synchronisation (the completion signal's round
// trip cost ~10 us a call). No device-side copies, no session, no export round trips.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "skq.h"
#include "skq_internal.h"

namespace {

int sfail(int code, const std::string& msg) {
    skq::set_error(code, msg.c_str());
    return code;
}

#define SHIP(expr)                                                                     \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) return sfail(-3, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

constexpr uint32_t SK_WG = 256;
constexpr uint32_t SK_LDS_MAX = 48 * 1024;  // sequences staged in LDS; longer ones are read in place

// bytes -> 2-bit code, 4 = a byte ntHash skips
__device__ __forceinline__ uint32_t sk_code(uint8_t b) {
    switch (b) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'T': case 't': case 'U': case 'u': return 2;
    case 'G': case 'g': return 3;
    default: return 4;
    }
}

// out[0] = retained windows, out[1 ..] = their hashes (up to cap; unordered, repeats kept)
__global__ __launch_bounds__(SK_WG) void k_sketch_one(const uint8_t* src, uint32_t len, uint32_t k, uint32_t thr,
                                                      uint32_t* out, uint32_t cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_seq[];
    __shared__ uint8_t s_code[256];
    __shared__ uint32_t s_cnt;
    const uint32_t t = threadIdx.x;
    s_code[t] = (uint8_t)sk_code((uint8_t)t);
    if (t == 0) s_cnt = 0;
    const bool staged = len <= SK_LDS_MAX;
    if (staged) {  // (the host buffer is 16-B aligned and padded to 16 B)
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
        uint4* d4 = reinterpret_cast<uint4*>(s_seq);
        for (uint32_t q = t; q < (len + 15) / 16; q += SK_WG) d4[q] = s4[q];
    }
    __syncthreads();
    const uint8_t* s = staged ? s_seq : src;
    const uint32_t nw = len >= k && k ? len - k + 1 : 0;
    // a chunk of windows per thread, rolled from its first base
    const uint32_t chunk = max(1u, (nw + SK_WG - 1) / SK_WG);
    uint64_t seed[4], rk[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        seed[c] = skq::SEED33[c];
        const uint32_t d = k % 33;
        rk[c] = d ? (((skq::SEED33[c] << d) | (skq::SEED33[c] >> (33 - d))) & skq::M33) : skq::SEED33[c];
    }
    for (uint32_t w0 = t * chunk; w0 < nw; w0 += SK_WG * chunk) {
        uint64_t h = 0;
        uint32_t run = 0;  // valid bases ending at p, counted from w0
        const uint32_t pend = min(len, w0 + chunk + k - 1);
        for (uint32_t p = w0; p < pend; ++p) {
            const uint32_t c = s_code[s[p]];
            if (c == 4) {
                run = 0;
                h = 0;
                continue;
            }
            ++run;
            h = ((h << 1) | (h >> 32)) & skq::M33;
            h ^= seed[c];
            if (run > k) h ^= rk[s_code[s[p - k]]];
            if (run >= k && (uint32_t)h <= thr) {  // src/sketch.cpp:33-35
                const uint32_t at = atomicAdd(&s_cnt, 1u);
                if (at < cap) out[1 + at] = (uint32_t)h;
            }
        }
    }
    __syncthreads();
    if (t == 0) {
        __threadfence_system();  // (the hashes reach the host before the count that releases them)
        __hip_atomic_store(out, s_cnt, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

constexpr uint32_t SK_PENDING = 0xFFFFFFFFu;  // out[0] until the kernel's count lands

}  // namespace

struct skq_sketcher {
    int device = 0;
    hipStream_t st = nullptr;
    uint64_t cap_len = 0;   // bytes the pinned input holds
    uint8_t* hin = nullptr;  // pinned, mapped: the sequence
    uint32_t* hout = nullptr;  // pinned, mapped: [count, hashes...], cap_len + 1 words
    uint8_t* din = nullptr;   // device views of the two
    uint32_t* dout = nullptr;
};

namespace {

void release(skq_sketcher* h) {
    if (h->hin) (void)hipHostFree(h->hin);
    if (h->hout) (void)hipHostFree(h->hout);
    h->hin = nullptr;
    h->hout = nullptr;
    h->din = nullptr;
    h->dout = nullptr;
    h->cap_len = 0;
}

int grow(skq_sketcher* h, uint64_t len) {
    if (len <= h->cap_len) return 0;
    release(h);
    const uint64_t cap = std::max<uint64_t>(4096, (len + 4095) & ~4095ull);
    // coherent: the device reads the host's bytes and the host reads the device's words with no
    // cache maintenance between them
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    SHIP(hipHostMalloc(reinterpret_cast<void**>(&h->hin), cap + 16, fl));
    SHIP(hipHostMalloc(reinterpret_cast<void**>(&h->hout), (cap + 1) * 4, fl));
    SHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->din), h->hin, 0));
    SHIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->dout), h->hout, 0));
    h->cap_len = cap;
    return 0;
}

}  // namespace

int skq_sketcher_create(int device, uint64_t max_len, skq_sketcher** out) {
    if (!out) return sfail(-1, "null argument");
    *out = nullptr;
    int prev = 0;
    SHIP(hipGetDevice(&prev));
    SHIP(hipSetDevice(device));
    skq_sketcher* h = new skq_sketcher();
    h->device = device;
    int rc = 0;
    if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) rc = sfail(-3, "stream creation failed");
    if (!rc) rc = grow(h, max_len);
    if (!rc && hipFuncSetAttribute(reinterpret_cast<const void*>(k_sketch_one), hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)SK_LDS_MAX) != hipSuccess)
        rc = sfail(-3, "LDS attribute failed");
    (void)hipSetDevice(prev);
    if (rc) {
        skq_sketcher_free(h);
        return rc;
    }
    *out = h;
    return 0;
}

int skq_sketcher_run(skq_sketcher* h, const char* seq, uint64_t len, uint32_t k, uint32_t threshold, uint32_t* hashes,
                     uint64_t cap, uint64_t* count) {
    if (!h || (!seq && len) || !count) return sfail(-1, "null argument");
    if (len > 0xFFFFFFF0ull) return sfail(-1, "sequence too long for skq_sketcher_run");
    int prev = 0;
    SHIP(hipGetDevice(&prev));
    if (prev != h->device) SHIP(hipSetDevice(h->device));
    int rc = grow(h, len);
    if (!rc) {
        if (len) std::memcpy(h->hin, seq, len);
        const uint64_t nw = len >= k && k ? len - k + 1 : 0;
        const size_t lds = len <= SK_LDS_MAX ? (size_t)((len + 15) & ~15ull) : 0;
        __atomic_store_n(h->hout, SK_PENDING, __ATOMIC_RELEASE);
        hipLaunchKernelGGL(k_sketch_one, dim3(1), dim3(SK_WG), lds, h->st, h->din, (uint32_t)len, k, threshold, h->dout,
                           (uint32_t)std::min<uint64_t>(nw, h->cap_len));
        bool ok = hipGetLastError() == hipSuccess;
        // the count word, polled (a bounded spin: the stream's own completion settles the rest)
        uint32_t c = SK_PENDING;
        for (int spin = 0; ok && spin < (1 << 16) && (c = __atomic_load_n(h->hout, __ATOMIC_ACQUIRE)) == SK_PENDING; ++spin)
            __builtin_ia32_pause();
        if (ok && c == SK_PENDING) ok = hipStreamSynchronize(h->st) == hipSuccess;
        if (!ok) {
            rc = sfail(-3, "sketcher kernel failed");
        } else {
            const uint64_t n = __atomic_load_n(h->hout, __ATOMIC_ACQUIRE);
            *count = n;
            if (hashes && cap) std::memcpy(hashes, h->hout + 1, std::min(n, cap) * 4);
        }
    }
    if (prev != h->device) (void)hipSetDevice(prev);
    return rc;
}

int skq_sketcher_free(skq_sketcher* h) {
    if (!h) return 0;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(h->device);
    if (h->st) (void)hipStreamSynchronize(h->st);
    release(h);
    if (h->st) (void)hipStreamDestroy(h->st);
    (void)hipSetDevice(prev);
    delete h;
    return 0;
}
