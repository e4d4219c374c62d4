// skq_sketcher.hip — one sequence per call, for the reference's per-sequence call sites
// (src/main.cpp:79 index side, :143-144 read side: createSketch_FracMinhash_direct once per
// sequence per k, through the C++ drop-in include/dropin/sketch.h).
//
// A call cannot amortise a launch, so it does not pay one: a resident single-workgroup server
// (k_sketch_server) waits on a mailbox in pinned host memory the device maps. The caller's bytes
// go into a mapped pinned buffer, the request word is bumped, the server stages the bytes into
// LDS with 16-B loads over the link, rolls ntHash over the windows (skq_sketch_seqs semantics:
// windows holding a byte outside ACGTUacgtu are skipped, lowercase hashes like uppercase, U like
// T), appends the retained hashes to mapped pinned memory and releases them with the done word
// (after a system-scope fence); the host spins on that word. The server leaves after 2 ms without
// a request (or when stopped), and the next call launches it again. No device-side copies, no
// session, no export round trips, no launch or stream synchronisation per call.
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
constexpr uint32_t SK_LDS_MAX = 48 * 1024;  // the LDS tile of a sequence's bytes

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

// the mailbox in pinned mapped host memory (coherent): the host posts a request by writing the
// parameters, then req (0: stop), in one 16-B word the server reads with one load (a request's
// parameters arrive with it: one link round trip, not five); the server answers with the hashes
// and count in out, then done = req, on a line of its own
struct alignas(64) SkMail {
    uint32_t req, len, k, thr;
    uint32_t pad0[12];
    uint32_t done, alive;
    uint32_t pad1[14];
};

__device__ __forceinline__ void sys_store(uint32_t* a, uint32_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// the mailbox word (req, len, k, thr): one 16-B load past the caches, waited on
__device__ __forceinline__ u32x4 mail_load(const SkMail* m) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(&m->req) : "memory");
    return v;
}

// idle time after which the server exits (s_memrealtime ticks at 100 MHz): 2 ms
constexpr uint64_t SK_IDLE = 200000;

// One resident workgroup serving the host's requests in order, one sequence each: out[0] =
// retained windows, out[1 ..] = their hashes (up to cap; unordered, repeats kept). It exits when
// the host posts request 0 or after SK_IDLE without a request (clearing alive first and looking once
// more, so a request posted meanwhile is still served), so the grid always drains. `last` is the
// request the host saw completed before this launch.
__global__ __launch_bounds__(SK_WG) void k_sketch_server(SkMail* m, const uint8_t* src, uint32_t* out, uint32_t last,
                                                          uint32_t ocap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_seq[];
    __shared__ uint8_t s_code[256];
    __shared__ uint32_t s_cnt, s_cmd[4];  // go, len, k, thr
    const uint32_t t = threadIdx.x;
    s_code[t] = (uint8_t)sk_code((uint8_t)t);
    for (;;) {
        if (t == 0) {
            bool go = false;
            u32x4 mb;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                mb = mail_load(m);
                if (mb.x != last) {
                    go = mb.x != 0;  // (0: stop)
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > SK_IDLE) {
                    sys_store(&m->alive, 0u);
                    __threadfence_system();
                    mb = mail_load(m);
                    go = mb.x != last && mb.x != 0;
                    if (go) sys_store(&m->alive, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (!go) sys_store(&m->alive, 0u);
            s_cmd[0] = go ? 1u : 0u;
            s_cmd[1] = mb.y;
            s_cmd[2] = mb.z;
            s_cmd[3] = mb.w;
            last = mb.x;
            s_cnt = 0;
            // (acquire at system scope: the sequence's bytes are read after the request word)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        }
        __syncthreads();
        if (!s_cmd[0]) return;
        const uint32_t len = s_cmd[1], k = s_cmd[2], thr = s_cmd[3];
        const uint32_t cap = min(len >= k && k ? len - k + 1 : 0u, ocap);
        const uint32_t nw = len >= k && k ? len - k + 1 : 0;
        uint64_t seed[4], rk[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            seed[c] = skq::SEED33[c];
            const uint32_t d = k % 33;
            rk[c] = d ? (((skq::SEED33[c] << d) | (skq::SEED33[c] >> (33 - d))) & skq::M33) : skq::SEED33[c];
        }
        // the windows in tiles whose bytes (the tile's windows and the k - 1 bases after them) are
        // staged in LDS once, so a long sequence (a transcript at the index side) is read from the
        // link in 16-B pieces, not byte by byte per window (k past half the LDS: read in place)
        const bool tiled = k <= SK_LDS_MAX / 2;
        const uint32_t tw = tiled ? (SK_LDS_MAX - k) & ~15u : (nw ? nw : 1u);  // windows per tile (16-B aligned)
        for (uint32_t t0 = 0; t0 < nw; t0 += tw) {
            const uint32_t tn = min(tw, nw - t0);
            if (tiled) {  // (the host buffer is 16-B aligned and padded to 16 B)
                const uint32_t b1 = min(len, t0 + tn + k - 1);
                const uint4* s4 = reinterpret_cast<const uint4*>(src + t0);
                uint4* d4 = reinterpret_cast<uint4*>(s_seq);
                for (uint32_t q = t; q < (b1 - t0 + 15) / 16; q += SK_WG) d4[q] = s4[q];
                __syncthreads();
            }
            // (indexed by position - t0: a pointer formed as s_seq - t0 would leave the LDS
            // aperture — the compiler moves only its low word — and fault when p is added)
            const uint8_t* s = tiled ? s_seq : src;  // (untiled: one tile, t0 = 0)
            // a chunk of the tile's windows per thread, rolled from its first base
            const uint32_t chunk = max(1u, (tn + SK_WG - 1) / SK_WG);
            for (uint32_t w0 = t0 + t * chunk; w0 < t0 + tn; w0 += SK_WG * chunk) {
                uint64_t h = 0;
                uint32_t run = 0;  // valid bases ending at p, counted from w0
                const uint32_t pend = min(min(len, w0 + chunk + k - 1), t0 + tn + k - 1);
                for (uint32_t p = w0; p < pend; ++p) {
                    const uint32_t c = s_code[s[p - t0]];
                    if (c == 4) {
                        run = 0;
                        h = 0;
                        continue;
                    }
                    ++run;
                    h = ((h << 1) | (h >> 32)) & skq::M33;
                    h ^= seed[c];
                    if (run > k) h ^= rk[s_code[s[p - t0 - k]]];
                    if (run >= k && (uint32_t)h <= thr) {  // src/sketch.cpp:33-35
                        const uint32_t at = atomicAdd(&s_cnt, 1u);
                        if (at < cap) out[1 + at] = (uint32_t)h;
                    }
                }
            }
            __syncthreads();  // (the tile's bytes are dead)
        }
        // every thread releases its own hash stores at system scope before the barrier, so thread
        // 0's count and done words, stored after it, reach the host after all of them
        __threadfence_system();
        __syncthreads();
        if (t == 0) {
            sys_store(out, s_cnt);
            sys_store(&m->done, last);
        }
    }
}

}  // namespace

struct skq_sketcher {
    int device = 0;
    hipStream_t st = nullptr;
    uint64_t cap_len = 0;   // bytes the pinned input holds
    uint8_t* hin = nullptr;  // pinned, mapped: the sequence
    uint32_t* hout = nullptr;  // pinned, mapped: [count, hashes...], cap_len + 1 words
    SkMail* mail = nullptr;  // pinned, mapped
    uint8_t* din = nullptr;   // device views of the three
    uint32_t* dout = nullptr;
    SkMail* dmail = nullptr;
    uint32_t seq = 0;        // the last request posted (and completed: calls are synchronous)
    bool running = false;    // a server was launched and may still be resident
};

namespace {

// stop the server (if any) and wait until it has left the device
int stop_server(skq_sketcher* h) {
    if (!h->running) return 0;
    __atomic_store_n(&h->mail->req, 0u, __ATOMIC_RELEASE);  // (0: stop)
    const hipError_t e = hipStreamSynchronize(h->st);
    h->running = false;
    return e == hipSuccess ? 0 : sfail(-3, "sketcher server failed");
}

int launch_server(skq_sketcher* h) {
    __atomic_store_n(&h->mail->alive, 1u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(k_sketch_server, dim3(1), dim3(SK_WG), SK_LDS_MAX, h->st, h->dmail, h->din, h->dout, h->seq - 1,
                       (uint32_t)std::min<uint64_t>(h->cap_len, 0xFFFFFFFFull));
    if (hipGetLastError() != hipSuccess) return sfail(-3, "sketcher server launch failed");
    h->running = true;
    return 0;
}

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
    if (int rc = stop_server(h)) return rc;  // (the server holds the old buffers)
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
    if (!rc && (hipHostMalloc(reinterpret_cast<void**>(&h->mail), sizeof(SkMail), hipHostMallocMapped | hipHostMallocCoherent) !=
                    hipSuccess ||
                hipHostGetDevicePointer(reinterpret_cast<void**>(&h->dmail), h->mail, 0) != hipSuccess))
        rc = sfail(-3, "sketcher mailbox allocation failed");
    if (!rc) {
        std::memset(h->mail, 0, sizeof(SkMail));
        rc = grow(h, max_len);
    }
    if (!rc && hipFuncSetAttribute(reinterpret_cast<const void*>(k_sketch_server), hipFuncAttributeMaxDynamicSharedMemorySize,
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
        SkMail* m = h->mail;
        m->len = (uint32_t)len;
        m->k = k;
        m->thr = threshold;
        uint32_t r = h->seq + 1;
        if (r == 0) r = 1;  // (never a request of 0... nor the previous one)
        // (sequentially consistent: a release store followed by an acquire load may be reordered
        // on x86, and the server does the mirror image — clears alive, then rereads req — so both
        // sides could read stale words and the request would wait for the slow-path check)
        __atomic_store_n(&m->req, r, __ATOMIC_SEQ_CST);
        h->seq = r;
        if (!h->running || !__atomic_load_n(&m->alive, __ATOMIC_SEQ_CST)) {
            // no server, or one that has gone idle: wait for it to leave unless it took this request
            // on its way out, then launch one (it serves the pending request first)
            while (h->running && __atomic_load_n(&m->done, __ATOMIC_ACQUIRE) != r) {
                const hipError_t q = hipStreamQuery(h->st);
                if (q == hipSuccess) h->running = false;
                else if (q != hipErrorNotReady) rc = sfail(-3, "sketcher server failed");
                if (rc) break;
            }
            if (!rc && __atomic_load_n(&m->done, __ATOMIC_ACQUIRE) != r) rc = launch_server(h);
        }
        // the answer: done = r (bounded: a server that left without it is relaunched once)
        for (uint64_t spin = 0; !rc && __atomic_load_n(&m->done, __ATOMIC_ACQUIRE) != r; ++spin) {
            __builtin_ia32_pause();
            if ((spin & 4095) == 4095) {
                const hipError_t q = hipStreamQuery(h->st);
                if (q == hipSuccess) {  // the server left (idle race): launch one again
                    h->running = false;
                    if (__atomic_load_n(&m->done, __ATOMIC_ACQUIRE) != r) rc = launch_server(h);
                } else if (q != hipErrorNotReady) {
                    rc = sfail(-3, "sketcher server failed");
                }
            }
            if (spin > (1ull << 28)) rc = sfail(-3, "sketcher server timed out");  // (~10 s)
        }
        if (!rc) {
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
    if (h->mail) (void)stop_server(h);
    if (h->st) (void)hipStreamSynchronize(h->st);
    release(h);
    if (h->mail) (void)hipHostFree(h->mail);
    if (h->st) (void)hipStreamDestroy(h->st);
    (void)hipSetDevice(prev);
    delete h;
    return 0;
}
