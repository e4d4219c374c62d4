// skq_ingest.hip — FASTQ ingest on the GPU: process_fastq_single_pass's record reader
// (src/main.cpp:113-148) with the text itself parsed in HBM.
//
// Host side: a reader thread fills pinned staging buffers straight from the file (parallel
// pread by a pool of workers; the buffers are cached across ingests) and copies each chunk to the device on its own stream, two chunks ahead, so file I/O and
// PCIe overlap the GPU work and the caller's result handling. The host never touches the bytes.
//
// Device side, per chunk (a run of whole lines, plus the line that follows as a halo so the
// last record's sequence line is present):
//   k_fq_func   one thread per 64-byte segment: line starts (a byte after '\n'), and the
//               reader's record machine over them as a packed function of its 4 states
//   (scan)      exclusive scan of those functions (hipcub, composition) -> state at each segment
//   k_fq_count  records opened per segment, given its entry state -> exclusive sum -> slots
//   k_fq_emit   header positions in file order
//   k_fq_rec    per record: id extent + 64-bit id hash, sequence line extent
//   (scan)      sequence lengths -> offsets of a flat batch
//   k_fq_gather sequences copied into the flat batch, which skq_map then sketches and chains
// The record machine (src/main.cpp:119-129): state 0 = between records, where a line starting
// with '@' opens a record (-> 1) and any other line is skipped; states 1, 2, 3 = the sequence,
// '+' and quality lines, consumed whatever they hold. The state at a chunk's end carries to the
// next chunk on the device.
//
// "The last record of an id with a valid sequence wins" (read_sketches[read.id] = ...,
// src/main.cpp:147) is resolved at the end (skq_ingest_finish): the records with status OK are
// radix-sorted by id hash; a hash seen once is a unique id, and the rare groups sharing a hash are
// settled on the host by comparing the id strings themselves (the file stays mapped), so the
// result is exact whatever the hash does.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <hipcub/hipcub.hpp>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "skq_internal.h"

namespace {

constexpr uint32_t SEG = 64;   // bytes per thread in the line-start passes
constexpr uint32_t PAD = 64;   // device text buffers are readable this far past their length

// Functions of the 4 machine states, f(s) in bits 2s..2s+1
constexpr uint32_t F_ID = 0xE4;   // s -> s
constexpr uint32_t F_AT = 0x39;   // line starting with '@': 0->1, 1->2, 2->3, 3->0
constexpr uint32_t F_NON = 0x38;  // any other line:         0->0, 1->2, 2->3, 3->0

__host__ __device__ __forceinline__ uint32_t fapply(uint32_t f, uint32_t s) { return (f >> (2 * s)) & 3u; }
// first a, then b
__host__ __device__ __forceinline__ uint32_t fthen(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (uint32_t s = 0; s < 4; ++s) r |= fapply(b, fapply(a, s)) << (2 * s);
    return r;
}
struct Then {
    __host__ __device__ __forceinline__ uint8_t operator()(uint8_t a, uint8_t b) const { return (uint8_t)fthen(a, b); }
};

// exact per-byte match of c in a 32-bit word -> 4 bits
__device__ __forceinline__ uint32_t bytes_eq4(uint32_t w, uint32_t c) {
    const uint32_t x = w ^ (c * 0x01010101u);
    const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // high bit: byte != c
    const uint32_t m = (~nz & 0x80808080u) >> 7;                                  // bits 0, 8, 16, 24
    return (m | (m >> 7) | (m >> 14) | (m >> 21)) & 0xFu;
}

// segment i: line-start mask and '@' mask of bytes [64i, 64i+64) that lie before `own`
__device__ __forceinline__ void seg_masks(const uint8_t* text, uint64_t own, uint64_t i, uint64_t& starts,
                                          uint64_t& at) {
    const uint64_t b0 = i * SEG;
    const uint4* q = reinterpret_cast<const uint4*>(text + b0);
    uint64_t nl = 0;
    at = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const uint4 w = q[v];
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            nl |= (uint64_t)bytes_eq4(ws[c], '\n') << (16 * v + 4 * c);
            at |= (uint64_t)bytes_eq4(ws[c], '@') << (16 * v + 4 * c);
        }
    }
    starts = (nl << 1) | (b0 == 0 ? 1ull : (text[b0 - 1] == '\n' ? 1ull : 0ull));
    const uint64_t lim = own - b0;
    if (lim < 64) starts &= (1ull << lim) - 1;
}

// one step of the machine on all 4 entry states at once (packed function f)
__device__ __forceinline__ uint32_t fstep(uint32_t f, bool is_at) { return fthen(f, is_at ? F_AT : F_NON); }

__global__ __launch_bounds__(256) void k_fq_func(const uint8_t* text, uint64_t own, uint64_t nseg, uint8_t* func) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    uint64_t starts, at;
    seg_masks(text, own, i, starts, at);
    uint32_t f = F_ID;
    while (starts) {
        const int j = __builtin_ctzll(starts);
        starts &= starts - 1;
        f = fstep(f, (at >> j) & 1);
    }
    func[i] = (uint8_t)f;
}

// records opened in segment i (entry state from the scanned prefix); the last segment also
// writes the state after the chunk for the next one
__global__ __launch_bounds__(256) void k_fq_count(const uint8_t* text, uint64_t own, uint64_t nseg,
                                                  const uint8_t* prefix, const uint32_t* state_in,
                                                  uint32_t* state_out, uint32_t* cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    uint64_t starts, at;
    seg_masks(text, own, i, starts, at);
    uint32_t s = fapply(prefix[i], *state_in), c = 0;
    while (starts) {
        const int j = __builtin_ctzll(starts);
        starts &= starts - 1;
        const bool a = (at >> j) & 1;
        c += (s == 0 && a);
        s = fapply(a ? F_AT : F_NON, s);
    }
    cnt[i] = c;
    if (i == nseg - 1) *state_out = s;
}

__global__ __launch_bounds__(256) void k_fq_emit(const uint8_t* text, uint64_t own, uint64_t nseg,
                                                 const uint8_t* prefix, const uint32_t* state_in,
                                                 const uint32_t* slot, uint32_t* hdr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nseg) return;
    uint64_t starts, at;
    seg_masks(text, own, i, starts, at);
    uint32_t s = fapply(prefix[i], *state_in), o = slot[i];
    while (starts) {
        const int j = __builtin_ctzll(starts);
        starts &= starts - 1;
        const bool a = (at >> j) & 1;
        if (s == 0 && a) hdr[o++] = (uint32_t)(i * SEG + j);
        s = fapply(a ? F_AT : F_NON, s);
    }
}

// first '\n' at or after p (or len)
__device__ __forceinline__ uint32_t line_end(const uint8_t* text, uint32_t p, uint32_t len) {
    while (p < len && (p & 15)) {
        if (text[p] == '\n') return p;
        ++p;
    }
    for (; p < len; p += 16) {
        const uint4 w = *reinterpret_cast<const uint4*>(text + p);
        const uint32_t m = bytes_eq4(w.x, '\n') | bytes_eq4(w.y, '\n') << 4 | bytes_eq4(w.z, '\n') << 8 |
                           bytes_eq4(w.w, '\n') << 12;
        if (m) return min(p + (uint32_t)__builtin_ctz(m), len);
    }
    return len;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

// 64-bit hash of text[a, b)
__device__ uint64_t id_hash(const uint8_t* text, uint32_t a, uint32_t b) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(b - a);
    uint32_t p = a;
    for (; p + 8 <= b; p += 8) {
        uint64_t w = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) w |= (uint64_t)text[p + c] << (8 * c);
        h = mix64(h ^ w) + 0x632BE59BD9B4E019ull;
    }
    uint64_t w = 0;
    for (int c = 0; p + c < b; ++c) w |= (uint64_t)text[p + c] << (8 * c);
    return mix64(h ^ w ^ 0xA0761D6478BD642Full);
}

struct RecOut {
    uint32_t* seq_pos;     // chunk-relative start of the sequence line
    uint64_t* seq_len;     // its length (scanned into batch offsets)
    uint64_t* id_hash;     // per file record
    uint64_t* id_pos;      // file offset of the id (after '@')
    uint32_t* id_len;
    uint32_t* max_len;
};

__global__ __launch_bounds__(256) void k_fq_rec(const uint8_t* text, uint32_t len, uint64_t file_off,
                                                const uint32_t* hdr, uint32_t n, uint64_t first, RecOut o) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint32_t p = hdr[r];
    const uint32_t e1 = line_end(text, p + 1, len);   // the id: rest of the header line
    const uint32_t s0 = min(e1 + 1, len);             // std::getline at end of file: empty sequence
    const uint32_t s1 = line_end(text, s0, len);
    o.seq_pos[r] = s0;
    o.seq_len[r] = s1 - s0;
    o.id_hash[first + r] = id_hash(text, p + 1, e1);
    o.id_pos[first + r] = file_off + p + 1;
    o.id_len[first + r] = e1 - p - 1;
    atomicMax(o.max_len, s1 - s0);
}

// one wave per record
__global__ __launch_bounds__(256) void k_fq_gather(const uint8_t* text, const uint32_t* seq_pos,
                                                   const uint64_t* offs, uint32_t n, uint8_t* out) {
    const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint8_t* src = text + seq_pos[r];
    uint8_t* dst = out + offs[r];
    const uint32_t m = (uint32_t)(offs[r + 1] - offs[r]);
    for (uint32_t j = lane; j < m; j += 64) dst[j] = src[j];
}

__global__ void k_copy_status(const uint8_t* st, uint8_t* dst, uint32_t n) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) dst[r] = st[r] & SKQ_STATUS_MASK;
}

// duplicate resolution: sort keys (~0 = not a candidate: status not OK)
__global__ void k_dup_keys(const uint8_t* status, const uint64_t* hash, uint64_t n, uint64_t* keys, uint64_t* vals) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t h = hash[r] == ~0ull ? ~0ull - 1 : hash[r];
    keys[r] = status[r] == SKQ_READ_OK ? h : ~0ull;
    vals[r] = r;
}

// kept[r] = 1: the only OK record with its hash; 2: shares its hash (settled on the host)
__global__ void k_dup_mark(const uint64_t* keys, const uint64_t* vals, uint64_t n, uint8_t* kept) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    if (k == ~0ull) return;
    const bool alone = (i == 0 || keys[i - 1] != k) && (i + 1 == n || keys[i + 1] != k);
    kept[vals[i]] = alone ? 1 : 2;
}

uint32_t blocks(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

}  // namespace

// ---- host side ---------------------------------------------------------------------------------

namespace {

int ifail(int code, const std::string& msg) {
    skq::set_error(code, msg.c_str());
    return code;
}

#define IHIP(expr)                                                                     \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) return ifail(-3, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

template <typename T>
struct DevArray {
    T* p = nullptr;
    uint64_t cap = 0;
    ~DevArray() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // grows to at least n elements keeping the first `keep` (synchronous when it moves)
    hipError_t reserve(uint64_t n, uint64_t keep = 0) {
        if (n <= cap) return hipSuccess;
        const uint64_t nc = std::max<uint64_t>(n, cap + cap / 2);
        T* q = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&q), std::max<uint64_t>(nc, 1) * sizeof(T) + PAD);
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

// chunk slots: the reader fills one while the device copies another and the consumer parses and
// maps a third (pread, H2D and the map overlap; two slots serialised the pread with the copy; a
// fourth absorbs the consumer's uneven chunks)
constexpr int NSLOT = 4;

struct Slot {
    uint8_t* host = nullptr;   // pinned
    uint64_t host_cap = 0;
    uint8_t* dev = nullptr;
    uint64_t dev_cap = 0;
    hipEvent_t h2d{}, consumed{};
    bool consumed_pending = false;
    bool h2d_pending = false;  // the host buffer is still being copied to the device
    int state = 0;             // 0 free, 1 ready (copy issued), 2 in use by the consumer
    uint64_t file_off = 0, own = 0, len = 0;
};

// The reader's pread workers, started once per ingest (a chunk's preads used to start and join
// io_threads threads of their own: ~1,200 thread starts per 3.2-GB file). run() splits [off,
// off + n) into one part per worker and returns when every part is in.
struct PreadPool {
    std::vector<std::thread> ws;
    std::mutex mu;
    std::condition_variable go, done;
    int fd = -1;
    uint8_t* dst = nullptr;
    uint64_t off = 0, n = 0;
    uint64_t gen = 0;
    int left = 0;
    bool fail = false, stop = false;

    void start(int nthreads, int file) {
        fd = file;
        for (int t = 0; t < nthreads; ++t) ws.emplace_back([this, t, nthreads] { work(t, nthreads); });
    }
    void work(int t, int T) {
        uint64_t seen = 0;
        for (;;) {
            uint8_t* d;
            uint64_t a, b, o;
            {
                std::unique_lock<std::mutex> lk(mu);
                go.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                const uint64_t step = (n + T - 1) / T;
                d = dst;
                o = off;
                a = off + std::min<uint64_t>(n, step * t);
                b = off + std::min<uint64_t>(n, step * (t + 1));
            }
            bool ok = true;
            while (a < b) {
                const ssize_t got = ::pread(fd, d + (a - o), (size_t)std::min<uint64_t>(b - a, 1ull << 30), (off_t)a);
                if (got <= 0) {
                    ok = false;
                    break;
                }
                a += (uint64_t)got;
            }
            std::lock_guard<std::mutex> lk(mu);
            fail |= !ok;
            if (--left == 0) done.notify_all();
        }
    }
    int run(uint8_t* d, uint64_t o, uint64_t len) {
        std::unique_lock<std::mutex> lk(mu);
        dst = d;
        off = o;
        n = len;
        fail = false;
        left = (int)ws.size();
        ++gen;
        go.notify_all();
        done.wait(lk, [&] { return left == 0; });
        return fail ? -1 : 0;
    }
    void shut() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        go.notify_all();
        for (auto& w : ws) w.join();
        ws.clear();
    }
};

// Pinned staging buffers outlive their ingest (hipHostFree of three 32-MiB slots cost ~13 ms of
// every file's close): a closed ingest returns them here and the next one on the process takes
// them back, as a caching host allocator does.
std::mutex g_pin_mu;
struct Pin {
    uint8_t* p;
    uint64_t cap;
    int device;  // (the device current when it was allocated)
};
std::vector<Pin> g_pins;

uint8_t* pin_take(uint64_t need, uint64_t& cap, int device) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    for (size_t i = 0; i < g_pins.size(); ++i)
        if (g_pins[i].cap >= need && g_pins[i].device == device) {
            uint8_t* p = g_pins[i].p;
            cap = g_pins[i].cap;
            g_pins.erase(g_pins.begin() + (long)i);
            return p;
        }
    return nullptr;
}

// (bounded by bytes: one ingest's slots per device, at most 512 MiB in all; what does not fit is
// freed at once)
constexpr uint64_t PIN_CACHE_BYTES = 512ull << 20;
void pin_give(uint8_t* p, uint64_t cap, int device) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    uint64_t held = 0, mine = 0;
    for (const Pin& x : g_pins) {
        held += x.cap;
        mine += x.device == device ? 1u : 0u;
    }
    if (mine < (uint64_t)NSLOT && held + cap <= PIN_CACHE_BYTES) {
        g_pins.push_back({p, cap, device});
        return;
    }
    (void)hipHostFree(p);
}

}  // namespace

struct skq_ingest {
    skq_session* s = nullptr;
    int device = 0;
    uint64_t max_reads = 0;
    int fd = -1;
    uint64_t fsize = 0;
    uint64_t lo = 0, hi = 0;     // this ingest's records: those whose header line starts in [lo, hi)
    const char* map = nullptr;   // the file, mapped for duplicate-id comparisons
    uint64_t chunk = 0;
    int io_threads = 1;
    PreadPool pool;
    hipStream_t copy = nullptr;
    hipStream_t pst = nullptr;  // the parse's first phase (record count), beside the caller's map
    // reader thread
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    Slot slot[NSLOT];
    uint64_t produced = 0, consumed_chunks = 0;
    bool eof = false, stop = false;
    std::string io_err;
    // parse workspace
    DevArray<uint8_t> func, prefix;
    DevArray<uint32_t> cnt, slotoff, hdr, seq_pos, state, scal;
    DevArray<uint64_t> seq_len, offs;   // sequence lengths -> batch offsets
    DevArray<uint8_t> batch;
    DevArray<uint8_t> cub_tmp;
    uint32_t* h_scal = nullptr;   // pinned: [n, max_len]
    // current chunk
    int cur = -1;
    uint64_t cur_n = 0, cur_done = 0;
    uint32_t cur_maxlen = 0;
    // per file record
    uint64_t records = 0;
    DevArray<uint64_t> id_hash, id_pos;
    DevArray<uint32_t> id_len;
    DevArray<uint8_t> status;
    bool finished = false;
    // SKQ_INGEST_TRACE=1: where the time goes, printed to stderr on close (seconds): the reader's
    // preads and its waits for a free slot, the consumer's waits for a ready chunk, its parse
    // (with the two host syncs) and its map launches
    bool trace = false;
    double t_read = 0, t_slot = 0, t_ready = 0, t_parse = 0, t_map = 0;
    uint64_t n_chunks = 0;
};

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// first '\n' in h[from, to) or `to`
uint64_t find_nl(const uint8_t* h, uint64_t from, uint64_t to) {
    const void* q = from < to ? std::memchr(h + from, '\n', (size_t)(to - from)) : nullptr;
    return q ? (uint64_t)(static_cast<const uint8_t*>(q) - h) : to;
}

// Reader thread: chunk = whole lines from `off` (at least `chunk` bytes unless the range ends)
// plus the line after them (the halo, which may lie past the range).
void reader_main(skq_ingest* g) {
    (void)hipSetDevice(g->device);
    uint64_t off = g->lo;
    std::string err;
    for (uint64_t c = 0; off < g->hi; ++c) {
        Slot& sl = g->slot[c % NSLOT];
        const double tw = g->trace ? now_s() : 0.0;
        {
            std::unique_lock<std::mutex> lk(g->mu);
            g->cv.wait(lk, [&] { return g->stop || sl.state == 0; });
            if (g->stop) return;
        }
        if (sl.consumed_pending) {  // the consumer's kernels are done with the device buffer
            (void)hipEventSynchronize(sl.consumed);
            sl.consumed_pending = false;
        }
        if (sl.h2d_pending) {  // (the host buffer's last copy: done before it is refilled)
            (void)hipEventSynchronize(sl.h2d);
            sl.h2d_pending = false;
        }
        const double tr = g->trace ? now_s() : 0.0;
        if (g->trace) g->t_slot += tr - tw;
        // read until the own region ends at a newline (or EOF) and the halo line is complete
        const uint64_t lim = g->hi - off;  // bytes of the range left (hi is a line start or EOF)
        uint64_t have = 0, want = std::min<uint64_t>(g->fsize - off, std::min(lim, g->chunk) + (1u << 16));
        uint64_t own = 0, len = 0;
        for (;;) {
            if (want > sl.host_cap) {
                uint64_t cap = std::max<uint64_t>(want, sl.host_cap * 2);
                uint8_t* h = pin_take(cap, cap, g->device);
                if (!h && hipHostMalloc(reinterpret_cast<void**>(&h), cap, hipHostMallocDefault) != hipSuccess) {
                    err = "pinned staging allocation failed";
                    break;
                }
                if (have) std::memcpy(h, sl.host, have);
                if (sl.host) pin_give(sl.host, sl.host_cap, g->device);
                sl.host = h;
                sl.host_cap = cap;
            }
            if (want > have) {
                if (g->pool.run(sl.host + have, off + have, want - have)) {
                    err = "FASTQ read failed";
                    break;
                }
                have = want;
            }
            const bool at_eof = off + have == g->fsize;
            if (lim <= g->chunk) {  // the rest of the range, then the line after it
                own = lim;
                if (off + own == g->fsize) {
                    len = own;
                    break;
                }
                if (have > own) {
                    const uint64_t h = find_nl(sl.host, own, have);
                    if (h < have || at_eof) {
                        len = h < have ? h + 1 : have;
                        break;
                    }
                }
                want = std::min<uint64_t>(g->fsize - off, std::max<uint64_t>(have * 2, own + (1u << 16)));
                continue;
            }
            const uint64_t e = find_nl(sl.host, g->chunk - 1, have);
            if (e < have) {
                own = e + 1;
                const uint64_t h = find_nl(sl.host, own, have);
                if (h < have || at_eof) {
                    len = h < have ? h + 1 : have;
                    break;
                }
            } else if (at_eof) {
                own = len = have;
                break;
            }
            want = std::min<uint64_t>(g->fsize - off, have * 2);
        }
        if (!err.empty()) break;
        if (g->trace) {
            g->t_read += now_s() - tr;
            ++g->n_chunks;
        }
        if (len + PAD > sl.dev_cap) {
            if (sl.dev) (void)hipFree(sl.dev);
            sl.dev = nullptr;
            const uint64_t cap = std::max<uint64_t>(len + PAD, g->chunk + (1u << 17));
            if (hipMalloc(reinterpret_cast<void**>(&sl.dev), cap) != hipSuccess) {
                err = "device chunk allocation failed";
                sl.dev_cap = 0;
                break;
            }
            sl.dev_cap = cap;
        }
        if (hipMemcpyAsync(sl.dev, sl.host, len, hipMemcpyHostToDevice, g->copy) != hipSuccess ||
            hipEventRecord(sl.h2d, g->copy) != hipSuccess) {
            err = "chunk upload failed";
            break;
        }
        // (the consumer's stream waits for sl.h2d; this host buffer is refilled only after it)
        sl.h2d_pending = true;
        sl.file_off = off;
        sl.own = own;
        sl.len = len;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            sl.state = 1;
            ++g->produced;
        }
        g->cv.notify_all();
        off += own;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    g->eof = true;
    if (!err.empty()) g->io_err = err;
    g->cv.notify_all();
}

template <typename F>
int cub_call(skq_ingest* g, F&& f) {
    size_t bytes = 0;
    IHIP(f(nullptr, bytes));
    IHIP(g->cub_tmp.reserve(bytes + 1));
    IHIP(f(g->cub_tmp.p, bytes));
    return 0;
}

// parse the chunk in slot c into the flat batch; sets cur_n / cur_maxlen
int parse_chunk(skq_ingest* g, int c, hipStream_t st) {
    Slot& sl = g->slot[c];
    // first phase (line starts, record machine, record count) on the parse stream: it touches only
    // the parse's own arrays, so it runs beside the previous chunk's map on the caller's stream and
    // its host sync does not wait for that map
    hipStream_t ps = g->pst;
    IHIP(hipStreamWaitEvent(ps, sl.h2d, 0));
    IHIP(hipStreamWaitEvent(st, sl.h2d, 0));
    const uint64_t nseg = (sl.own + SEG - 1) / SEG;
    if (sl.len >= (1ull << 32) - PAD) return ifail(-1, "FASTQ line too long for one chunk");
    IHIP(g->func.reserve(nseg));
    IHIP(g->prefix.reserve(nseg));
    IHIP(g->cnt.reserve(nseg + 1));
    IHIP(g->slotoff.reserve(nseg + 1));
    const uint8_t* text = sl.dev;
    const uint32_t* s_in = g->state.p + (g->consumed_chunks & 1);
    uint32_t* s_out = g->state.p + ((g->consumed_chunks + 1) & 1);
    k_fq_func<<<blocks(nseg, 256), 256, 0, ps>>>(text, sl.own, nseg, g->func.p);
    IHIP(hipGetLastError());
    if (int rc = cub_call(g, [&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveScan(t, b, g->func.p, g->prefix.p, Then(), (uint8_t)F_ID, (int)nseg, ps);
        }))
        return rc;
    IHIP(hipMemsetAsync(g->cnt.p + nseg, 0, 4, ps));
    k_fq_count<<<blocks(nseg, 256), 256, 0, ps>>>(text, sl.own, nseg, g->prefix.p, s_in, s_out, g->cnt.p);
    IHIP(hipGetLastError());
    if (int rc = cub_call(g, [&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveSum(t, b, g->cnt.p, g->slotoff.p, (int)(nseg + 1), ps);
        }))
        return rc;
    IHIP(hipMemcpyAsync(g->h_scal, g->slotoff.p + nseg, 4, hipMemcpyDeviceToHost, ps));
    IHIP(hipStreamSynchronize(ps));  // (the second phase, on the caller's stream, follows it)
    const uint32_t n = g->h_scal[0];
    g->cur_n = n;
    g->cur_done = 0;
    g->cur_maxlen = 0;
    if (n == 0) {
        IHIP(hipEventRecord(sl.consumed, st));
        return 0;
    }
    IHIP(g->hdr.reserve(n));
    IHIP(g->seq_pos.reserve(n));
    IHIP(g->seq_len.reserve(n + 1));
    IHIP(g->offs.reserve(n + 1));
    const uint64_t need = g->records + n;
    IHIP(g->id_hash.reserve(need, g->records));
    IHIP(g->id_pos.reserve(need, g->records));
    IHIP(g->id_len.reserve(need, g->records));
    IHIP(g->status.reserve(need, g->records));
    k_fq_emit<<<blocks(nseg, 256), 256, 0, st>>>(text, sl.own, nseg, g->prefix.p, s_in, g->slotoff.p, g->hdr.p);
    IHIP(hipGetLastError());
    IHIP(hipMemsetAsync(g->scal.p, 0, 8, st));
    IHIP(hipMemsetAsync(g->seq_len.p + n, 0, 8, st));
    RecOut o{g->seq_pos.p, g->seq_len.p, g->id_hash.p, g->id_pos.p, g->id_len.p, g->scal.p + 1};
    k_fq_rec<<<blocks(n, 256), 256, 0, st>>>(text, (uint32_t)sl.len, sl.file_off, g->hdr.p, n, g->records, o);
    IHIP(hipGetLastError());
    if (int rc = cub_call(g, [&](void* t, size_t& b) {
            return hipcub::DeviceScan::ExclusiveSum(t, b, g->seq_len.p, g->offs.p, (int)(n + 1), st);
        }))
        return rc;
    IHIP(hipMemcpyAsync(g->h_scal, g->scal.p, 8, hipMemcpyDeviceToHost, st));
    uint64_t total = 0;
    IHIP(hipMemcpyAsync(&total, g->offs.p + n, 8, hipMemcpyDeviceToHost, st));
    IHIP(hipStreamSynchronize(st));
    g->cur_maxlen = g->h_scal[1];
    IHIP(g->batch.reserve(total + 1));
    k_fq_gather<<<blocks(n, 4), 256, 0, st>>>(text, g->seq_pos.p, g->offs.p, n, g->batch.p);
    IHIP(hipGetLastError());
    IHIP(hipEventRecord(sl.consumed, st));  // the text buffer may be refilled after this
    return 0;
}

}  // namespace

extern "C" {

int skq_ingest_open(skq_session* s, const char* path, uint64_t chunk_bytes, int io_threads, skq_ingest** out) {
    return skq_ingest_open_range(s, path, 0, ~0ull, 0, chunk_bytes, io_threads, out);
}

int skq_ingest_open_range(skq_session* s, const char* path, uint64_t lo, uint64_t hi, uint32_t entry_state,
                          uint64_t chunk_bytes, int io_threads, skq_ingest** out) {
    if (!s || !path || !out) return ifail(-1, "null argument");
    if (entry_state > 3) return ifail(-1, "record-machine state must be 0..3");
    *out = nullptr;
    auto* g = new skq_ingest();
    g->s = s;
    g->device = skq::session_device(s);
    g->max_reads = skq::session_max_reads(s);
    // (64 MiB, 16 pread workers, four slots: profiles/r3_ingest_pool.log; before the worker pool
    // 12 x 32 MiB was best, profiles/r3_ingest_sweep.log)
    g->chunk = std::max<uint64_t>(chunk_bytes ? chunk_bytes : (64ull << 20), 1u << 12);
    g->io_threads = io_threads > 0 ? std::min(io_threads, 64) : 16;  // (workers started per ingest)
    if (const char* e = std::getenv("SKQ_INGEST_TRACE")) g->trace = std::atoi(e) != 0;
    g->fd = ::open(path, O_RDONLY);
    if (g->fd < 0) {
        delete g;
        return ifail(-2, std::string("Could not open FASTQ file: ") + path);
    }
    struct stat stt {};
    if (fstat(g->fd, &stt) != 0) {
        skq_ingest_close(g);
        return ifail(-2, std::string("Could not stat FASTQ file: ") + path);
    }
    g->fsize = (uint64_t)stt.st_size;
    if (g->fsize) {
        void* m = mmap(nullptr, g->fsize, PROT_READ, MAP_PRIVATE, g->fd, 0);
        if (m == MAP_FAILED) {
            skq_ingest_close(g);
            return ifail(-2, "FASTQ mmap failed");
        }
        g->map = static_cast<const char*>(m);
    }
    g->hi = std::min(hi, g->fsize);
    g->lo = std::min(lo, g->hi);
    if ((g->lo > 0 && g->map[g->lo - 1] != '\n') || (g->hi < g->fsize && g->map[g->hi - 1] != '\n')) {
        skq_ingest_close(g);
        return ifail(-1, "range bounds must be line starts (skq_fastq_split)");
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    int rc = 0;
    if (hipStreamCreateWithFlags(&g->copy, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&g->pst, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&g->h_scal), 16, hipHostMallocDefault) != hipSuccess ||
        g->state.reserve(2) != hipSuccess || g->scal.reserve(2) != hipSuccess ||
        hipMemset(g->state.p, 0, 8) != hipSuccess ||
        hipMemcpy(g->state.p, &entry_state, 4, hipMemcpyHostToDevice) != hipSuccess)
        rc = ifail(-3, "ingest setup failed");
    for (auto& sl : g->slot)
        if (!rc && (hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&sl.consumed, hipEventDisableTiming) != hipSuccess))
            rc = ifail(-3, "ingest setup failed");
    (void)hipSetDevice(prev);
    if (rc) {
        skq_ingest_close(g);
        return rc;
    }
    g->pool.start(g->io_threads, g->fd);
    g->th = std::thread(reader_main, g);
    *out = g;
    return 0;
}

int skq_ingest_map(skq_ingest* g, uint32_t threshold, double fraction, int accumulate, void* stream, uint64_t* n,
                   uint64_t* first) {
    if (!g || !n) return ifail(-1, "null argument");
    *n = 0;
    if (first) *first = g->records;
    if (g->finished) return ifail(-1, "ingest already finished");
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = 0;
    while (g->cur < 0 || g->cur_done >= g->cur_n) {
        if (g->cur >= 0) {  // the previous chunk is used up: hand its slot back
            {
                std::lock_guard<std::mutex> lk(g->mu);
                g->slot[g->cur].consumed_pending = true;
                g->slot[g->cur].state = 0;
                ++g->consumed_chunks;
            }
            g->cv.notify_all();
            g->cur = -1;
        }
        const int c = (int)(g->consumed_chunks % NSLOT);
        const double tw = g->trace ? now_s() : 0.0;
        {
            std::unique_lock<std::mutex> lk(g->mu);
            g->cv.wait(lk, [&] { return g->slot[c].state == 1 || (g->eof && g->produced == g->consumed_chunks); });
            if (g->slot[c].state != 1) {
                rc = g->io_err.empty() ? 0 : ifail(-2, g->io_err);
                (void)hipSetDevice(prev);
                return rc;  // end of file
            }
            g->slot[c].state = 2;
        }
        g->cur = c;
        const double tp = g->trace ? now_s() : 0.0;
        if (g->trace) g->t_ready += tp - tw;
        if ((rc = parse_chunk(g, c, st))) {
            (void)hipSetDevice(prev);
            return rc;
        }
        if (g->trace) g->t_parse += now_s() - tp;
    }
    const double tm = g->trace ? now_s() : 0.0;
    const uint64_t m = std::min<uint64_t>(g->cur_n - g->cur_done, g->max_reads);
    const uint64_t* offs = g->offs.p + g->cur_done;
    rc = skq_map(g->s, g->batch.p, offs, 0, m, std::max<uint32_t>(g->cur_maxlen, 1), threshold, fraction, accumulate,
                 stream);
    if (!rc) {
        skq_results res{};
        rc = skq::session_results(g->s, &res, false);
        if (!rc) {
            k_copy_status<<<blocks(m, 256), 256, 0, st>>>(res.status, g->status.p + g->records, (uint32_t)m);
            if (hipGetLastError() != hipSuccess) rc = ifail(-3, "status copy failed");
        }
    }
    if (!rc) {
        *n = m;
        g->records += m;
        g->cur_done += m;
    }
    if (g->trace) g->t_map += now_s() - tm;
    (void)hipSetDevice(prev);
    return rc;
}

uint64_t skq_ingest_records(const skq_ingest* g) { return g ? g->records : 0; }

int skq_ingest_finish(skq_ingest* g, uint8_t* kept) {
    if (!g) return ifail(-1, "null argument");
    const uint64_t N = g->records;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    auto done = [&](int rc) {
        (void)hipSetDevice(prev);
        return rc;
    };
    IHIP(hipDeviceSynchronize());
    g->finished = true;
    if (N == 0) return done(0);
    DevArray<uint64_t> k0, k1, v0, v1;
    DevArray<uint8_t> dk;
    IHIP(k0.reserve(N));
    IHIP(k1.reserve(N));
    IHIP(v0.reserve(N));
    IHIP(v1.reserve(N));
    IHIP(dk.reserve(N));
    IHIP(hipMemset(dk.p, 0, N));
    k_dup_keys<<<blocks(N, 256), 256>>>(g->status.p, g->id_hash.p, N, k0.p, v0.p);
    IHIP(hipGetLastError());
    if (int rc = cub_call(g, [&](void* t, size_t& b) {
            return hipcub::DeviceRadixSort::SortPairs(t, b, k0.p, k1.p, v0.p, v1.p, (int)N, 0, 64, nullptr);
        }))
        return done(rc);
    k_dup_mark<<<blocks(N, 256), 256>>>(k1.p, v1.p, N, dk.p);
    IHIP(hipGetLastError());
    std::vector<uint8_t> hk(N);
    IHIP(hipMemcpy(hk.data(), dk.p, N, hipMemcpyDeviceToHost));
    // groups sharing a hash: exact comparison of the ids (src/main.cpp:147, last valid wins)
    std::vector<uint64_t> amb;
    for (uint64_t r = 0; r < N; ++r)
        if (hk[r] == 2) amb.push_back(r);
    if (!amb.empty()) {
        std::vector<uint64_t> pos(N);
        std::vector<uint32_t> len(N);
        IHIP(hipMemcpy(pos.data(), g->id_pos.p, N * 8, hipMemcpyDeviceToHost));
        IHIP(hipMemcpy(len.data(), g->id_len.p, N * 4, hipMemcpyDeviceToHost));
        std::unordered_map<std::string_view, uint64_t> last;
        for (uint64_t r : amb) last[std::string_view(g->map + pos[r], len[r])] = r;  // ascending r
        for (uint64_t r : amb) hk[r] = last[std::string_view(g->map + pos[r], len[r])] == r ? 1 : 0;
    }
    if (kept) std::memcpy(kept, hk.data(), N);
    return done(0);
}

int skq_ingest_id(const skq_ingest* g, uint64_t ordinal, const char** id, uint64_t* len) {
    if (!g || ordinal >= g->records) return ifail(-1, "record out of range");
    uint64_t pos = 0;
    uint32_t l = 0;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    const bool ok = hipMemcpy(&pos, g->id_pos.p + ordinal, 8, hipMemcpyDeviceToHost) == hipSuccess &&
                    hipMemcpy(&l, g->id_len.p + ordinal, 4, hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipSetDevice(prev);
    if (!ok) return ifail(-3, "id lookup failed");
    if (id) *id = g->map + pos;
    if (len) *len = l;
    return 0;
}

int skq_ingest_supersede(skq_ingest* const* gs, uint32_t nparts, uint8_t* const* kept) {
    if ((!gs || !kept) && nparts) return ifail(-1, "null argument");
    // every range's kept records (id hash, range, ordinal), grouped by the hash's top bits so that
    // threads can each sort and scan one group
    struct E {
        uint64_t h;
        uint32_t d;
        uint64_t r;
        bool operator<(const E& o) const { return h != o.h ? h < o.h : d < o.d; }
    };
    constexpr int TB = 16;
    std::vector<std::vector<E>> bk(TB);
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (uint32_t d = 0; d < nparts; ++d) {
        const skq_ingest* g = gs[d];
        // (a part may hold no records — a short file split many ways — and then no kept array:
        // an empty std::vector's data() is null)
        if (!g || (!kept[d] && g->records)) return ifail(-1, "null part");
        if (!g->finished) return ifail(-1, "call skq_ingest_finish on every part first");
        std::vector<uint64_t> h(g->records);
        (void)hipSetDevice(g->device);
        const bool ok = !g->records ||
                        hipMemcpy(h.data(), g->id_hash.p, g->records * 8, hipMemcpyDeviceToHost) == hipSuccess;
        (void)hipSetDevice(prev);
        if (!ok) return ifail(-3, "id hash copy failed");
        for (uint64_t r = 0; r < g->records; ++r)
            if (kept[d][r]) bk[h[r] >> 60].push_back({h[r], d, r});
    }
    std::vector<int> rcs(TB, 0);
    std::vector<std::thread> ts;
    for (int b = 0; b < TB; ++b)
        ts.emplace_back([&, b] {
            auto& v = bk[b];
            std::sort(v.begin(), v.end());
            for (size_t i = 0; i < v.size();) {
                size_t j = i + 1;
                while (j < v.size() && v[j].h == v[i].h) ++j;
                if (v[j - 1].d != v[i].d) {  // one hash kept in several ranges: compare the ids
                    std::unordered_map<std::string_view, size_t> last;  // id -> its entry in the latest range
                    std::vector<std::string_view> ids(j - i);
                    for (size_t q = i; q < j; ++q) {
                        const char* id = nullptr;
                        uint64_t len = 0;
                        if (skq_ingest_id(gs[v[q].d], v[q].r, &id, &len)) {
                            rcs[b] = -3;
                            return;
                        }
                        ids[q - i] = std::string_view(id, len);
                        last[ids[q - i]] = q;  // (ranges ascending within the group)
                    }
                    for (size_t q = i; q < j; ++q)
                        if (last[ids[q - i]] != q) kept[v[q].d][v[q].r] = 0;
                }
                i = j;
            }
        });
    for (auto& t : ts) t.join();
    for (int rc : rcs)
        if (rc) return ifail(rc, "id lookup failed");
    return 0;
}

int skq_ingest_close(skq_ingest* g) {
    if (!g) return 0;
    const double tc = g->trace ? now_s() : 0.0;
    if (g->th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(g->mu);
            g->stop = true;
        }
        g->cv.notify_all();
        g->th.join();
    }
    g->pool.shut();
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(g->device);
    (void)hipDeviceSynchronize();
    for (auto& sl : g->slot) {
        if (sl.host) pin_give(sl.host, sl.host_cap, g->device);
        if (sl.dev) (void)hipFree(sl.dev);
        if (sl.h2d) (void)hipEventDestroy(sl.h2d);
        if (sl.consumed) (void)hipEventDestroy(sl.consumed);
    }
    if (g->h_scal) (void)hipHostFree(g->h_scal);
    if (g->copy) (void)hipStreamDestroy(g->copy);
    if (g->pst) (void)hipStreamDestroy(g->pst);
    if (g->map) munmap(const_cast<char*>(g->map), g->fsize);
    if (g->fd >= 0) ::close(g->fd);
    if (g->trace)
        std::fprintf(stderr,
                     "[skq ingest] %llu chunks: reader pread %.4f s, waits for a slot %.4f s; consumer waits %.4f s, "
                     "parse %.4f s, map %.4f s; close %.4f s\n",
                     (unsigned long long)g->n_chunks, g->t_read, g->t_slot, g->t_ready, g->t_parse, g->t_map,
                     now_s() - tc);
    delete g;  // DevArrays free themselves on this device
    (void)hipSetDevice(prev);
    return 0;
}

}  // extern "C"
