// skq_capi.hip — host side of the C ABI (include/skq.h): device index construction, session
// workspaces, kernel launches, result export and kernel timing. HIP runtime calls only; the
// kernels themselves are in skq_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <future>
#include <cmath>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "skq_internal.h"

namespace skq {
thread_local LaunchEvents g_launch_ev;
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(-3, std::string(#expr ": ") + hipGetErrorString(e_));          \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

int skq::set_error(int code, const char* msg) { return fail(code, msg); }

struct skq_index {
    int device = 0;
    uint32_t ntx = 0;
    uint32_t nk = 0;
    uint32_t ks[SKQ_MAX_K] = {};
    uint32_t maxk = 0, mink = 0;
    skq::DevTable tabs[SKQ_MAX_K] = {};
    uint32_t* d_buckets = nullptr;
    uint32_t* d_lists = nullptr;
    uint64_t* d_rolltab = nullptr;
    uint64_t nbucket_words = 0, nlist_words = 0, npostings = 0;
    uint32_t max_list = 0;
    // direct tables (one per distinct k; slot i uses dir[i]): u32 list offset per possible key
    uint32_t* d_dir_t[SKQ_MAX_K] = {};
    const uint32_t* dir[SKQ_MAX_K] = {};
    uint64_t dir_len[SKQ_MAX_K] = {};
    uint4* d_rank_t[SKQ_MAX_K] = {};
    uint32_t* d_rovf_t[SKQ_MAX_K] = {};
    const uint32_t* rank[SKQ_MAX_K] = {};
    const uint32_t* rovf[SKQ_MAX_K] = {};
    uint32_t* d_wdir_t[SKQ_MAX_K] = {};
    const uint32_t* wdir[SKQ_MAX_K] = {};
    // compact tables: per distinct k, the pilots; per k slot, the view
    uint16_t* d_wpil_t[SKQ_MAX_K] = {};
    const uint16_t* wpil[SKQ_MAX_K] = {};
    uint32_t wnb[SKQ_MAX_K] = {}, wseed[SKQ_MAX_K] = {};
    uint64_t dir_bytes = 0;
    // (build time only) per distinct k, each key's compact slot: the chained entries over compact
    // tables sit at the same slots; cleared once the chained tables are built
    std::vector<uint32_t> cmp_slots_t[SKQ_MAX_K];
    // chained tables (per k slot; ChainParams::chain): a 128-B entry per possible key up to the
    // largest (over compact tables: per present key, at its compact slot), carrying the key's postings list and those of the keys that follow it in the
    // transcripts; k_map1 then settles a read with ~1.5 entry requests instead of one per hash
    uint4* d_chain[SKQ_MAX_K] = {};
    uint64_t chain_len[SKQ_MAX_K] = {};
    uint64_t chain_bytes = 0;
    double chain_succ = 0;  // mean successor records per entry over the slots' tables (stats)
    double chain_build_s = 0;      // host seconds building the chained entries (this index's share)
    uint64_t chain_host_bytes = 0;  // host peak of one slot's build: entries + sorted candidates
    uint32_t chain_slots = 0;
    // 1 = dir tables, 2 = rank tables (the sketch probes), 3 = wide tables, 5 = compact tables
    // (4 was the block tables, retired in round 3: compact tables are smaller and faster)
    int mode = 0;
    bool direct = false;  // every slot with a table has a direct table: the sketch probes
};

struct TimedLaunch {
    int kind;
    hipEvent_t start, stop;
};

// A frame: every per-batch array a map and its tail (the slow paths, the totals binning) read or
// write. A fused map whose tail runs on the session's side stream takes the other frame from the
// previous batch's (skq_session::f and alt swap), so the next batch's map on the launch stream
// writes one frame while the previous batch's tail on the side stream still reads and writes the
// other: the launch stream then runs the maps back to back (the batch tail).
struct Frame {
    uint8_t* status = nullptr;
    uint32_t* hash_cnt = nullptr;
    uint32_t* hashes = nullptr;
    uint32_t* lofs = nullptr;    // list offsets per probe (k_probe -> k_count), shaped like hashes
    uint8_t* pflag = nullptr;
    uint32_t* hash_ext = nullptr;
    uint32_t* ovf1 = nullptr;
    uint32_t* ovf2 = nullptr;
    uint32_t* ovf3 = nullptr;  // second-level lists behind k_slow_wave
    uint32_t* ovf4 = nullptr;
    uint32_t* cand_cnt = nullptr;
    uint32_t* cand_tid = nullptr;
    uint32_t* cand_score = nullptr;
    uint32_t* cand_wtot = nullptr;  // per wave of 64 reads: its packed candidate words (k_bin_packed)
    uint32_t* cand_ext = nullptr;
    uint64_t* scratch = nullptr;
    // control words: two halves of C_WORDS; ctrl is the current batch's. A small fused batch's tail
    // (on the launch stream) zeroes the other half on its way (k_general_slow) and the next such
    // batch takes it, so no reset runs between the two maps; every other path resets ctrl itself
    uint32_t* ctrl = nullptr;
    uint32_t* ctrl_mem = nullptr;
    bool other_zeroed = false;
    uint32_t* ktab = nullptr;    // multi-k map by passes: per-k count tables (allocated on first use)
    uint8_t* kcnt = nullptr;
    uint32_t* stash = nullptr;   // multi-k map by passes: the first pass's staged bases (SketchParams::stash)
    uint64_t stash_words = 0;
    uint32_t hcap_alloc = 0;     // stride the hashes buffer was sized for
};

struct skq_session {
    skq_index* idx = nullptr;
    uint64_t max_reads = 0;
    uint32_t max_len = 0;
    uint32_t hcap = 0;         // stride of the current results
    uint64_t n_reads = 0;      // reads in the current results
    bool have_sketch = false;
    bool probed = false;       // the last skq_sketch also filled lofs/pflag (fused probe)
    bool have_chain = false;   // candidates belong to the current batch
    bool hash_packed = false;  // hashes in the per-wave packed layout (single-k fused map)
    bool cand_packed = false;  // candidates likewise
    Frame f;                   // the current batch's frame (its results)
    Frame alt;                 // the other frame (allocated with the first batch whose tail runs on the side stream)
    int fid = 0;               // which of the two frames f is (events below are per frame)
    uint64_t hash_ext_cap = 0;
    uint32_t ovf_cap = 0;
    uint64_t cand_ext_cap = 0;
    uint64_t scratch_cap = 0;
    // per-transcript totals by buckets of 2^bin_bits ids (k_bin / k_bin_sum); bin_nb = 0: direct.
    // One set: every kernel that bins runs after the previous batch's k_bin_sum (the side stream
    // runs the tails in order; the launch stream waits for it before binning itself)
    uint32_t bin_bits = 13, bin_nb = 0;
    uint32_t* bin_hdr = nullptr;
    uint32_t* bin_region = nullptr;
    // the batches' packed sums (reads << 40 | score per transcript: k_bin_sum, k_tot_small), folded
    // into tx_reads / tx_score (k_fold_totals) when they are read, or before the reads they hold
    // could pass 2^24 (acc_reads: the reads of the batches added since the last fold)
    uint64_t* tx_acc = nullptr;
    uint64_t acc_reads = 0;
    uint64_t* tx_reads = nullptr;
    uint64_t* tx_score = nullptr;
    // explicit-sketch chaining (skq_chain_sketches) keeps its inputs' layout for export
    const uint32_t* x_hashes = nullptr;
    const uint64_t* x_offs = nullptr;
    bool timing = false;
    std::vector<TimedLaunch> timed;
    uint64_t* stamps = nullptr;  // development: k_map1 phase clocks (skq_session_set_stamps)
    // the side stream (batch tails), created on first use; per frame x, ev_done[x] follows the last
    // side-stream work on frame x (its tail, then the reset of its control words once the next
    // batch has taken the other frame: zeroed[x])
    hipStream_t side = nullptr;
    hipEvent_t ev_fork{}, ev_map{}, ev_done[2]{};
    hipStream_t last_st{};
    hipEvent_t ev_snap[2]{};  // (skq_session_totals_async: the consumer's work, the copy)  // (the stream of the last batch's tail: where a results call folds the sums)  // (ev_map: bound to a side batch's map dispatch)
    bool done_rec[2] = {false, false};
    bool zeroed[2] = {false, false};
    bool tail_side[2] = {false, false};  // the frame's batch ran its tail on the side stream
};

int skq::session_device(const skq_session* s) { return s->idx->device; }
uint64_t skq::session_max_reads(const skq_session* s) { return s->max_reads; }

namespace {

template <typename T>
int dev_alloc(T** p, uint64_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
    return 0;
}

// the gather tables (wide and chained entries, GBs read at random): plain hipMalloc (physically
// contiguous memory, hipDeviceMallocContiguous, measured the same in round 4: DESIGN.md §5)
template <typename T>
int dev_alloc_table(T** p, uint64_t count) {
    return dev_alloc(p, count);
}

template <typename T>
void dev_free(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

// choose the raw-retained capacity per (read, k) for a batch: the smallest of 16/32/64 holding
// the expected count plus 4 sigma (reads beyond it are still exact, through the wave slow path;
// at 150 bp, 5 %: 16 at k = 31 (1.3e-4 of the reads past it), 32 at k = 21, 25, 31; 3 sigma (16
// there) sent 18k of 10M reads to the slow path: 4 % slower at cfg5)
// (sigmas 3 for the multi-k passes: a capacity of 32 holds k_map1 at 3 workgroups per CU for
// 2.0 ms a pass at cfg5 against 1.47 ms at 16, and the ~2e-4 of the reads past 16 at k = 21, 25
// cost the wave slow path far less)
uint32_t pick_hcap(uint32_t max_len, uint32_t mink, uint32_t threshold, double sigmas = 4.0) {
    const uint32_t L = std::min<uint32_t>(max_len, skq::LFAST);
    const double w = L >= mink ? (double)(L - mink + 1) : 0.0;
    const double f = ((double)threshold + 1.0) / 4294967296.0;
    const double mu = w * f;
    const double need = mu + sigmas * std::sqrt(mu * (1.0 - f));
    if (need <= 16) return 16;
    if (need <= 32) return 32;
    return 64;
}

// Development switches (A/B builds of the shipped library's choices, and the parity tests that pin
// both sides of them) are read only beside SKQ_DEV=1; without it the library reads SKQ_PROBE,
// SKQ_CHAIN, SKQ_CHAIN_MB, SKQ_DIRECT_MB (the index's kinds and budgets), SKQ_DEVICE (the drop-in's
// device) and SKQ_INGEST_TRACE, and nothing else.
static const char* dev_env(const char* name) {
    static const bool dev = [] {
        const char* e = std::getenv("SKQ_DEV");
        return e && std::atoi(e) == 1;
    }();
    return dev ? std::getenv(name) : nullptr;
}

// the multi-k passes stage from the first pass's image of the bases; SKQ_STASH=0 (development)
// re-reads the bases in every pass (read per batch, so the parity tests run both)
static bool use_stash() {
    const char* e = dev_env("SKQ_STASH");
    return !e || std::atoi(e) != 0;
}

// the multi-k passes' raw capacity: the mean retained windows of the pass's k plus this many
// standard deviations (reads beyond it take k_slow_wave); SKQ_PASS_SIGMAS (development) overrides
double pass_sigmas() {
    static const double v = [] {
        const char* e = dev_env("SKQ_PASS_SIGMAS");
        return e ? std::atof(e) : 3.0;
    }();
    return v;
}

// a timing scope: kinds 0-2 (the launch stream's map, sketch, probe, count) bind their events to
// the scope's dispatches (skq::launch_timed); kind 3 (the side stream's tail) records marker events
void record(skq_session* s, int kind, hipEvent_t* start, hipStream_t st) {
    if (!s->timing) return;
    (void)hipEventCreate(start);
    if (kind == 3) {
        (void)hipEventRecord(*start, st);
        return;
    }
    hipEvent_t stop;
    (void)hipEventCreate(&stop);
    skq::g_launch_ev = {*start, stop};
}

void record_stop(skq_session* s, int kind, hipEvent_t start, hipStream_t st) {
    if (!s->timing) return;
    hipEvent_t stop;
    if (kind == 3) {
        (void)hipEventCreate(&stop);
        (void)hipEventRecord(stop, st);
    } else {
        stop = static_cast<hipEvent_t>(skq::g_launch_ev.stop);
        const bool launched = skq::g_launch_ev.start == nullptr;  // (consumed by a first launch)
        skq::g_launch_ev = {};
        if (!launched) {
            (void)hipEventDestroy(start);
            (void)hipEventDestroy(stop);
            return;
        }
    }
    s->timed.push_back({kind, start, stop});
}

int ensure_hashes(skq_session* s, uint32_t hcap) {
    if (s->f.hcap_alloc >= hcap) return 0;
    (void)hipDeviceSynchronize();
    dev_free(s->f.hashes);
    dev_free(s->f.lofs);
    if (dev_alloc(&s->f.hashes, s->max_reads * s->idx->nk * (uint64_t)hcap)) return -3;
    if (dev_alloc(&s->f.lofs, s->max_reads * s->idx->nk * (uint64_t)hcap)) return -3;
    s->f.hcap_alloc = hcap;
    return 0;
}

// Direct tables: for each distinct k, dir[h] = list offset of key h (~0u = no key), for every h
// up to the table's largest key, so the sketch kernel probes with one 4-B gather per retained
// hash. At the reference's fraction (double)0.05f keys are <= 214748367: 859 MB per k, which
// HBM3E holds easily. Built only while the total stays inside SKQ_DIRECT_MB (default 8192 MiB;
// 0 disables) and half the free device memory; otherwise probes go through the bucket table.
int build_rank(skq_index* ix, uint32_t ntables, const skq_kmer_table* tables,
               const std::vector<uint32_t>* dkeys, const std::vector<uint32_t>* dvals) {
    uint64_t need = 0;
    for (uint32_t t = 0; t < ntables; ++t) {
        if (dkeys[t].empty()) continue;
        const uint64_t nb = ((uint64_t)dkeys[t].back() >> 5) + 1;
        std::vector<uint4> blk(nb, make_uint4(0, 0, ~0u, ~0u));
        std::vector<uint32_t> ovf;
        for (size_t j = 0; j < dkeys[t].size(); ++j) {
            const uint32_t key = dkeys[t][j];
            uint4& b = blk[key >> 5];
            const uint32_t pos = __builtin_popcount(b.x);
            if (pos == 0) b.z = dvals[t][j];
            else if (pos == 1) b.w = dvals[t][j];
            else {
                if (pos == 2) b.y = (uint32_t)ovf.size();
                ovf.push_back(dvals[t][j]);
            }
            b.x |= 1u << (key & 31);
        }
        ovf.push_back(0);
        if (dev_alloc(&ix->d_rank_t[t], nb) || dev_alloc(&ix->d_rovf_t[t], ovf.size()))
            return fail(-3, "rank table allocation failed");
        if (hipMemcpy(ix->d_rank_t[t], blk.data(), nb * 16, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(ix->d_rovf_t[t], ovf.data(), ovf.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            return fail(-3, "rank table upload failed");
        need += nb * 16 + ovf.size() * 4;
        for (uint32_t i = 0; i < ix->nk; ++i)
            if (tables[t].k == ix->ks[i]) {
                ix->rank[i] = reinterpret_cast<const uint32_t*>(ix->d_rank_t[t]);
                ix->rovf[i] = ix->d_rovf_t[t];
                ix->dir_len[i] = nb;
            }
    }
    ix->dir_bytes = need;
    ix->mode = 2;
    ix->direct = true;
    return 0;
}

// Wide direct tables: for each distinct k, an 8-word entry per possible key holding the key's
// whole postings list when it has at most 7 transcripts (the first 7 and the list offset when
// longer), so a retained hash costs the chain one 64-B line and the sketch no probe at all.
// 32 B per key up to the largest: 6.9 GB per k at (double)0.05f. Only for k_count3's id range.
int build_wide(skq_index* ix, uint32_t ntables, const skq_kmer_table* tables, const std::vector<uint32_t>* dkeys,
               const std::vector<uint32_t>* dvals, const uint64_t* len) {
    hipStream_t st = nullptr;
    uint64_t need = 0;
    uint32_t *dk = nullptr, *dv = nullptr;
    for (uint32_t t = 0; t < ntables; ++t) {
        const uint64_t m = dkeys[t].size();
        if (m && dvals[t].back() >= 0x80000000u) return fail(-1, "index too large for wide tables");
        if (dev_alloc_table(&ix->d_wdir_t[t], len[t] * 8) || dev_alloc(&dk, m) || dev_alloc(&dv, m)) {
            dev_free(dk);
            dev_free(dv);
            return fail(-3, "wide table allocation failed");
        }
        if (hipMemsetAsync(ix->d_wdir_t[t], 0, len[t] * 32, st) != hipSuccess ||
            hipMemcpy(dk, dkeys[t].data(), m * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dv, dvals[t].data(), m * 4, hipMemcpyHostToDevice) != hipSuccess ||
            skq::launch_wdir_scatter(ix->d_wdir_t[t], dk, dv, ix->d_lists, m, st) ||
            hipStreamSynchronize(st) != hipSuccess) {
            dev_free(dk);
            dev_free(dv);
            return fail(-3, "wide table build failed");
        }
        dev_free(dk);
        dev_free(dv);
        need += len[t] * 32;
    }
    ix->dir_bytes = need;
    for (uint32_t i = 0; i < ix->nk; ++i)
        for (uint32_t t = 0; t < ntables; ++t)
            if (tables[t].k == ix->ks[i]) {
                ix->wdir[i] = ix->d_wdir_t[t];
                ix->dir_len[i] = len[t];
            }
    ix->direct = true;
    ix->mode = 3;
    return 0;
}

// Minimal perfect hash of one k's keys, PTHash-style: keys hash into nb buckets; buckets, largest
// first, each take the first 16-bit pilot that sends all their keys to distinct free slots among
// nslots (cmp_slot, skq_internal.h). slot[j] receives key j's slot. false: some bucket found no
// pilot (the caller retries with another seed).
bool mph_place(const std::vector<uint32_t>& keys, uint32_t seed, uint64_t nslots, uint32_t nb,
               std::vector<uint16_t>& pil, std::vector<uint32_t>& slot) {
    const uint64_t m = keys.size();
    std::vector<uint32_t> kh(m), start(nb + 1, 0), member(m);
    for (uint64_t j = 0; j < m; ++j) {
        kh[j] = skq::cmp_key_hash(keys[j], seed);
        ++start[skq::cmp_scale(kh[j], nb) + 1];
    }
    uint32_t maxb = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        maxb = std::max(maxb, start[b + 1]);
        start[b + 1] += start[b];
    }
    {
        std::vector<uint32_t> fill(start.begin(), start.end() - 1);
        for (uint64_t j = 0; j < m; ++j) member[fill[skq::cmp_scale(kh[j], nb)]++] = (uint32_t)j;
    }
    // buckets by size, largest first (counting sort)
    std::vector<uint32_t> by(maxb + 2, 0), order(nb);
    for (uint32_t b = 0; b < nb; ++b) ++by[maxb - (start[b + 1] - start[b]) + 1];
    for (uint32_t s = 0; s <= maxb; ++s) by[s + 1] += by[s];
    for (uint32_t b = 0; b < nb; ++b) order[by[maxb - (start[b + 1] - start[b])]++] = b;
    std::vector<uint64_t> taken((nslots + 63) / 64, 0);
    auto is_taken = [&](uint32_t s) { return (taken[s >> 6] >> (s & 63)) & 1ull; };
    pil.assign(nb, 0);
    slot.assign(m, 0);
    std::vector<uint32_t> cur(maxb);
    for (const uint32_t b : order) {
        const uint32_t a = start[b], z = start[b + 1];
        if (a == z) break;  // (sizes descending: the rest are empty)
        uint32_t p = 0;
        for (; p < 65536; ++p) {
            bool ok = true;
            for (uint32_t q = a; q < z && ok; ++q) {
                const uint32_t s = skq::cmp_slot(kh[member[q]], p, nslots);
                ok = !is_taken(s);
                for (uint32_t u = a; u < q && ok; ++u) ok = cur[u - a] != s;
                cur[q - a] = s;
            }
            if (ok) break;
        }
        if (p == 65536) return false;
        pil[b] = (uint16_t)p;
        for (uint32_t q = a; q < z; ++q) {
            taken[cur[q - a] >> 6] |= 1ull << (cur[q - a] & 63);
            slot[member[q]] = cur[q - a];
        }
    }
    return true;
}

// Compact tables: for each distinct k, each key's 8-word entry ([key, t0 | F << 22, t1..t6],
// skq_internal.h) in one of m / 0.95 slots placed by mph_place (m / 5 buckets). A lookup reads
// the bucket's pilot (2 B per 5 keys: 1.7 MB at 4.24M keys, held in L2) and then one 32-B entry;
// the entries (143 MB at 4.24M keys) stay in the 256 MB Infinity Cache, which the wide direct
// table (6.9 GB, one entry per possible key) cannot. Only for k_count3's id range (tids < 2^22).
int build_compact(skq_index* ix, uint32_t ntables, const skq_kmer_table* tables, const std::vector<uint32_t>* dkeys,
                  const std::vector<uint32_t>* dvals, const std::vector<uint32_t>& lists) {
    uint64_t need = 0;
    for (uint32_t t = 0; t < ntables; ++t) {
        const uint64_t m = dkeys[t].size();
        if (m == 0) continue;
        const uint64_t nslots = std::max<uint64_t>(m + 1, (uint64_t)std::ceil((double)m / 0.95));
        // (5 keys per bucket: larger buckets, for a smaller pilot array, fail to place at 0.8-0.9
        // load within 16-bit pilots; 2.7 s of host time at 4.24M keys)
        const uint32_t nb = (uint32_t)std::max<uint64_t>(1, (m + 4) / 5);
        // (slots are listed as slot | lane << 26 in k_map1)
        if (nslots > (1ull << 26)) return fail(-1, "index too large for compact tables");
        std::vector<uint16_t> pil;
        std::vector<uint32_t> slot;
        uint32_t seed = 0x5EED5EEDu;
        int tries = 0;
        while (!mph_place(dkeys[t], seed, nslots, nb, pil, slot)) {
            if (++tries == 8) return fail(-1, "compact table placement failed");
            seed = skq::cmp_mix(seed + 0x9E3779B9u);
        }
        std::vector<uint32_t> ent(nslots * 8, 0);
        ix->cmp_slots_t[t] = slot;
        for (uint64_t j = 0; j < m; ++j) {
            const uint32_t off = dvals[t][j], n = lists[off];
            uint32_t* e = ent.data() + (uint64_t)slot[j] * 8;
            e[0] = dkeys[t][j];
            for (uint32_t q = 0; q < 7 && q < n; ++q) e[1 + q] = lists[off + 1 + q];
            e[1] |= std::min<uint32_t>(n, skq::CMP_LONG) << 22;
            if (n > 7) {
                e[4] |= (off & 0x3FFu) << 22;
                e[5] |= ((off >> 10) & 0x3FFu) << 22;
                e[6] |= ((off >> 20) & 0x3FFu) << 22;
                e[7] |= (off >> 30) << 22;
            }
        }
        if (dev_alloc(&ix->d_wdir_t[t], nslots * 8) || dev_alloc(&ix->d_wpil_t[t], nb))
            return fail(-3, "compact table allocation failed");
        if (hipMemcpy(ix->d_wdir_t[t], ent.data(), nslots * 32, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(ix->d_wpil_t[t], pil.data(), (size_t)nb * 2, hipMemcpyHostToDevice) != hipSuccess)
            return fail(-3, "compact table upload failed");
        need += nslots * 32 + (uint64_t)nb * 2;
        for (uint32_t i = 0; i < ix->nk; ++i)
            if (tables[t].k == ix->ks[i]) {
                ix->wdir[i] = ix->d_wdir_t[t];
                ix->dir_len[i] = nslots;
                ix->wpil[i] = ix->d_wpil_t[t];
                ix->wnb[i] = nb;
                ix->wseed[i] = seed;
            }
    }
    ix->dir_bytes = need;
    ix->direct = true;
    ix->mode = 5;
    return 0;
}


// Chained tables for one k slot (ChainParams::chain; entry layout skq_internal.h CHN_*). The
// transcripts are sketched in position order (the index's own hashing: skq::sketch_positions);
// every retained k-mer's successors within CHAIN_HOPS retained positions in any transcript are
// candidates for its entry, nearest first (ties: smaller key). An entry takes the key's own record,
// then successors while they fit: at most CHN_KEYS records and CHN_TIDS distinct transcripts over
// the whole entry (their ids stored once, each with the set of records whose list holds it); a
// successor that does not fit is skipped, a later one may. A record names its
// key's WHOLE postings list (the index's own lists[]), so whatever it settles is exactly what a
// lookup of that key returns. The entries (one per present key) are built on the host and
// scattered on the device into a table of 128-B entries for every possible key up to the largest
// (27.5 GB at (double)0.05f and 4.24M keys: HBM3E holds it); entries of absent keys stay zero.
// One entry settles all of a read's retained hashes for 92 % of cfg3's reads (tools/chain_sim.py).
constexpr uint32_t CHAIN_HOPS = 12;

__global__ void k_chain_scatter(uint4* tab, const uint32_t* keys, const uint4* ent, uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n * 8) return;
    tab[(uint64_t)keys[j >> 3] * 8 + (j & 7)] = ent[j];
}

// one key's entry: its own record (a list of <= CHN_TIDS transcripts), then successors in order
// while they fit (records, distinct transcripts); returns the successors taken
static uint32_t chain_entry(uint32_t* e, uint32_t key, uint32_t off, const std::vector<uint32_t>& lists,
                            const uint32_t* sk, const uint32_t* so, size_t ns) {
    if (lists[off] > skq::CHN_TIDS) {
        e[skq::CHN_W_KEY] = skq::CHN_LONG;
        return 0;
    }
    uint32_t tids[skq::CHN_TIDS], sets[skq::CHN_TIDS] = {}, nt = 0, nr = 0;
    auto add = [&](uint32_t k2, uint32_t o2) -> bool {
        const uint32_t n = lists[o2];
        if (n == 0 || n > skq::CHN_TIDS) return false;
        uint32_t tt[skq::CHN_TIDS], ntt = nt, mk = 0;
        std::copy(tids, tids + nt, tt);
        for (uint32_t q = 0; q < n; ++q) {
            const uint32_t t = lists[o2 + 1 + q];
            uint32_t s = 0;
            while (s < ntt && tt[s] != t) ++s;
            if (s == ntt) {
                if (ntt == skq::CHN_TIDS) return false;
                tt[ntt++] = t;
            }
            mk |= 1u << s;
        }
        std::copy(tt, tt + ntt, tids);
        nt = ntt;
        for (uint32_t s = 0; s < nt; ++s)
            if ((mk >> s) & 1u) sets[s] |= 1u << nr;
        e[skq::CHN_W_KEY + nr++] = k2 ^ skq::CHN_KEY_LIMIT;
        return true;
    };
    add(key, off);  // (always fits)
    uint32_t taken = 0;
    for (size_t q = 0; q < ns && nr < skq::CHN_KEYS; ++q) taken += add(sk[q], so[q]) ? 1u : 0u;
    for (uint32_t t = 0; t < nt; ++t) {
        e[skq::CHN_W_SET + t / 2] |= sets[t] << (16 * (t & 1));
        e[skq::CHN_W_TID + t] = tids[t];
    }
    return taken;
}

// The host side of one k slot's chained table: the entries of the present keys (128 B each) and
// their successor count. Indexes built at once on several devices from the same tables (the CLI's
// one thread per device) share one build: the first caller builds, the others wait for it, and the
// entries are dropped when the last of them has uploaded its table.
struct ChainHost {
    std::vector<uint32_t> ent;
    uint64_t nsucc = 0;
    double seconds = 0;  // host build time
    uint64_t triples = 0;  // (key, successor, hop) candidates sorted (host peak: 12 B each + ent)
};
// (keyed on what the callers have in common: the caller's table arrays and transcript sequences,
// not the per-call host image derived from them, whose address differs in every call)
struct ChainKey {
    const void* seqs;
    const void* offs;
    const void* tkeys;
    const void* toffs;
    const void* ttids;
    uint64_t nseq, k, thr, m, last, nlists;
    bool operator==(const ChainKey& o) const {
        return seqs == o.seqs && offs == o.offs && tkeys == o.tkeys && toffs == o.toffs && ttids == o.ttids &&
               nseq == o.nseq && k == o.k && thr == o.thr && m == o.m && last == o.last && nlists == o.nlists;
    }
};
struct ChainShare {
    ChainKey key;
    std::shared_future<std::shared_ptr<const ChainHost>> fut;
    int users;
};
static std::mutex g_chain_mu;
static std::vector<ChainShare> g_chain_share;

static std::shared_ptr<const ChainHost> chain_host_build(const std::vector<uint32_t>& keys, const std::vector<uint32_t>& vals,
                                                        const std::vector<uint32_t>& lists, uint32_t k,
                                                        const uint8_t* seqs, const uint64_t* offs, uint32_t nseq,
                                                        uint32_t threshold) {
    const auto t0 = std::chrono::steady_clock::now();
    auto out = std::make_shared<ChainHost>();
    const uint64_t m = keys.size();
    const uint64_t len = (uint64_t)keys.back() + 1;
    const uint32_t P = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    // (key, successor, hop) triples, bucketed by key range, one sort per bucket
    constexpr uint32_t NB = 256;
    struct Cand {
        uint32_t h, g, d;
        bool operator<(const Cand& o) const {
            return h != o.h ? h < o.h : (d != o.d ? d < o.d : g < o.g);
        }
    };
    const uint64_t span = len / NB + 1;
    std::vector<std::vector<std::vector<Cand>>> part(P, std::vector<std::vector<Cand>>(NB));
    {
        std::atomic<uint32_t> next{0};
        std::vector<std::thread> pool;
        for (uint32_t w = 0; w < P; ++w)
            pool.emplace_back([&, w] {
                std::vector<uint32_t> run;
                for (uint32_t t; (t = next.fetch_add(64)) < nseq;)
                    for (uint32_t u = t; u < std::min(nseq, t + 64); ++u) {
                        run.clear();
                        skq::sketch_positions(seqs + offs[u], offs[u + 1] - offs[u], k, threshold, run);
                        for (size_t i = 0; i < run.size(); ++i)
                            for (uint32_t d = 1; d <= CHAIN_HOPS && i + d < run.size(); ++d)
                                if (run[i + d] != run[i] && run[i] < len)
                                    part[w][run[i] / span].push_back({run[i], run[i + d], d});
                    }
            });
        for (auto& t : pool) t.join();
    }
    for (auto& pw : part)
        for (auto& pb : pw) out->triples += pb.size();
    std::vector<uint32_t>& ent = out->ent;
    ent.assign(m * skq::CHAIN_WORDS, 0);
    std::vector<uint8_t> built(m, 0);
    std::atomic<uint64_t> nsucc{0};
    auto index_of = [&](uint32_t key) -> int64_t {
        const auto it = std::lower_bound(keys.begin(), keys.end(), key);
        return it != keys.end() && *it == key ? (int64_t)(it - keys.begin()) : -1;
    };
    {
        std::atomic<uint32_t> next{0};
        std::vector<std::thread> pool;
        for (uint32_t w = 0; w < P; ++w)
            pool.emplace_back([&] {
                std::vector<Cand> c;
                std::vector<uint32_t> sk, so;
                uint64_t ns = 0;
                for (uint32_t b; (b = next.fetch_add(1)) < NB;) {
                    c.clear();
                    for (uint32_t q = 0; q < P; ++q) c.insert(c.end(), part[q][b].begin(), part[q][b].end());
                    std::sort(c.begin(), c.end());
                    for (size_t i = 0; i < c.size();) {
                        size_t j = i;
                        while (j < c.size() && c[j].h == c[i].h) ++j;
                        const int64_t x = index_of(c[i].h);
                        if (x >= 0 && !built[x]) {
                            // the key's successors, each once, nearest first
                            sk.clear();
                            so.clear();
                            for (size_t q = i; q < j; ++q) {
                                if (std::find(sk.begin(), sk.end(), c[q].g) != sk.end()) continue;
                                const int64_t y = index_of(c[q].g);
                                if (y < 0) continue;
                                sk.push_back(c[q].g);
                                so.push_back(vals[y]);
                            }
                            ns += chain_entry(ent.data() + (uint64_t)x * skq::CHAIN_WORDS, c[i].h, vals[x], lists,
                                              sk.data(), so.data(), sk.size());
                            built[x] = 1;
                        }
                        i = j;
                    }
                    for (uint32_t q = 0; q < P; ++q) std::vector<Cand>().swap(part[q][b]);  // (this thread's bucket)
                }
                nsucc += ns;
            });
        for (auto& t : pool) t.join();
    }
    // keys no transcript of `seqs` retained still get their own record; word 28 names the entry's
    // key (read by k_map1 over compact tables, where a slot may be asked for a key it does not hold)
    for (uint64_t x = 0; x < m; ++x) {
        if (!built[x]) chain_entry(ent.data() + x * skq::CHAIN_WORDS, keys[x], vals[x], lists, nullptr, nullptr, 0);
        ent[x * skq::CHAIN_WORDS + skq::CHN_W_SELF] = keys[x] ^ skq::CHN_KEY_LIMIT;
    }
    out->nsucc = nsucc.load();
    out->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return out;
}

// one line on stderr per (k, reason) the first time a k slot keeps the wide entries alone
static void chain_note(uint32_t k, const char* why, uint64_t need, uint64_t fr) {
    static std::mutex mu;
    static std::vector<std::pair<uint32_t, std::string>> seen;
    std::lock_guard<std::mutex> g(mu);
    for (auto& x : seen)
        if (x.first == k && x.second == why) return;
    seen.emplace_back(k, why);
    std::fprintf(stderr, "[skq] k=%u: no chained table (%s: %.1f GB needed, %.1f GB free on the device); the k slot "
                 "keeps the wide entries\n", k, why, need / 1e9, fr / 1e9);
}

// slots: the keys' compact slots (chained entries over compact tables, nslots of them), or null
// (one entry per possible key up to the largest)
int build_chain(skq_index* ix, uint32_t slot, const skq_kmer_table& src, const std::vector<uint32_t>& keys,
                const std::vector<uint32_t>& vals, const std::vector<uint32_t>& lists, uint32_t k, const uint8_t* seqs,
                const uint64_t* offs, uint32_t nseq, uint32_t threshold, const std::vector<uint32_t>* slots,
                uint64_t nslots) {
    const uint64_t m = keys.size();
    if (m == 0 || keys.back() >= skq::CHN_KEY_LIMIT) return 0;  // (records hold key ^ CHN_KEY_LIMIT)
    if (slots && slots->size() != m) return fail(-3, "chained table: compact slots missing");
    const uint64_t len = (uint64_t)keys.back() + 1;
    const uint64_t ents = slots ? nslots : len;  // (entries allocated)
    // 128 B per entry, up to SKQ_CHAIN_MB (default 64 GiB) and half the free memory
    uint64_t budget = 65536ull << 20;
    if (const char* e = std::getenv("SKQ_CHAIN_MB")) budget = std::strtoull(e, nullptr, 10) << 20;
    size_t fr = 0, tot = 0;
    // (half of what is free past a 32 GiB reserve for sessions: several indexes may share a device)
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < (32ull << 30) || ents * 128 > (fr - (32ull << 30)) / 2 ||
        ents * 128 > budget) {
        chain_note(k, ents * 128 > budget ? "over SKQ_CHAIN_MB" : "past half the free memory above 32 GiB", ents * 128, fr);
        return 0;
    }
    // the host entries: shared with the other devices building the same tables at the same time
    const ChainKey key{seqs, offs, src.keys, src.offs, src.tids, nseq, k, threshold, m, len, lists.size()};
    std::shared_future<std::shared_ptr<const ChainHost>> fut;
    std::promise<std::shared_ptr<const ChainHost>> prom;
    bool builder = false;
    {
        std::lock_guard<std::mutex> g(g_chain_mu);
        for (auto& x : g_chain_share)
            if (x.key == key) {
                fut = x.fut;
                ++x.users;
            }
        if (!fut.valid()) {
            fut = prom.get_future().share();
            g_chain_share.push_back({key, fut, 1});
            builder = true;
        }
    }
    if (builder) {
        try {
            prom.set_value(chain_host_build(keys, vals, lists, k, seqs, offs, nseq, threshold));
        } catch (...) {
            prom.set_exception(std::current_exception());
        }
    }
    std::shared_ptr<const ChainHost> hc;
    try {
        hc = fut.get();
    } catch (...) {
        hc = nullptr;
    }
    auto done_with = [&] {
        std::lock_guard<std::mutex> g(g_chain_mu);
        for (size_t i = 0; i < g_chain_share.size(); ++i)
            if (g_chain_share[i].key == key && --g_chain_share[i].users == 0) {
                g_chain_share.erase(g_chain_share.begin() + (ptrdiff_t)i);
                break;
            }
    };
    if (!hc) {
        done_with();
        return fail(-3, "chained table build failed (host)");
    }
    uint32_t* dk = nullptr;
    uint4* de = nullptr;
    uint4*& dch = ix->d_chain[slot];
    if (dev_alloc_table(&dch, ents * 8) || dev_alloc(&dk, m) || dev_alloc(&de, m * 8)) {
        // (the device is shared, e.g. several indexes on it: this slot keeps the wide entries)
        dev_free(dk);
        dev_free(de);
        dev_free(dch);
        (void)hipGetLastError();
        done_with();
        chain_note(k, "allocation failed", ents * 128, fr);
        return 0;
    }
    hipStream_t st = nullptr;
    // (the scatter's destinations: the keys themselves, or their compact slots)
    const bool ok = hipMemsetAsync(dch, 0, ents * 128, st) == hipSuccess &&
                    hipMemcpy(dk, slots ? slots->data() : keys.data(), m * 4, hipMemcpyHostToDevice) == hipSuccess &&
                    hipMemcpy(de, hc->ent.data(), m * 128, hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_chain_scatter, dim3((unsigned)((m * 8 + 255) / 256)), dim3(256), 0, st, dch, dk, de, m);
    }
    const bool done = ok && hipGetLastError() == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
    dev_free(dk);
    dev_free(de);
    const uint64_t nsucc = hc->nsucc;
    ix->chain_build_s += builder ? hc->seconds : 0.0;
    ix->chain_host_bytes = std::max<uint64_t>(ix->chain_host_bytes, hc->ent.size() * 4 + hc->triples * 12);
    hc.reset();
    done_with();
    if (!done) {
        dev_free(dch);
        return fail(-3, "chained table build failed");
    }
    ix->chain_len[slot] = len;  // (k_map1: a query past the largest key is no key)
    ix->chain_bytes += ents * 128;
    ix->chain_succ = (ix->chain_succ * ix->chain_slots + (double)nsucc / (double)m) / (ix->chain_slots + 1);
    ++ix->chain_slots;
    return 0;
}

// Probe structure, for ids that fit k_count3: wide tables when they fit SKQ_DIRECT_MB (default
// 49152 MiB) and half the free device memory, else compact tables (a few % of the wide tables'
// size); otherwise 4-B direct tables when they fit, else the bucket table alone.
// SKQ_PROBE = wide | compact | dir | rank | bucket forces one kind (A/B measurements and the
// parity tests, which run every kind; anything else is an error). Dir and rank tables serve
// transcript ids past 2^22, which the wide and compact entries cannot hold.
int build_direct(skq_index* ix, uint32_t ntables, const skq_kmer_table* tables,
                 const std::vector<uint32_t>* dkeys, const std::vector<uint32_t>* dvals,
                 const std::vector<uint32_t>& lists, bool prefer_compact) {
    uint64_t budget = 49152ull << 20;
    if (const char* e = std::getenv("SKQ_DIRECT_MB")) budget = std::strtoull(e, nullptr, 10) << 20;
    if (budget == 0) return 0;
    const char* force = std::getenv("SKQ_PROBE");
    if (force && *force) {
        static const char* kinds[] = {"wide", "compact", "dir", "rank", "bucket"};
        bool known = false;
        for (const char* k : kinds) known |= !std::strcmp(force, k);
        if (!known) return fail(-1, std::string("SKQ_PROBE: unknown probe kind ") + force);
        if (!std::strcmp(force, "bucket")) return 0;
    } else {
        force = nullptr;
    }
    // (prefer_compact: SKQ_CHAIN=2, or the sizing rule of index_create_impl — compact entries first,
    // within the same budget checks as an unforced choice; if their placement fails, the wide
    // entries when they fit, then the other kinds, as an unforced index falls back)
    if (force && !std::strcmp(force, "rank")) return build_rank(ix, ntables, tables, dkeys, dvals);
    uint64_t need = 0, len[SKQ_MAX_K] = {};
    for (uint32_t t = 0; t < ntables; ++t) {
        len[t] = dkeys[t].empty() ? 0 : (uint64_t)dkeys[t].back() + 1;  // keys ascending
        need += len[t] * 4;
    }
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
    if (need == 0) return 0;
    const bool ids_ok = ix->ntx <= (1u << 22) && ix->nlist_words < 0x80000000ull;
    auto forced = [&](const char* kind) { return force && !std::strcmp(force, kind); };
    const bool wide_ok = ids_ok && need * 8 <= budget && need * 8 <= fr / 2;
    if (wide_ok && !prefer_compact && (!force || forced("wide"))) return build_wide(ix, ntables, tables, dkeys, dvals, len);
    if (forced("wide")) return 0;  // forced but does not fit: bucket table
    uint64_t cmp_need = 0;  // compact tables: m / 0.95 slots of 32 B + 2-B pilots per 5 keys, per k
    for (uint32_t t = 0; t < ntables; ++t)
        cmp_need += (uint64_t)std::ceil((double)dkeys[t].size() / 0.95) * 32 + 64 + (dkeys[t].size() + 4) / 5 * 2;
    if (ids_ok && (forced("compact") || (!force && cmp_need <= budget && cmp_need <= fr / 2))) {
        const int rc = build_compact(ix, ntables, tables, dkeys, dvals, lists);
        if (rc == 0 || forced("compact")) return rc;  // (SKQ_PROBE=compact: its error)
        for (auto& d : ix->d_wdir_t) dev_free(d);  // (placement or allocation failed: another kind)
        for (auto& d : ix->d_wpil_t) dev_free(d);
        for (auto& w : ix->wdir) w = nullptr;
        for (auto& w : ix->wpil) w = nullptr;
        (void)hipGetLastError();
    }
    if (wide_ok && prefer_compact && !force) return build_wide(ix, ntables, tables, dkeys, dvals, len);
    if (need > budget || need > fr / 2) return 0;
    hipStream_t st = nullptr;
    uint32_t *dk = nullptr, *dv = nullptr;
    for (uint32_t t = 0; t < ntables; ++t) {
        const uint64_t m = dkeys[t].size();
        if (dev_alloc(&ix->d_dir_t[t], len[t]) || dev_alloc(&dk, m) || dev_alloc(&dv, m)) {
            dev_free(dk);
            dev_free(dv);
            return fail(-3, "direct table allocation failed");
        }
        if (hipMemsetAsync(ix->d_dir_t[t], 0xFF, len[t] * 4, st) != hipSuccess ||
            hipMemcpy(dk, dkeys[t].data(), m * 4, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(dv, dvals[t].data(), m * 4, hipMemcpyHostToDevice) != hipSuccess ||
            skq::launch_dir_scatter(ix->d_dir_t[t], dk, dv, m, st) || hipStreamSynchronize(st) != hipSuccess) {
            dev_free(dk);
            dev_free(dv);
            return fail(-3, "direct table build failed");
        }
        dev_free(dk);
        dev_free(dv);
    }
    ix->dir_bytes = need;
    for (uint32_t i = 0; i < ix->nk; ++i)
        for (uint32_t t = 0; t < ntables; ++t)
            if (tables[t].k == ix->ks[i]) {
                ix->dir[i] = ix->d_dir_t[t];
                ix->dir_len[i] = len[t];
            }
    ix->direct = true;
    ix->mode = 1;
    return 0;
}

}  // namespace

// The side stream runs batch tails (a fused map's slow paths and totals; a large two-kernel batch's
// totals) in batch order. wait_side: a launch-stream point after every side-stream piece of work so
// far (every reader of the running totals, and every batch that does not take the other frame).
static int wait_side(skq_session* s, hipStream_t st) {
    for (int b = 0; b < 2; ++b)
        if (s->side && s->done_rec[b]) HIP_TRY(hipStreamWaitEvent(st, s->ev_done[b], 0));
    return 0;
}

// the host waits for the side stream's work on the current frame (its results) and the totals
static int sync_side(skq_session* s) {
    for (int b = 0; b < 2; ++b)
        if (s->side && s->done_rec[b]) HIP_TRY(hipEventSynchronize(s->ev_done[b]));
    return 0;
}

// the packed sums into the running totals, on st, behind every batch's totals (the readers of
// tx_reads / tx_score call this first)
static int fold_totals(skq_session* s, hipStream_t st) {
    if (!s->acc_reads) return 0;
    if (int rc = wait_side(s, st)) return rc;
    if (skq::launch_fold_totals(s->tx_acc, s->tx_reads, s->tx_score, s->idx->ntx, st)) return fail(-3, "fold failed");
    s->acc_reads = 0;
    return 0;
}

static int ensure_side(skq_session* s) {
    if (s->side) return 0;
    HIP_TRY(hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_map, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_done[0], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&s->ev_done[1], hipEventDisableTiming));
    return 0;
}

extern "C" {

const char* skq_last_error(void) { return g_err.c_str(); }
int skq_version(void) { return 1; }

int skq_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

uint32_t skq_threshold(double fraction) {
    const uint32_t H = 0xFFFFFFFFu;  // std::numeric_limits<uint32_t>::max(), src/sketch.cpp:25
    return static_cast<uint32_t>(H * fraction);
}

static int index_create_impl(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks, uint32_t ntables,
                             const skq_kmer_table* tables, const uint8_t* seqs, const uint64_t* seq_offs,
                             uint32_t nseq, uint32_t threshold, skq_index** out) {
    if (!out) return fail(-1, "out is null");
    *out = nullptr;
    if (nk == 0 || nk > SKQ_MAX_K) return fail(-1, "k list must hold 1..SKQ_MAX_K entries");
    if (ntables > SKQ_MAX_K) return fail(-1, "too many tables");
    for (uint32_t i = 0; i < nk; ++i)
        if (ks[i] == 0) return fail(-1, "k must be greater than 0");
    DeviceGuard g(device);
    auto* ix = new skq_index();
    ix->device = device;
    ix->ntx = ntx;
    ix->nk = nk;
    ix->mink = ~0u;
    for (uint32_t i = 0; i < nk; ++i) {
        ix->ks[i] = ks[i];
        ix->maxk = std::max(ix->maxk, ks[i]);
        ix->mink = std::min(ix->mink, ks[i]);
    }
    // host image (skq_internal.h): distinct postings lists stored once ([n, tid...], 16-B
    // aligned) and, per distinct k, a table of 64-B buckets mapping keys to list offsets
    std::vector<uint32_t> buckets;
    std::vector<uint32_t> lists;
    std::unordered_map<uint64_t, std::vector<uint32_t>> seen;  // list hash -> offsets
    auto list_offset = [&](const uint32_t* a, uint64_t n) -> uint64_t {
        uint64_t h = 1469598103934665603ull ^ n;
        for (uint64_t q = 0; q < n; ++q) h = (h ^ a[q]) * 1099511628211ull;
        auto& cand = seen[h];
        for (uint32_t off : cand)
            if (lists[off] == n && std::equal(a, a + n, lists.begin() + off + 1)) return off;
        const uint64_t off = lists.size();
        lists.push_back((uint32_t)n);
        lists.insert(lists.end(), a, a + n);
        lists.resize((lists.size() + 3) & ~3ull, 0);
        cand.push_back((uint32_t)off);
        return off;
    };
    uint64_t tbase[SKQ_MAX_K] = {};
    uint32_t tnb[SKQ_MAX_K] = {}, tprobe[SKQ_MAX_K] = {};
    std::vector<uint32_t> dkeys[SKQ_MAX_K], dvals[SKQ_MAX_K];  // per table, for the direct table
    for (uint32_t t = 0; t < ntables; ++t) {
        const skq_kmer_table& T = tables[t];
        for (uint32_t u = 0; u < t; ++u)
            if (tables[u].k == T.k) { delete ix; return fail(-1, "duplicate table for one k"); }
        std::vector<std::pair<uint32_t, uint32_t>> recs;  // (key, list offset)
        recs.reserve(T.nkeys);
        for (uint64_t j = 0; j < T.nkeys; ++j) {
            if (j && T.keys[j] <= T.keys[j - 1]) { delete ix; return fail(-1, "keys must be ascending and unique"); }
            const uint64_t a = T.offs[j], b = T.offs[j + 1];
            if (b < a) { delete ix; return fail(-1, "offsets must be non-decreasing"); }
            for (uint64_t q = a; q < b; ++q) {
                if (T.tids[q] >= ntx) { delete ix; return fail(-1, "transcript id out of range"); }
                if (q > a && T.tids[q] <= T.tids[q - 1]) { delete ix; return fail(-1, "tids of a key must be ascending and unique"); }
            }
            if (b == a) continue;  // a key with no postings behaves as a miss
            const uint64_t off = list_offset(T.tids + a, b - a);
            if (off >= 0xFFFFFFF0ull) { delete ix; return fail(-1, "index too large"); }
            recs.emplace_back(T.keys[j], (uint32_t)off);
            ix->npostings += b - a;
            ix->max_list = std::max<uint32_t>(ix->max_list, (uint32_t)(b - a));
        }
        const uint64_t nb64 = std::max<uint64_t>(64, (uint64_t)(recs.size() / (skq::BUCKET_MAX_RECORDS * 0.80)) + 1);
        if (nb64 >= 0xFFFFFFFFull) { delete ix; return fail(-1, "index too large"); }
        const uint32_t nb = (uint32_t)nb64;
        tbase[t] = buckets.size() / skq::BUCKET_WORDS;
        tnb[t] = nb;
        buckets.resize(buckets.size() + (uint64_t)nb * skq::BUCKET_WORDS, 0);
        uint32_t* B = buckets.data() + tbase[t] * skq::BUCKET_WORDS;
        // place records in home-bucket order, each at the first bucket from home with room
        std::vector<std::pair<uint32_t, uint32_t>> order;  // (home, record)
        order.reserve(recs.size());
        for (uint32_t j = 0; j < recs.size(); ++j) order.emplace_back(skq::home_bucket(recs[j].first, nb), j);
        std::sort(order.begin(), order.end());
        uint32_t maxd = 0;
        for (const auto& [home, j] : order) {
            uint32_t b = home, d = 0;
            while ((B[(uint64_t)b * skq::BUCKET_WORDS] & 7u) == skq::BUCKET_MAX_RECORDS) {
                B[(uint64_t)b * skq::BUCKET_WORDS] |= 8u;  // a key homed here or earlier continues
                b = b + 1 == nb ? 0 : b + 1;
                if (++d > nb) { delete ix; return fail(-1, "bucket table overflow"); }
            }
            maxd = std::max(maxd, d);
            uint32_t* H = B + (uint64_t)b * skq::BUCKET_WORDS;
            const uint32_t m = H[0] & 7u;
            H[1 + m] = recs[j].first;
            H[skq::BUCKET_LIST0 + m] = recs[j].second;
            H[0] = (H[0] & ~7u) | (m + 1);
        }
        tprobe[t] = maxd + 1;
        dkeys[t].reserve(recs.size());
        dvals[t].reserve(recs.size());
        for (const auto& [key, off] : recs) {
            dkeys[t].push_back(key);
            dvals[t].push_back(off);
        }
    }
    lists.resize(lists.size() + 4, 0);  // a uint4 read at any list start stays inside
    for (uint32_t i = 0; i < nk; ++i) {
        ix->tabs[i].present = 0;
        for (uint32_t t = 0; t < ntables; ++t)
            if (tables[t].k == ks[i]) {
                ix->tabs[i].bucket_base = tbase[t];
                ix->tabs[i].nbuckets = tnb[t];
                ix->tabs[i].max_probe = tprobe[t];
                ix->tabs[i].present = 1;
            }
    }
    // per k slot: E[in*4 + out] = seed(in) ^ rot33^k(seed(out)) (one roll step's XOR), then the
    // 4 seeds for the first window
    std::vector<uint64_t> roll((size_t)nk * 16 + 4, 0);
    for (uint32_t i = 0; i < nk; ++i)
        for (uint32_t in = 0; in < 4; ++in)
            for (uint32_t o = 0; o < 4; ++o)
                roll[i * 16 + in * 4 + o] = skq::SEED33[in] ^ skq::rot33(skq::SEED33[o], ks[i]);
    for (uint32_t c = 0; c < 4; ++c) roll[(size_t)nk * 16 + c] = skq::SEED33[c];
    ix->nbucket_words = buckets.size();
    ix->nlist_words = lists.size();
    int rc = 0;
    if ((rc = dev_alloc(&ix->d_buckets, buckets.size())) || (rc = dev_alloc(&ix->d_lists, lists.size())) ||
        (rc = dev_alloc(&ix->d_rolltab, roll.size()))) {
        skq_index_free(ix);
        return rc;
    }
    if (hipMemcpy(ix->d_buckets, buckets.data(), buckets.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ix->d_lists, lists.data(), lists.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ix->d_rolltab, roll.data(), roll.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
        skq_index_free(ix);
        return fail(-3, "index upload failed");
    }
    // SKQ_CHAIN: 0 no chained tables, 1 chained over whichever probe structure the index takes,
    // 2 chained over compact tables (the compact probe unless SKQ_PROBE names another)
    const char* chain_env = std::getenv("SKQ_CHAIN");
    const int cm = chain_env ? std::atoi(chain_env) : 1;
    if (cm < 0 || cm > 2) {
        skq_index_free(ix);
        return fail(-1, "SKQ_CHAIN: 0, 1 or 2");
    }
    const bool chain_ok = seqs && seq_offs && nk <= (uint32_t)skq::NK_FAST && ix->ntx <= (1u << 22) &&
                          ix->nlist_words < 0x80000000ull;
    // the index sized by the device: wide entries + chained tables per possible key where both fit
    // (the fastest), else compact entries + chained tables per present key (cfg3: 0.77 GB against
    // 34.4 GB, k_map1 19 % slower, and 20 % faster than the wide entries alone)
    bool prefer_compact = cm == 2 && chain_ok;
    if (cm == 1 && chain_ok && !std::getenv("SKQ_PROBE")) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            uint64_t wide = 0, budget = 49152ull << 20, cbudget = 65536ull << 20;
            if (const char* e = std::getenv("SKQ_DIRECT_MB")) budget = std::strtoull(e, nullptr, 10) << 20;
            if (const char* e = std::getenv("SKQ_CHAIN_MB")) cbudget = std::strtoull(e, nullptr, 10) << 20;
            for (uint32_t t = 0; t < ntables; ++t) wide += dkeys[t].empty() ? 0 : ((uint64_t)dkeys[t].back() + 1) * 32;
            bool fits = wide <= budget && wide <= fr / 2;  // (build_direct's rule for the wide entries)
            uint64_t f = fr > wide ? fr - wide : 0;
            for (uint32_t i = 0; i < nk && fits; ++i)  // (build_chain's rule, slot by slot)
                for (uint32_t t = 0; t < ntables; ++t)
                    if (tables[t].k == ks[i] && !dkeys[t].empty()) {
                        const uint64_t c = ((uint64_t)dkeys[t].back() + 1) * 128;
                        fits = f >= (32ull << 30) && c <= (f - (32ull << 30)) / 2 && c <= cbudget;
                        f -= fits ? c : 0;
                    }
            prefer_compact = !fits;
        }
    }
    if (int rc2 = build_direct(ix, ntables, tables, dkeys, dvals, lists, prefer_compact)) {
        skq_index_free(ix);
        return rc2;
    }
    // chained tables (per k slot, ids within 22 bits, transcripts given): the default (SKQ_CHAIN = 0
    // turns them off; cfg3: k_map1 0.91 against 1.35 ms over the wide entries alone);
    // a slot whose table does not fit after all keeps the probe entries alone
    // (the entry list behind the chain step gathers wide or compact entries)
    if (chain_ok && cm != 0 && (ix->mode == 3 || ix->mode == 5))
        for (uint32_t i = 0; i < nk; ++i)
            for (uint32_t t = 0; t < ntables; ++t)
                if (tables[t].k == ks[i]) {
                    const bool cmp = ix->mode == 5;
                    if (int rc2 = build_chain(ix, i, tables[t], dkeys[t], dvals[t], lists, ks[i], seqs, seq_offs, nseq, threshold,
                                              cmp ? &ix->cmp_slots_t[t] : nullptr, cmp ? ix->dir_len[i] : 0)) {
                        skq_index_free(ix);
                        return rc2;
                    }
                }
    for (auto& v : ix->cmp_slots_t) std::vector<uint32_t>().swap(v);
    *out = ix;
    return 0;
}

int skq_index_create(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks, uint32_t ntables,
                     const skq_kmer_table* tables, skq_index** out) {
    return index_create_impl(device, ntx, nk, ks, ntables, tables, nullptr, nullptr, 0, 0, out);
}

int skq_index_create_chained(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks, uint32_t ntables,
                             const skq_kmer_table* tables, const uint8_t* seqs, const uint64_t* seq_offs,
                             uint32_t nseq, uint32_t threshold, skq_index** out) {
    if (nseq && (!seqs || !seq_offs)) return fail(-1, "null sequences");
    return index_create_impl(device, ntx, nk, ks, ntables, tables, seqs, seq_offs, nseq, threshold, out);
}

int skq_index_free(skq_index* ix) {
    if (!ix) return 0;
    DeviceGuard g(ix->device);
    for (auto& d : ix->d_dir_t) dev_free(d);
    for (auto& d : ix->d_wdir_t) dev_free(d);
    for (auto& d : ix->d_wpil_t) dev_free(d);
    for (auto& d : ix->d_rank_t) dev_free(d);
    for (auto& d : ix->d_rovf_t) dev_free(d);
    for (auto& d : ix->d_chain) dev_free(d);
    dev_free(ix->d_buckets);
    dev_free(ix->d_lists);
    dev_free(ix->d_rolltab);
    delete ix;
    return 0;
}

int skq_index_stats(const skq_index* ix, uint64_t* device_bytes, uint64_t* npostings, uint32_t* max_list) {
    if (!ix) return fail(-1, "null index");
    if (device_bytes) *device_bytes = ix->nbucket_words * 4 + ix->nlist_words * 4 + ix->dir_bytes + ix->chain_bytes;
    if (npostings) *npostings = ix->npostings;
    if (max_list) *max_list = ix->max_list;
    return 0;
}

int skq_session_slow_reads(skq_session* s, uint32_t* sketch_slow, uint32_t* chain_slow) {
    if (!s) return fail(-1, "null session");
    DeviceGuard g(s->idx->device);
    if (int rc = sync_side(s)) return rc;
    uint32_t c[skq::C_WORDS];
    HIP_TRY(hipMemcpy(c, s->f.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    if (sketch_slow) *sketch_slow = c[skq::C_OVF1];
    if (chain_slow) *chain_slow = c[skq::C_OVF2];
    return 0;
}

int skq_session_slow_counts(skq_session* s, uint32_t* counts) {
    if (!s || !counts) return fail(-1, "null argument");
    DeviceGuard g(s->idx->device);
    if (int rc = sync_side(s)) return rc;
    uint32_t c[skq::C_WORDS];
    HIP_TRY(hipMemcpy(c, s->f.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    counts[0] = c[skq::C_OVF1];
    counts[1] = c[skq::C_OVF2];
    counts[2] = c[skq::C_OVF3];
    counts[3] = c[skq::C_OVF4];
    return 0;
}

int skq_index_direct(const skq_index* ix) { return ix && ix->direct ? ix->mode : 0; }
double skq_index_chained(const skq_index* ix) { return ix && ix->chain_slots ? 1.0 + ix->chain_succ : 0.0; }

int skq_index_chain_build(const skq_index* ix, double* host_seconds, uint64_t* host_peak_bytes) {
    if (!ix) return fail(-1, "null index");
    if (host_seconds) *host_seconds = ix->chain_build_s;
    if (host_peak_bytes) *host_peak_bytes = ix->chain_host_bytes;
    return 0;
}

// one frame's buffers for the session's sizes (the hashes and lofs: ensure_hashes)
static int frame_alloc(skq_session* s, Frame& fr, uint32_t hcap) {
    const uint64_t R = s->max_reads;
    const uint32_t nk = s->idx->nk;
    int rc = 0;
    if ((rc = dev_alloc(&fr.status, R)) || (rc = dev_alloc(&fr.hash_cnt, R * nk)) ||
        (rc = dev_alloc(&fr.hash_ext, s->hash_ext_cap)) || (rc = dev_alloc(&fr.ovf1, s->ovf_cap)) ||
        (rc = dev_alloc(&fr.ovf2, s->ovf_cap)) || (rc = dev_alloc(&fr.ovf3, s->ovf_cap)) ||
        (rc = dev_alloc(&fr.ovf4, s->ovf_cap)) || (rc = dev_alloc(&fr.cand_cnt, R)) || (rc = dev_alloc(&fr.pflag, R)) ||
        (rc = dev_alloc(&fr.cand_tid, R * skq::CCAP)) || (rc = dev_alloc(&fr.cand_wtot, (R + 63) / 64)) ||
        (rc = dev_alloc(&fr.cand_score, R * skq::CCAP)) || (rc = dev_alloc(&fr.cand_ext, 2 * s->cand_ext_cap)) ||
        (rc = dev_alloc(&fr.scratch, s->scratch_cap)) || (rc = dev_alloc(&fr.ctrl_mem, 2 * skq::C_WORDS)))
        return rc;
    fr.ctrl = fr.ctrl_mem;
    if (hipMemset(fr.ctrl_mem, 0, 2 * skq::C_WORDS * 4) != hipSuccess) return fail(-3, "memset failed");
    if (dev_alloc(&fr.hashes, R * nk * (uint64_t)hcap) || dev_alloc(&fr.lofs, R * nk * (uint64_t)hcap)) return -3;
    fr.hcap_alloc = hcap;
    return 0;
}

static void frame_free(Frame& fr) {
    dev_free(fr.status);
    dev_free(fr.hash_cnt);
    dev_free(fr.hashes);
    dev_free(fr.lofs);
    dev_free(fr.pflag);
    dev_free(fr.hash_ext);
    dev_free(fr.ovf1);
    dev_free(fr.ovf2);
    dev_free(fr.ovf3);
    dev_free(fr.ovf4);
    dev_free(fr.cand_cnt);
    dev_free(fr.cand_tid);
    dev_free(fr.cand_score);
    dev_free(fr.cand_wtot);
    dev_free(fr.cand_ext);
    dev_free(fr.scratch);
    dev_free(fr.ctrl_mem);
    dev_free(fr.ktab);
    dev_free(fr.kcnt);
    dev_free(fr.stash);
    fr = Frame{};
}

int skq_session_create(skq_index* ix, uint64_t max_reads, uint32_t max_len, skq_session** out) {
    if (!ix || !out) return fail(-1, "null argument");
    *out = nullptr;
    if (max_reads == 0) max_reads = 1;
    if (max_reads > skq::MAX_BATCH) return fail(-1, "max_reads must be below 2^24 (split larger batches)");
    DeviceGuard g(ix->device);
    auto* s = new skq_session();
    s->idx = ix;
    s->max_reads = max_reads;
    s->max_len = std::max<uint32_t>(max_len, 1);
    s->ovf_cap = (uint32_t)max_reads;  // any read may take a slow path (e.g. > 4 k slots)
    const uint32_t Lc = std::min<uint32_t>(s->max_len, skq::LFAST);
    // (8-word multiples: packed-layout runs start 8-word aligned; run marks address < RUN_MAX words)
    s->hash_ext_cap = std::min<uint64_t>(skq::RUN_MAX, ((std::max<uint64_t>(1ull << 24, (uint64_t)s->ovf_cap * 4) + 7) & ~7ull) +
                                                         (uint64_t)skq::SW_GRID * skq::SW_HCH);
    s->cand_ext_cap = (1ull << 22) + (uint64_t)skq::SW_GRID * skq::SW_CCH;
    s->scratch_cap = 1ull << 24;
    const uint32_t hcap0 = pick_hcap(Lc, ix->mink, skq_threshold((double)0.05f));
    int rc = 0;
    if ((rc = frame_alloc(s, s->f, hcap0)) || (rc = dev_alloc(&s->tx_reads, ix->ntx)) ||
        (rc = dev_alloc(&s->tx_score, ix->ntx)) || (rc = dev_alloc(&s->tx_acc, ix->ntx))) {
        skq_session_free(s);
        return rc;
    }
    // totals buckets: at most WG buckets of at most 2^14 ids (the LDS histogram), else direct
    // (2^12-id buckets for large transcript sets, 2^13 for small ones: cfg3 1.071 against 1.094 ms
    // per step with 1024 k_bin_sum workgroups, cfg2 the same either way; profiles/r5_totals_sweep.log)
    s->bin_bits = ix->ntx > (1u << 16) ? 12u : 13u;
    if (const char* e = dev_env("SKQ_BIN_BITS")) s->bin_bits = (uint32_t)std::max(8, std::min(14, std::atoi(e)));
    while (((uint64_t)ix->ntx + (1ull << s->bin_bits) - 1) >> s->bin_bits > (uint64_t)skq::WG) ++s->bin_bits;
    s->bin_nb = s->bin_bits <= 14 ? (uint32_t)(((uint64_t)ix->ntx + (1ull << s->bin_bits) - 1) >> s->bin_bits) : 0u;
    const uint64_t nW = (max_reads + skq::WG - 1) / skq::WG;
    const uint64_t rwords = nW * skq::WG * skq::CCAP;
    if (s->bin_nb && ((rc = dev_alloc(&s->bin_hdr, (uint64_t)(s->bin_nb + 1) * nW)) ||
                      (rc = dev_alloc(&s->bin_region, rwords)))) {
        skq_session_free(s);
        return rc;
    }
    if (hipMemset(s->tx_reads, 0, ix->ntx * 8ull) != hipSuccess ||
        hipMemset(s->tx_acc, 0, ix->ntx * 8ull) != hipSuccess ||
        hipMemset(s->tx_score, 0, ix->ntx * 8ull) != hipSuccess) {
        skq_session_free(s);
        return fail(-3, "memset failed");
    }
    *out = s;
    return 0;
}

int skq_session_free(skq_session* s) {
    if (!s) return 0;
    DeviceGuard g(s->idx->device);
    for (auto& t : s->timed) {
        (void)hipEventDestroy(t.start);
        (void)hipEventDestroy(t.stop);
    }
    if (s->ev_snap[0]) (void)hipEventDestroy(s->ev_snap[0]);
    if (s->ev_snap[1]) (void)hipEventDestroy(s->ev_snap[1]);
    if (s->side) {
        (void)hipStreamSynchronize(s->side);
        (void)hipStreamDestroy(s->side);
        (void)hipEventDestroy(s->ev_fork);
        (void)hipEventDestroy(s->ev_map);
        (void)hipEventDestroy(s->ev_done[0]);
        (void)hipEventDestroy(s->ev_done[1]);
    }
    frame_free(s->f);
    frame_free(s->alt);
    dev_free(s->bin_hdr);
    dev_free(s->bin_region);
    dev_free(s->tx_acc);
    dev_free(s->tx_reads);
    dev_free(s->tx_score);
    delete s;
    return 0;
}


// prep: fill *prep and the session's batch state without launching (the fused map launches)
static int sketch_impl(skq_session* s, const uint8_t* d_reads, const uint64_t* d_offs, uint32_t fixed_len,
                       uint64_t n_reads, uint32_t max_len, uint32_t threshold, int nthash, void* stream,
                       skq::SketchParams* prep = nullptr) {
    if (!s) return fail(-1, "null session");
    if (n_reads > s->max_reads) return fail(-1, "batch larger than the session's max_reads");
    if (n_reads && !d_reads) return fail(-1, "null reads");
    if (!d_offs) max_len = fixed_len;
    DeviceGuard g(s->idx->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const skq_index* ix = s->idx;
    const uint32_t Lc = std::max<uint32_t>(1, std::min<uint32_t>(std::min(max_len, s->max_len), skq::LFAST));
    const uint32_t hcap = pick_hcap(Lc, ix->mink, threshold);
    if (int rc = ensure_hashes(s, hcap)) return rc;
    skq::SketchParams p{};
    p.reads = d_reads;
    p.offs = d_offs;
    p.fixed_len = fixed_len;
    p.n = n_reads;
    p.nk = ix->nk;
    p.maxk = ix->maxk;
    for (uint32_t i = 0; i < ix->nk; ++i) p.ks[i] = ix->ks[i];
    p.threshold = threshold;
    p.tile_chunks = (64 * Lc + 31) / 16 + 1;  // per wave
    p.hcap = hcap;
    p.ovf_cap = s->ovf_cap;
    p.rolltab = ix->d_rolltab;
    p.status = s->f.status;
    p.hash_cnt = s->f.hash_cnt;
    p.hashes = s->f.hashes;
    p.hash_ext = s->f.hash_ext;
    p.hash_ext_cap = s->hash_ext_cap - (uint64_t)skq::SW_GRID * skq::SW_HCH;  // (the rest: k_slow_wave's stretches)
    p.ctrl = s->f.ctrl;
    p.ovf1 = s->f.ovf1;
    p.ovf_word = skq::C_OVF1;
    p.fuse = ix->mode;
    for (uint32_t i = 0; i < ix->nk; ++i) {
        p.dir[i] = ix->dir[i];
        p.dir_len[i] = ix->dir_len[i];
        p.rank[i] = ix->rank[i];
        p.rovf[i] = ix->rovf[i];
    }
    p.lofs = s->f.lofs;
    p.pflag = s->f.pflag;
    p.nthash = nthash;
    if (prep) {
        *prep = p;
    } else {
        if (int rc = wait_side(s, st)) return rc;  // (the frame's previous tail, the totals' bins)
        s->zeroed[s->fid] = false;
        s->tail_side[s->fid] = false;
        HIP_TRY(hipMemsetAsync(s->f.ctrl, 0, 8 * 4, st));
        hipEvent_t t0{};
        record(s, 0, &t0, st);
        if (skq::launch_sketch(p, stream)) return fail(-3, "sketch launch failed");
        record_stop(s, 0, t0, st);
        if (skq::launch_sketch_slow(p, stream)) return fail(-3, "sketch slow-path launch failed");
    }
    s->hcap = hcap;
    s->n_reads = n_reads;
    s->have_sketch = true;
    s->have_chain = false;
    s->hash_packed = false;
    s->probed = ix->direct;
    s->x_hashes = nullptr;
    s->x_offs = nullptr;
    return 0;
}

int skq_sketch(skq_session* s, const uint8_t* d_reads, const uint64_t* d_offs, uint32_t fixed_len,
               uint64_t n_reads, uint32_t max_len, uint32_t threshold, void* stream) {
    return sketch_impl(s, d_reads, d_offs, fixed_len, n_reads, max_len, threshold, 0, stream);
}

int skq_sketch_seqs(skq_session* s, const uint8_t* d_seqs, const uint64_t* d_offs, uint32_t fixed_len,
                    uint64_t n_seqs, uint32_t max_len, uint32_t threshold, void* stream) {
    return sketch_impl(s, d_seqs, d_offs, fixed_len, n_seqs, max_len, threshold, 1, stream);
}

// The tail of a batch: the slow paths, then the per-transcript totals (k_bin_packed over the fused
// map's packed candidates, or k_bin_sum over the bins the count kernel wrote, then k_fold_totals:
// atomics into the running totals, commuting with the slow paths' direct adds).
// side = true (a fused map that took the other frame): the whole tail runs on the side stream,
// beside the next batch's map on the launch stream (the batch tail); ev_done of the
// frame follows it. Else the slow paths run on the launch stream and the totals, for batches of
// 512k+ reads, on the side stream (the launch stream waits for them before it bins again).
// bins already written for this batch (the count kernels' epilogue); else launch_bin writes them
// (k_bin, or k_bin_packed over the fused map's packed candidates)
static int binned(const skq::ChainParams& p) { return p.slow_totals && !p.cpack ? 1 : 0; }

static int chain_tail(skq_session* s, const skq::SketchParams* sp, const skq::ChainParams& p, int accumulate,
                      hipStream_t st, bool side, hipEvent_t map_end = nullptr) {
    hipEvent_t t0{};
    const bool totals = accumulate != 0;
    s->last_st = st;
    const bool fork = side || (totals && p.slow_totals && !p.cpack && p.n >= (1u << 19));
    hipStream_t tq = st;  // the stream of the totals
    if (fork) {
        if (int rc = ensure_side(s)) return rc;
        if (!map_end) {  // (else the event bound to the map's dispatch: no marker on the launch stream)
            HIP_TRY(hipEventRecord(s->ev_fork, st));
            map_end = s->ev_fork;
        }
        HIP_TRY(hipStreamWaitEvent(s->side, map_end, 0));
        tq = s->side;
    }
    hipStream_t sq = side ? s->side : st;  // the stream of the slow paths
    if (!fork && totals)
        if (int rc = wait_side(s, st)) return rc;  // (tx_acc and the bins: an earlier batch's totals may run)
    auto do_totals = [&]() -> int {
        if (!totals) return 0;
        // (timed on the side stream only: on the launch stream a pair of timing events is ~5 us of
        // the step between two maps)
        if (fork) record(s, 3, &t0, tq);
        // the packed sums fold when this batch could carry a transcript's reads past 2^24 (every
        // earlier writer of tx_acc is ahead of tq: the side stream runs tails in order, and a
        // launch-stream tail waited for it above)
        if (s->acc_reads + p.n > skq::MAX_BATCH) {
            if (skq::launch_fold_totals(s->tx_acc, s->tx_reads, s->tx_score, s->idx->ntx, tq)) return fail(-3, "fold failed");
            s->acc_reads = 0;
        }
        const int rb = skq::launch_bin(p, binned(p), tq, fork);
        if (rb < 0) return fail(-3, "totals launch failed");
        s->acc_reads += p.n;
        if (fork) record_stop(s, 3, t0, tq);
        return 0;
    };
    // (with the count kernel's bins, a two-kernel batch's totals go first: its slow paths add their
    // own reads' totals directly; else k_bin reads every read's final list, the slow ones' too)
    const bool totals_first = !side && p.slow_totals;
    if (totals_first)
        if (int rc = do_totals()) return rc;
    if (sp && (p.wide == 1 || p.wide == 3) && p.nk <= (uint32_t)skq::NK_FAST) {
        // the fused map's slow reads: the wave path first, then k_general_slow for what it leaves
        if (int rc = skq::launch_slow_wave(*sp, p, s->f.ovf3, s->f.ovf4, sq))
            return fail(-3, rc == -4 ? "slow path: unsupported tables" : "slow-path launch failed");
        skq::SketchParams sp2 = *sp;
        sp2.ovf1 = s->f.ovf3;
        sp2.ovf_word = skq::C_OVF3;
        skq::ChainParams p2 = p;
        p2.ovf2 = s->f.ovf4;
        p2.ovf_word = skq::C_OVF4;
        // (32 workgroups: the general reads are rare — none at cfg2, 3, 5 — and each of its workgroups
        // needs 33 KB of LDS, which beside a running map only frees up as map workgroups retire. On
        // the launch stream it also zeroes the frame's other control words for the next batch.)
        uint32_t* zn = side ? nullptr : (s->f.ctrl == s->f.ctrl_mem ? s->f.ctrl_mem + skq::C_WORDS : s->f.ctrl_mem);
        if (skq::launch_general_slow(sp2, p2, sq, 32, zn)) return fail(-3, "general slow-path launch failed");
        if (zn) s->f.other_zeroed = true;
    } else {
        if (sp && skq::launch_sketch_slow(*sp, sq)) return fail(-3, "sketch slow-path launch failed");
        if (skq::launch_chain_slow(p, sq)) return fail(-3, "chain slow-path launch failed");
    }
    if (!totals_first)
        if (int rc = do_totals()) return rc;
    if (fork) {
        HIP_TRY(hipEventRecord(s->ev_done[s->fid], s->side));
        s->done_rec[s->fid] = true;
    }
    return 0;
}

// SKQ_MAPK=1 (development): the multi-k map as one k_mapk launch (every workgroup runs the k slots
// in turn) instead of one k_map1 launch per k slot: 1.4 % slower at cfg5 (its loop holds 128
// VGPRs, 4 waves per SIMD against the passes' 5; profiles/r5_mapk_ab.log), so not the default.
// Read at every map, so one process can run both.
static bool mapk_dev() {
    const char* e = dev_env("SKQ_MAPK");
    return e && std::atoi(e) == 1;
}

// SKQ_ABLATE (development phase pricing: k_map1 skips phases, so results are WRONG) is honoured
// only beside SKQ_DEV=1, and announced once on stderr whenever it is active
static uint32_t ablate_mask() {
    static const uint32_t m = [] {
        const char* e = std::getenv("SKQ_ABLATE");
        const char* dev = std::getenv("SKQ_DEV");
        if (!e || !*e) return 0u;
        const uint32_t v = (uint32_t)std::strtoul(e, nullptr, 0);
        if (!dev || std::atoi(dev) != 1) {
            std::fprintf(stderr, "[skq] SKQ_ABLATE=%s ignored (a development switch: set SKQ_DEV=1 as well)\n", e);
            return 0u;
        }
        if (v) std::fprintf(stderr, "[skq] SKQ_ABLATE=0x%x ACTIVE: k_map1 skips phases, results are wrong\n", v);
        return v;
    }();
    return m;
}

static int chain_impl(skq_session* s, uint64_t n, const uint8_t* status, const uint32_t* hash_cnt,
                      const uint32_t* hashes, const uint64_t* hash_offs, const uint8_t* present,
                      uint32_t hcap, double fraction, int accumulate, bool probed, void* stream,
                      skq::ChainParams* prep = nullptr) {
    DeviceGuard g(s->idx->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const skq_index* ix = s->idx;
    if (!prep)  // (two-kernel path: the current frame, once no side-stream work has it)
        if (int rc = wait_side(s, st)) return rc;
    skq::ChainParams p{};
    p.n = n;
    p.nk = ix->nk;
    p.hcap = hcap;
    p.fraction = fraction;
    p.accumulate = accumulate;
    p.ovf_cap = s->ovf_cap;
    p.status = status;
    p.hash_cnt = hash_cnt;
    p.hashes = hashes;
    p.hpack = hashes == s->f.hashes && s->hash_packed ? 1u : 0u;
    p.hash_ext = s->f.hash_ext;
    p.hash_offs = hash_offs;
    p.present = present;
    p.buckets = ix->d_buckets;
    p.lists = ix->d_lists;
    for (uint32_t i = 0; i < ix->nk; ++i) p.tabs[i] = ix->tabs[i];
    p.cand_cnt = s->f.cand_cnt;
    p.cand_tid = s->f.cand_tid;
    p.cand_score = s->f.cand_score;
    p.cand_ext = s->f.cand_ext;
    p.cand_ext_cap = s->cand_ext_cap - (uint64_t)skq::SW_GRID * skq::SW_CCH;  // (the rest: k_slow_wave's stretches)
    p.scratch = s->f.scratch;
    p.scratch_cap = s->scratch_cap;
    p.tx_acc = s->tx_acc;
    p.ktab = s->f.ktab;
    p.kcnt = s->f.kcnt;
    p.tx_reads = s->tx_reads;
    p.tx_score = s->tx_score;
    p.ctrl = s->f.ctrl;
    p.ovf2 = s->f.ovf2;
    p.ovf_word = skq::C_OVF2;
    p.lofs = s->f.lofs;
    p.pflag = s->f.pflag;
    // lofs stride: the sketch's hcap when it probed (fused), else k_probe's own capacity
    p.lcap = probed ? hcap : std::min<uint32_t>(s->f.hcap_alloc, skq::HFAST);
    // wide tables: the count kernel reads the sketch's hashes and gathers the entries itself
    p.wide = !probed ? 0 : ix->mode == 3 ? 1 : ix->mode == 5 ? 3 : 0;
    if (p.wide) {
        p.lofs = const_cast<uint32_t*>(hashes);
        for (uint32_t i = 0; i < ix->nk; ++i) {
            p.wdir[i] = ix->wdir[i];
            p.wdir_len[i] = ix->dir_len[i];
            p.wpil[i] = ix->wpil[i];
            p.wnb[i] = ix->wnb[i];
            p.wseed[i] = ix->wseed[i];
        }
    }
    for (uint32_t i = 0; i < SKQ_MAX_K; ++i) {
        p.chain[i] = reinterpret_cast<const uint32_t*>(ix->d_chain[i]);
        p.chain_len[i] = ix->chain_len[i];
    }
    p.stamps = s->stamps;
    p.ablate = ablate_mask();
    p.ntx = ix->ntx;
    p.bin_bits = s->bin_bits;
    p.bin_nb = s->bin_nb;
    p.bin_hdr = s->bin_hdr;
    p.bin_region = s->bin_region;
    p.slow_totals = accumulate && skq::count_bins(p);
    if (prep) {
        *prep = p;
        return 0;
    }
    s->cand_packed = false;  // (the chain kernels write the padded rows)
    s->zeroed[s->fid] = false;
    s->tail_side[s->fid] = false;
    HIP_TRY(hipMemsetAsync(s->f.ctrl + 8, 0, 8 * 4, st));
    hipEvent_t t0{};
    if (!probed) {
        record(s, 1, &t0, st);
        if (skq::launch_probe(p, stream)) return fail(-3, "probe launch failed");
        record_stop(s, 1, t0, st);
    }
    record(s, 2, &t0, st);
    if (skq::launch_count(p, stream)) return fail(-3, "count launch failed");
    record_stop(s, 2, t0, st);
    if (int rc = chain_tail(s, nullptr, p, accumulate, st, false)) return rc;
    s->have_chain = true;
    return 0;
}

int skq_chain(skq_session* s, double fraction, int accumulate, void* stream) {
    if (!s) return fail(-1, "null session");
    if (!s->have_sketch) return fail(-1, "no sketch to chain: call skq_sketch first");
    return chain_impl(s, s->n_reads, s->f.status, s->f.hash_cnt, s->f.hashes, nullptr, nullptr, s->hcap,
                      fraction, accumulate, s->probed, stream);
}

// Fused map: k_map1 (compact or wide tables, one k slot, a raw capacity of 16 or 32) or
// k_map1 passes (compact or wide tables, 2..4 k slots); anything else takes the two-kernel path (a caller
// can always ask for that path itself with skq_sketch + skq_chain)
static bool map_fusable(const skq_session* s, const uint64_t* d_offs, uint32_t fixed_len, uint32_t max_len,
                        uint32_t threshold) {
    const skq_index* ix = s->idx;
    if (!d_offs) max_len = fixed_len;
    const uint32_t Lc = std::max<uint32_t>(1, std::min<uint32_t>(std::min(max_len, s->max_len), skq::LFAST));
    const uint32_t hcap = pick_hcap(Lc, ix->mink, threshold);
    if (ix->nk == 1) return ix->mode >= 3 && (hcap == 16 || hcap == 32);
    // 2..4 k slots: k_map1 passes (wide or compact tables, hcap 16 or 32)
    return (ix->mode == 3 || ix->mode == 5) && ix->nk <= (uint32_t)skq::NK_FAST && (hcap == 16 || hcap == 32);
}

static int map_fused(skq_session* s, const uint8_t* d_reads, const uint64_t* d_offs, uint32_t fixed_len,
                     uint64_t n_reads, uint32_t max_len, uint32_t threshold, double fraction, int accumulate,
                     void* stream) {
    DeviceGuard g(s->idx->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const skq_index* ix = s->idx;
    // the candidates packed (skq.h), unless the totals would be binned from the padded rows (k_bin);
    // then, for batches of 512k+ reads, the tail on the side stream in the other frame
    const bool slow_totals = accumulate && ix->ntx <= (1u << 22) && ix->nk <= (uint32_t)skq::NK_FAST && s->bin_nb > 0;
    const bool cpack = !accumulate || slow_totals;
    // (4M+ reads: beside a 1-ms map the tail's kernels overlap; beside cfg2's 0.09-ms map of 1M reads
    // they only queue behind its workgroups — 0.15 against 0.11 ms per step — so a small batch runs
    // its tail on the launch stream, between the maps)
    static const uint64_t side_min = [] {  // (SKQ_SIDE_MIN, development: the batch size from which)
        const char* e = dev_env("SKQ_SIDE_MIN");
        return e ? std::strtoull(e, nullptr, 10) : (1ull << 22);
    }();
    bool side = cpack && n_reads >= side_min;
    if (side) {
        if (int rc = ensure_side(s)) return rc;
        if (!s->alt.ctrl && frame_alloc(s, s->alt, s->f.hcap_alloc)) {  // (no room: the tail stays on the launch stream)
            frame_free(s->alt);
            (void)hipGetLastError();
            side = false;
        }
    }
    if (side) {
        // this batch takes the other frame; the previous batch's frame is no longer the results, so
        // its control words are reset on the side stream behind its tail (the host reads control
        // words only synchronously, after sync_side: nothing on the launch stream reads them, so
        // the reset needs no hand-off from it — one cross-queue wait fewer between two maps)
        std::swap(s->f, s->alt);
        s->fid ^= 1;
        const int o = s->fid ^ 1;
        if (!s->tail_side[o]) {  // (the previous batch ran on the launch stream: its kernels first)
            HIP_TRY(hipEventRecord(s->ev_fork, st));
            HIP_TRY(hipStreamWaitEvent(s->side, s->ev_fork, 0));
        }
        HIP_TRY(hipMemsetAsync(s->alt.ctrl, 0, skq::C_WORDS * 4, s->side));
        HIP_TRY(hipEventRecord(s->ev_done[o], s->side));
        s->done_rec[o] = true;
        s->zeroed[o] = true;
        // this frame's last tail (two batches back) and its reset
        // (a tail already done needs no barrier packet on the launch stream)
        if (s->done_rec[s->fid] && hipEventQuery(s->ev_done[s->fid]) != hipSuccess)
            HIP_TRY(hipStreamWaitEvent(st, s->ev_done[s->fid], 0));
        if (!s->zeroed[s->fid]) HIP_TRY(hipMemsetAsync(s->f.ctrl, 0, skq::C_WORDS * 4, st));
    } else {
        if (int rc = wait_side(s, st)) return rc;
        if (s->f.other_zeroed) {  // (the previous small batch's tail zeroed the other half)
            s->f.ctrl = s->f.ctrl == s->f.ctrl_mem ? s->f.ctrl_mem + skq::C_WORDS : s->f.ctrl_mem;
            s->f.other_zeroed = false;
        } else {
            HIP_TRY(hipMemsetAsync(s->f.ctrl, 0, skq::C_WORDS * 4, st));
        }
    }
    s->zeroed[s->fid] = false;
    s->tail_side[s->fid] = side;
    skq::SketchParams sp{};
    skq::ChainParams cp{};
    if (ix->nk > 1 && (!s->f.ktab || !s->f.kcnt)) {  // the per-k tables of the multi-k passes
        dev_free(s->f.ktab);  // (both or neither: a failed pair is retried whole)
        dev_free(s->f.kcnt);
        int rc = dev_alloc(&s->f.ktab, (uint64_t)ix->nk * skq::DCAP * s->max_reads);
        if (!rc) rc = dev_alloc(&s->f.kcnt, 2ull * ix->nk * s->max_reads);  // counts, needs
        if (rc) {
            dev_free(s->f.ktab);
            dev_free(s->f.kcnt);
            return rc;
        }
    }
    if (int rc = sketch_impl(s, d_reads, d_offs, fixed_len, n_reads, max_len, threshold, 0, stream, &sp)) return rc;
    if (ix->nk > 1 && use_stash()) {  // the first pass's image of the bases, for the later passes
        const uint64_t words = ((n_reads + 63) / 64) * (uint64_t)skq::stash_stride(sp.tile_chunks);
        if (words > s->f.stash_words) {
            dev_free(s->f.stash);
            s->f.stash_words = 0;
            if (int rc = dev_alloc(&s->f.stash, words)) return rc;
            s->f.stash_words = words;
        }
        sp.stash = s->f.stash;
        sp.stash_stride = skq::stash_stride(sp.tile_chunks);
    }
    // the hashes (and the multi-k passes' per-k tables) in the per-wave packed layout (whole
    // lines written; skq.h)
    s->hash_packed = true;
    sp.hpack = 1u;
    if (int rc = chain_impl(s, s->n_reads, s->f.status, s->f.hash_cnt, s->f.hashes, nullptr, nullptr, s->hcap, fraction,
                            accumulate, true, stream, &cp))
        return rc;
    // (chained records decode unused slots as the key 0x0FFFFFFF: reads sketched at a
    // threshold that reaches that far use the wide entries alone)
    if (sp.threshold >= skq::CHN_KEY_LIMIT)
        for (uint32_t i = 0; i < SKQ_MAX_K; ++i) {
            cp.chain[i] = nullptr;
            cp.chain_len[i] = 0;
        }
    if ((cp.slow_totals != 0) != slow_totals) return fail(-3, "internal: totals binning mismatch");
    s->cand_packed = cpack;
    cp.cpack = cpack ? 1u : 0u;
    cp.cand_wtot = s->f.cand_wtot;
    hipEvent_t t0{};
    record(s, 0, &t0, st);
    // (a side batch's tail waits for the map through an event bound to its last dispatch — the
    // timing scope's stop event when one is open)
    if (side && !skq::g_launch_ev.stop) skq::g_launch_ev.stop = s->ev_map;
    hipEvent_t map_end = side ? static_cast<hipEvent_t>(skq::g_launch_ev.stop) : nullptr;
    int rc = 0;
    if (ix->nk == 1) {
        rc = skq::launch_map1(sp, cp, stream);
    } else {
        // 2..4 k slots: one k_map1 pass per k slot (each with the raw capacity its k needs), their
        // per-k tables in the frame's ktab / kcnt; the last pass merges, filters and emits
        const uint32_t nk = ix->nk;
        const uint32_t ml = d_offs ? max_len : fixed_len;
        const uint32_t Lc = std::max<uint32_t>(1, std::min<uint32_t>(std::min(ml, s->max_len), skq::LFAST));
        uint32_t cap[SKQ_MAX_K] = {}, capmax = 0;
        for (uint32_t i = 0; i < nk; ++i) {
            cap[i] = std::min(s->hcap, pick_hcap(Lc, ix->ks[i], threshold, pass_sigmas()));
            capmax = std::max(capmax, cap[i]);
        }
        // a launch per k slot, each with its own capacity (or, SKQ_MAPK=1, one k_mapk launch for
        // them all when they share a table kind)
        rc = mapk_dev() ? skq::launch_mapk(sp, cp, capmax, stream) : -5;
        if (rc == -5) {
            rc = 0;
            for (uint32_t i = 0; i < nk && !rc; ++i) {
                skq::SketchParams pi = sp;
                pi.kslot = i;
                rc = skq::launch_map1_pass(pi, cp, cap[i], i + 1 == nk, stream);
            }
        }
    }
    if (rc) {
        skq::g_launch_ev = {};
        return fail(-3, rc == -4 ? "map kernel: unsupported capacity" : "map launch failed");
    }
    record_stop(s, 0, t0, st);
    skq::g_launch_ev = {};
    if (int rc = chain_tail(s, &sp, cp, accumulate, st, side, map_end)) return rc;
    s->have_chain = true;
    // the fused kernels filled no probe offsets (lofs): a later skq_chain on these sketches
    // probes them itself (k_probe, then the count kernel over the packed sets)
    s->probed = false;
    return 0;
}

int skq_map(skq_session* s, const uint8_t* d_reads, const uint64_t* d_offs, uint32_t fixed_len,
            uint64_t n_reads, uint32_t max_len, uint32_t threshold, double fraction, int accumulate,
            void* stream) {
    if (s && n_reads && map_fusable(s, d_offs, fixed_len, max_len, threshold))
        return map_fused(s, d_reads, d_offs, fixed_len, n_reads, max_len, threshold, fraction, accumulate, stream);
    if (int rc = skq_sketch(s, d_reads, d_offs, fixed_len, n_reads, max_len, threshold, stream)) return rc;
    return skq_chain(s, fraction, accumulate, stream);
}

int skq_chain_sketches(skq_session* s, uint64_t n_reads, const uint32_t* d_hashes,
                       const uint64_t* d_hash_offs, const uint32_t* d_hash_cnt, const uint8_t* d_present,
                       double fraction, int accumulate, void* stream) {
    if (!s) return fail(-1, "null session");
    if (n_reads > s->max_reads) return fail(-1, "batch larger than the session's max_reads");
    if (n_reads && (!d_hashes || !d_hash_offs || !d_hash_cnt)) return fail(-1, "null sketch arrays");
    s->n_reads = n_reads;
    s->have_sketch = false;
    s->have_chain = false;
    s->probed = false;
    s->x_hashes = d_hashes;
    s->x_offs = d_hash_offs;
    // every external sketch counts as sketched: the session's status array, set to SKQ_READ_OK,
    // stands in (the count kernels read a status for every read)
    if (int rc = wait_side(s, reinterpret_cast<hipStream_t>(stream))) return rc;  // (the frame may be a tail's)
    if (n_reads)
        HIP_TRY(hipMemsetAsync(s->f.status, SKQ_READ_OK, n_reads, reinterpret_cast<hipStream_t>(stream)));
    return chain_impl(s, n_reads, s->f.status, d_hash_cnt, d_hashes, d_hash_offs, d_present, 0, fraction,
                      accumulate, false, stream);
}

int skq_session_results(skq_session* s, skq_results* o) { return skq::session_results(s, o, true); }

}  // extern "C"

namespace skq {
// (fold = false: the per-read arrays only — the EM's append and the ingest's status copy — so no
// fold kernel is queued per batch)
int session_results(skq_session* s, skq_results* o, bool fold) {
    if (!s || !o) return fail(-1, "null argument");
    {  // the batch's tail and the totals may still run on the side stream (the host waits for it);
       // the packed sums fold on the stream of the last batch's tail, behind it, so tx_reads /
       // tx_score are current once the caller's stream is synchronized (skq.h)
        DeviceGuard g(s->idx->device);
        if (fold && s->acc_reads)
            if (int rc = fold_totals(s, s->last_st)) return rc;
        if (int rc = sync_side(s)) return rc;
    }
    o->n_reads = s->n_reads;
    o->nk = s->idx->nk;
    o->hcap = s->hcap;
    o->ccap = skq::CCAP;
    o->ntx = s->idx->ntx;
    o->status = s->f.status;
    o->hash_cnt = s->f.hash_cnt;
    o->hashes = s->f.hashes;
    o->hash_ext = s->f.hash_ext;
    o->hash_layout = s->hash_packed ? 1u : 0u;
    o->cand_layout = s->cand_packed ? 1u : 0u;
    o->cand_cnt = s->f.cand_cnt;
    o->cand_tid = s->f.cand_tid;
    o->cand_score = s->f.cand_score;
    o->cand_ext = s->f.cand_ext;
    o->tx_reads = s->tx_reads;
    o->tx_score = s->tx_score;
    return 0;
}
}  // namespace skq

extern "C" {

int skq_session_check(skq_session* s, void* stream) {
    if (!s) return fail(-1, "null session");
    DeviceGuard g(s->idx->device);
    uint32_t c[skq::C_WORDS];
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    if (int rc = sync_side(s)) return rc;
    HIP_TRY(hipMemcpy(c, s->f.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    const uint32_t err = c[skq::C_ERR1] | c[skq::C_ERR2];
    if (err) {
        char buf[160];
        std::snprintf(buf, sizeof buf,
                      "device workspace exhausted (error bits 0x%x: 1/2 overflow list, 4 hash_ext, 8 "
                      "chain scratch, 16 cand_ext); split the batch",
                      err);
        return fail(-4, buf);
    }
    return 0;
}

int skq_session_reset_totals(skq_session* s, void* stream) {
    if (!s) return fail(-1, "null session");
    DeviceGuard g(s->idx->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (int rc = wait_side(s, st)) return rc;
    HIP_TRY(hipMemsetAsync(s->tx_reads, 0, s->idx->ntx * 8ull, st));
    HIP_TRY(hipMemsetAsync(s->tx_acc, 0, s->idx->ntx * 8ull, st));
    s->acc_reads = 0;
    HIP_TRY(hipMemsetAsync(s->tx_score, 0, s->idx->ntx * 8ull, st));
    return 0;
}

int skq_session_export(skq_session* s, uint8_t* status, uint64_t* hash_offs, uint32_t* hashes,
                       uint64_t* cand_offs, uint32_t* cand_tid, uint32_t* cand_score, uint64_t* n_hashes,
                       uint64_t* n_cands) {
    if (!s) return fail(-1, "null session");
    if (int rc = skq_session_check(s, nullptr)) return rc;
    DeviceGuard g(s->idx->device);
    const uint64_t n = s->n_reads;
    const uint32_t nk = s->idx->nk;
    std::vector<uint32_t> hc, cc(n);
    std::vector<uint8_t> st(n);
    if (n) {
        if (s->have_chain) HIP_TRY(hipMemcpy(cc.data(), s->f.cand_cnt, cc.size() * 4, hipMemcpyDeviceToHost));
        if (s->have_sketch) {
            hc.resize(n * nk);  // [i][r]
            HIP_TRY(hipMemcpy(hc.data(), s->f.hash_cnt, hc.size() * 4, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(st.data(), s->f.status, n, hipMemcpyDeviceToHost));
        }
    }
    std::vector<uint32_t> cx;  // packed candidates: the read's cand_ext run (pair offset) or ~0u
    if (s->have_chain && s->cand_packed) {
        cx.assign(n, ~0u);
        for (uint64_t r = 0; r < n; ++r)
            if (cc[r] & skq::CAND_EXT) {
                cx[r] = cc[r] & ~skq::CAND_EXT;
                HIP_TRY(hipMemcpy(&cc[r], s->f.cand_ext + 2ull * cx[r], 4, hipMemcpyDeviceToHost));
            }
    }
    // packed layout: per (k slot, read) the hash_ext run ([count, region share, hashes...]) or ~0u,
    // and the read's share of its wave's region
    std::vector<uint32_t> xo, sh;
    if (s->have_sketch && s->hash_packed) {
        xo.assign(hc.size(), ~0u);
        sh = hc;
        for (uint64_t e = 0; e < hc.size(); ++e)
            if (hc[e] & skq::HASH_EXT) {
                xo[e] = (uint32_t)skq::run_at(hc[e]);
                sh[e] = skq::run_share(hc[e]);
                HIP_TRY(hipMemcpy(&hc[e], s->f.hash_ext + xo[e], 4, hipMemcpyDeviceToHost));
            }
    }
    uint64_t th = 0, tc = 0;
    for (uint64_t v : hc) th += v;
    for (uint64_t v : cc) tc += v;
    if (n_hashes) *n_hashes = th;
    if (n_cands) *n_cands = tc;
    if (status)
        for (uint64_t r = 0; r < n; ++r) status[r] = s->have_sketch ? (st[r] & SKQ_STATUS_MASK) : 0;
    if (hash_offs || hashes) {
        if (s->have_sketch) {
            const uint32_t hcap = s->hcap;
            std::vector<uint32_t> pad((uint64_t)nk * hcap * n);  // padded: [i][j][r]; packed: per wave
            if (n) HIP_TRY(hipMemcpy(pad.data(), s->f.hashes, pad.size() * 4, hipMemcpyDeviceToHost));
            uint64_t at = 0;
            if (s->hash_packed) {  // per k slot, sets in lane order per wave; runs in hash_ext
                std::vector<uint64_t> woff(nk, 0);
                for (uint64_t r = 0; r < n; ++r) {
                    if ((r & 63) == 0) std::fill(woff.begin(), woff.end(), 0);
                    for (uint32_t i = 0; i < nk; ++i) {
                        const uint64_t e = (uint64_t)i * n + r;
                        const uint32_t c = hc[e];
                        if (xo[e] != ~0u) {
                            if (hashes && c)
                                HIP_TRY(hipMemcpy(hashes + at, s->f.hash_ext + xo[e] + 2, c * 4ull, hipMemcpyDeviceToHost));
                        } else if (hashes) {
                            std::copy_n(pad.data() + (uint64_t)i * hcap * n + (r & ~63ull) * hcap + woff[i], c,
                                        hashes + at);
                        }
                        woff[i] += sh[e];
                        if (hash_offs) hash_offs[r * nk + i] = at;
                        at += c;
                    }
                }
            } else {
                for (uint64_t r = 0; r < n; ++r)
                    for (uint32_t i = 0; i < nk; ++i) {
                        const uint64_t e = r * nk + i;
                        const uint32_t c = hc[(uint64_t)i * n + r];
                        if (hash_offs) hash_offs[e] = at;
                        if (hashes) {
                            if (c <= hcap) {
                                for (uint32_t j = 0; j < c; ++j) hashes[at + j] = pad[((uint64_t)i * hcap + j) * n + r];
                            } else {
                                HIP_TRY(hipMemcpy(hashes + at, s->f.hash_ext + pad[(uint64_t)i * hcap * n + r], c * 4ull,
                                                  hipMemcpyDeviceToHost));
                            }
                        }
                        at += c;
                    }
            }
            if (hash_offs) hash_offs[n * nk] = at;
        } else if (hash_offs) {
            for (uint64_t e = 0; e <= n * nk; ++e) hash_offs[e] = 0;
        }
    }
    if (cand_offs || cand_tid || cand_score) {
        std::vector<uint32_t> t((uint64_t)skq::CCAP * n), sc((uint64_t)skq::CCAP * n);  // [j][r]
        if (n && s->have_chain) {
            HIP_TRY(hipMemcpy(t.data(), s->f.cand_tid, t.size() * 4, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(sc.data(), s->f.cand_score, sc.size() * 4, hipMemcpyDeviceToHost));
        }
        uint64_t at = 0, woff = 0;
        std::vector<uint32_t> ext;
        for (uint64_t r = 0; r < n; ++r) {
            if (cand_offs) cand_offs[r] = at;
            const uint32_t c = cc[r];
            if (s->cand_packed) {  // per wave in lane order (tid | score << 22), or a run
                if ((r & 63) == 0) woff = 0;
                if (cx[r] != ~0u) {
                    ext.resize(2ull * c);
                    if (c)
                        HIP_TRY(hipMemcpy(ext.data(), s->f.cand_ext + 2ull * (cx[r] + 1), ext.size() * 4,
                                          hipMemcpyDeviceToHost));
                    for (uint32_t j = 0; j < c; ++j) {
                        if (cand_tid) cand_tid[at + j] = ext[2 * j];
                        if (cand_score) cand_score[at + j] = ext[2 * j + 1];
                    }
                } else {
                    for (uint32_t j = 0; j < c; ++j) {
                        const uint32_t e = t[(r & ~63ull) * skq::CCAP + woff + j];
                        if (cand_tid) cand_tid[at + j] = e & 0x3FFFFFu;
                        if (cand_score) cand_score[at + j] = e >> 22;
                    }
                    woff += c;
                }
            } else if (c <= (uint32_t)skq::CCAP) {
                for (uint32_t j = 0; j < c; ++j) {
                    if (cand_tid) cand_tid[at + j] = t[(uint64_t)j * n + r];
                    if (cand_score) cand_score[at + j] = sc[(uint64_t)j * n + r];
                }
            } else {
                ext.resize(2ull * c);
                HIP_TRY(hipMemcpy(ext.data(), s->f.cand_ext + 2ull * t[r], ext.size() * 4, hipMemcpyDeviceToHost));
                for (uint32_t j = 0; j < c; ++j) {
                    if (cand_tid) cand_tid[at + j] = ext[2 * j];
                    if (cand_score) cand_score[at + j] = ext[2 * j + 1];
                }
            }
            at += c;
        }
        if (cand_offs) cand_offs[n] = at;
    }
    return 0;
}

int skq_session_totals(skq_session* s, uint64_t* tx_reads, uint64_t* tx_score, int to_device, void* stream) {
    if (!s) return fail(-1, "null session");
    DeviceGuard g(s->idx->device);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t bytes = s->idx->ntx * 8ull;
    const hipMemcpyKind kind = to_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (int rc = wait_side(s, st)) return rc;
    if (int rc = fold_totals(s, st)) return rc;
    if (tx_reads) HIP_TRY(hipMemcpyAsync(tx_reads, s->tx_reads, bytes, kind, st));
    if (tx_score) HIP_TRY(hipMemcpyAsync(tx_score, s->tx_score, bytes, kind, st));
    if (!to_device) HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int skq_session_totals_async(skq_session* s, uint64_t* d_reads, uint64_t* d_score, void* stream) {
    if (!s || !d_reads || !d_score) return fail(-1, "null argument");
    DeviceGuard g(s->idx->device);
    hipStream_t cs = reinterpret_cast<hipStream_t>(stream);
    // the stream of the last batch's tail: every earlier tail is ordered before it (a side batch's
    // tail waits for the launch stream's earlier ones, a launch-stream batch for the side stream's)
    hipStream_t ts = s->tail_side[s->fid] && s->side ? s->side : s->last_st;
    if (!s->ev_snap[0]) {
        HIP_TRY(hipEventCreateWithFlags(&s->ev_snap[0], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&s->ev_snap[1], hipEventDisableTiming));
    }
    if (ts != cs) {
        HIP_TRY(hipEventRecord(s->ev_snap[0], cs));
        HIP_TRY(hipStreamWaitEvent(ts, s->ev_snap[0], 0));
    }
    if (s->acc_reads) {
        if (skq::launch_fold_totals(s->tx_acc, s->tx_reads, s->tx_score, s->idx->ntx, ts)) return fail(-3, "fold failed");
        s->acc_reads = 0;
    }
    const size_t bytes = s->idx->ntx * 8ull;
    HIP_TRY(hipMemcpyAsync(d_reads, s->tx_reads, bytes, hipMemcpyDeviceToDevice, ts));
    HIP_TRY(hipMemcpyAsync(d_score, s->tx_score, bytes, hipMemcpyDeviceToDevice, ts));
    if (ts != cs) {
        HIP_TRY(hipEventRecord(s->ev_snap[1], ts));
        HIP_TRY(hipStreamWaitEvent(cs, s->ev_snap[1], 0));
    }
    if (s->side && ts == s->side) {  // (the frame's done event now follows the copy too: a later reset or
        // results call waits for it)
        HIP_TRY(hipEventRecord(s->ev_done[s->fid], s->side));
        s->done_rec[s->fid] = true;
    }
    return 0;
}

int skq_malloc(int device, size_t bytes, void** out) {
    DeviceGuard g(device);
    HIP_TRY(hipMalloc(out, bytes ? bytes : 1));
    return 0;
}

int skq_free(void* p) {
    if (p) HIP_TRY(hipFree(p));
    return 0;
}

int skq_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, reinterpret_cast<hipStream_t>(stream)));
    return 0;
}

int skq_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, reinterpret_cast<hipStream_t>(stream)));
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return 0;
}

int skq_stream_sync(void* stream) {
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return 0;
}

// Development hook (tools/kbench.py --stamps): a device buffer of 8 u64 per wave of k_map1 that
// receives the wave's phase clocks (s_memtime); null turns it off.
int skq_session_set_stamps(skq_session* s, void* d_stamps) {
    if (!s) return fail(-1, "null session");
    s->stamps = static_cast<uint64_t*>(d_stamps);
    return 0;
}

int skq_session_enable_timing(skq_session* s, int enable) {
    if (!s) return fail(-1, "null session");
    s->timing = enable != 0;
    return 0;
}

int skq_session_kernel_time(skq_session* s, int kind, double* total_ms, uint64_t* launches) {
    if (!s) return fail(-1, "null session");
    DeviceGuard g(s->idx->device);
    double tot = 0;
    uint64_t cnt = 0;
    std::vector<TimedLaunch> keep;
    for (auto& t : s->timed) {
        if (t.kind != kind) {
            keep.push_back(t);
            continue;
        }
        HIP_TRY(hipEventSynchronize(t.stop));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, t.start, t.stop));
        tot += ms;
        ++cnt;
        (void)hipEventDestroy(t.start);
        (void)hipEventDestroy(t.stop);
    }
    s->timed.swap(keep);
    if (total_ms) *total_ms = tot;
    if (launches) *launches = cnt;
    return 0;
}

}  // extern "C"
