// skq_internal.h — structures shared by the HIP kernels (skq_kernels.hip) and the C-ABI host
// side (skq_capi.hip). Not part of the public ABI.
#pragma once
#include <cstdint>
#include <vector>

#include "skq.h"

struct skq_tables;

namespace skq {

// kernel timing without marker packets: while a scope's events are set (skq_capi.hip record()),
// the timed launchers (launch_timed, skq_kernels.hip) bind them to the dispatches themselves —
// hipExtLaunchKernel: the start event to the first launch's start, the stop event to the last
// launch's end — so nothing is queued between a batch's kernels (a hipEventRecord pair around the
// map was ~6 us of each step, profiles/r6_tail_traces.log)
struct LaunchEvents {
    void* start = nullptr;
    void* stop = nullptr;
};
extern thread_local LaunchEvents g_launch_ev;

// skq_session_results with or without folding the packed per-transcript sums (skq_capi.hip)
int session_results(skq_session* s, skq_results* o, bool fold);

constexpr int WG = 256;            // threads per workgroup for both kernels (4 waves)
constexpr int LFAST = 256;         // reads longer than this take the slow path
constexpr int DCAP = 16;           // distinct transcripts per read on the fast chain path
constexpr int CCAP = DCAP;         // candidate slots per read (fast path can't exceed DCAP)
constexpr int HFAST = 255;         // hashes per (read, k) the fast chain path accepts (8-bit counts)
constexpr int NK_FAST = 4;         // k slots the fast chain path packs (8-bit counts)
constexpr uint32_t HASH_MUL = 0x9E3779B1u;
constexpr uint64_t MAX_BATCH = (1ull << 24) - 1;  // packed per-batch totals hold 24-bit counts

// status flags above SKQ_STATUS_MASK (internal)
constexpr uint8_t ST_SLOW1 = 0x10;  // sketch handled by the slow path
constexpr uint32_t HASH_EXT = 0x80000000u;  // packed hash layout: hash_cnt marks a hash_ext run
// A run's mark carries the read's share of its wave's region itself, so a reader summing the
// shares never needs a run header another workgroup may still be writing: HASH_EXT | share << 24
// | run offset / 8 (runs start 8-word aligned; hash_ext below RUN_MAX words).
constexpr uint64_t RUN_MAX = (1ull << 24) * 8;
constexpr uint32_t run_mark(uint64_t at, uint32_t share) {
    return HASH_EXT | (share << 24) | (uint32_t)(at >> 3);
}
constexpr uint64_t run_at(uint32_t c) { return (uint64_t)(c & 0xFFFFFFu) << 3; }
constexpr uint32_t run_share(uint32_t c) { return (c >> 24) & 0x7Fu; }
constexpr uint32_t run_words(uint32_t need) { return (need + 7u) & ~7u; }
// k_slow_wave's workgroups (a fixed grid) and the stretch of hash_ext / cand_ext each owns past the
// capacity the bump allocators see (SketchParams::hash_ext_cap, ChainParams::cand_ext_cap), so
// its runs take no shared atomic until a workgroup's stretch is used up
constexpr uint32_t SW_GRID = 4096;
constexpr uint32_t SW_HCH = 2048;  // hash_ext words per workgroup
constexpr uint32_t SW_CCH = 128;   // cand_ext pairs per workgroup
constexpr uint32_t CAND_EXT = 0x80000000u;  // packed candidate layout: cand_cnt marks a cand_ext run

// control block (u32 words): the sketch half (words 0-7) is zeroed before every sketch, the
// chain half (words 8-15) before every chain.
enum Ctrl : int {
    C_OVF1 = 0,     // sketch overflow list length
    C_ERR1 = 1,     // sketch error bits
    C_BUMP_H = 2,   // u64 (words 2-3): hash_ext words used
    C_OVF3 = 4,     // second-level sketch list (k_slow_wave -> k_sketch_slow)
    C_OVF2 = 8,     // chain overflow list length
    C_ERR2 = 9,     // chain error bits
    C_BUMP_S = 10,  // u64 (words 10-11): chain scratch u64 words used
    C_BUMP_C = 12,  // u64 (words 12-13): cand_ext pairs used
    C_OVF4 = 14,    // second-level chain list (k_slow_wave -> k_chain_slow)
    C_WORDS = 16
};
enum Err : uint32_t {
    E_OVF1_FULL = 1, E_OVF2_FULL = 2, E_HASH_EXT = 4, E_SCRATCH = 8, E_CAND_EXT = 16
};

// Device index. Postings lists are de-duplicated into equivalence classes: every distinct
// transcript set is stored once in the `lists` array as [n, tid_0 .. tid_{n-1}] (16-B aligned),
// and each k has a table of 64-byte buckets (16 u32 words) mapping keys to list offsets:
//   word 0       header: bits 0-2 m = records in the bucket (0..7); bit 3 = "continue": some key
//                homed at or before this bucket lives further on
//   words 1..7   keys of records 0..m-1
//   words 8..14  list offsets of records 0..m-1
// A key's home bucket is (uint64)(key * HASH_MUL) * nbuckets >> 32; records are placed at the
// first bucket from home with room (host build, in home order), so a probe reads one 64-B line
// unless the home bucket is marked "continue"; the max displacement is kept per table.
// A read usually hits 1-3 distinct lists, so k_chain counts per list, then expands.
constexpr uint32_t BUCKET_WORDS = 16;
constexpr uint32_t BUCKET_MAX_RECORDS = 7;
constexpr uint32_t BUCKET_LIST0 = 8;  // word of record 0's list offset

struct DevTable {
    uint64_t bucket_base;  // first bucket of this k's table in the bucket array
    uint32_t nbuckets;
    uint32_t max_probe;    // buckets a probe may have to read (displacement + 1)
    uint32_t present;      // 0: the index has no table for this k (skipped, src/sparse_chaining.cpp:51-53)
    uint32_t pad;
};

struct SketchParams {
    const uint8_t* reads;
    const uint64_t* offs;  // null => fixed_len
    uint64_t fixed_len;
    uint64_t n;
    uint32_t nk;
    uint32_t maxk;
    uint32_t ks[SKQ_MAX_K];
    uint32_t threshold;
    uint32_t tile_chunks;  // 16-byte chunks staged per wave (64 reads)
    uint32_t hcap;
    uint32_t ovf_cap;
    const uint64_t* rolltab;  // [nk][16] 33-bit seed(in) ^ rot^k(seed(out)) by (in*4 + out), then 4 seeds
    uint8_t* status;
    uint32_t* hash_cnt;
    uint32_t* hashes;
    uint32_t* hash_ext;
    uint64_t hash_ext_cap;
    uint32_t* ctrl;
    uint32_t* ovf1;
    uint32_t ovf_word;  // the control word counting ovf1 (k_sketch_slow: C_OVF1, or C_OVF3 behind k_slow_wave)
    uint32_t kslot;     // k_map1 pass mode: the k slot this pass sketches and counts
    // k_map1's per-wave LDS region (bytes) and the offset of its per-read overflow flags in it,
    // set by the launcher (map1_layout)
    uint32_t map_wave_bytes, map_flag_at;
    // hpack: the per-wave packed hash layout (fused maps; skq.h "hash layouts"): read r's set
    // at k slot i follows those of the reads before it in its wave, from hashes + i * hcap * n +
    // (r & ~63) * hcap, except runs in hash_ext, marked hash_cnt = HASH_EXT | offset ([count,
    // region share, hashes...]); the multi-k passes' per-k tables (ktab) likewise, TS per read
    uint32_t hpack;
    // multi-k passes: the first pass stores each wave's staged bases (2-bit codes, then the
    // per-chunk bad bits as u64 from word (tile_chunks + 1) & ~1) at stash + wave * stash_stride,
    // and the later passes stage from there instead of re-reading the bases (null: every pass
    // reads the bases)
    uint32_t* stash;
    uint32_t stash_stride;  // words per wave, a multiple of 16 (whole 64-B lines)
    // fused index probe (direct tables, DESIGN.md "Index"): when fuse is set, each retained hash
    // h of k slot i is looked up as dir[i][h] (h < dir_len[i], else a miss) and the list offset
    // lands in lofs[(i*hcap + j)*n + r]; pflag[r] = 1 marks reads the count kernel must hand to
    // the slow chain path. Slots without a table (dir[i] null) are skipped by the chain.
    // (3 = wide direct tables: the sketch does not probe; k_count3 gathers the entries)
    int fuse;                        // 1 = dir tables, 2 = rank tables, 3 = wide tables
    const uint32_t* dir[SKQ_MAX_K];
    uint64_t dir_len[SKQ_MAX_K];     // dir: entries; rank: blocks
    const uint32_t* rank[SKQ_MAX_K]; // rank table, 16-B blocks {bitmap of 32 keys, overflow base, v0, v1}
    const uint32_t* rovf[SKQ_MAX_K]; // list offsets of the 3rd+ key of a block
    uint32_t* lofs;
    uint8_t* pflag;
    // ntHash mode (createSketch_FracMinhash_direct on arbitrary sequences, transcripts): no read
    // is rejected; windows holding a byte outside ACGTUacgtu are skipped (src/sketch.cpp:31-36
    // through ntHash); a k longer than the sequence yields an empty set for that k.
    int nthash;
};

struct ChainParams {
    uint64_t n;
    uint32_t nk;
    uint32_t hcap;
    double fraction;
    int accumulate;
    uint32_t ovf_cap;
    const uint8_t* status;     // null => every read sketched (chain_sketches)
    const uint32_t* hash_cnt;
    const uint32_t* hashes;    // padded (session) or flat (explicit offsets)
    const uint32_t* hash_ext;
    const uint64_t* hash_offs; // null => padded layout
    uint32_t hpack;            // 1: per-wave packed layout (SketchParams::hpack)
    // cpack: candidates in the per-wave packed layout (fused maps; skq.h "candidate layouts"):
    // read r's, as tid | score << 22, follow those of the reads before it in its wave, from
    // cand_tid + (r & ~63) * CCAP, except runs in cand_ext, marked cand_cnt[r] = CAND_EXT | pair
    // offset (pair [count, 0], then the (tid, score) pairs)
    uint32_t cpack;
    const uint8_t* present;    // null => all k present
    const uint32_t* buckets;
    const uint32_t* lists;    // [n, tid...] per distinct postings list
    DevTable tabs[SKQ_MAX_K];
    uint32_t* cand_cnt;
    uint32_t* cand_tid;
    uint32_t* cand_wtot;  // (fused map, packed) per wave of 64 reads: its packed candidate words (k_bin_packed)
    uint32_t* cand_score;
    uint32_t* cand_ext;
    uint64_t cand_ext_cap;     // pairs
    uint64_t* scratch;
    uint64_t scratch_cap;      // u64 words
    uint64_t* tx_acc;          // per batch: (reads << 40) | score (k_bin_sum), folded by k_fold_totals
    uint64_t* tx_reads;
    uint64_t* tx_score;
    uint32_t* ctrl;
    uint32_t* ovf2;
    uint32_t ovf_word;         // the control word counting ovf2 (k_chain_slow: C_OVF2, or C_OVF4)
    uint32_t* lofs;            // k_probe or fused k_sketch -> k_count: list offset per probe,
                               // [(i*lcap + j)*n + r], ~0u = miss
    uint8_t* pflag;            // -> k_count: 1 = read goes to the slow chain path
    uint32_t lcap;             // probes per (read, k) slot in lofs (reads above it: slow path)
    uint32_t ntx;              // transcripts in the index
    // per-transcript totals by buckets of 2^bin_bits ids (k_count3 or k_bin, then k_bin_sum);
    // slow_totals: k_chain_slow adds its reads' totals itself (the count kernel binned)
    uint32_t bin_bits, bin_nb;
    uint32_t* bin_hdr;
    uint32_t* bin_region;
    int slow_totals;
    uint64_t* stamps;          // development: per-wave phase clocks (k_map1), null = off
    uint32_t ablate;           // development (SKQ_ABLATE, results WRONG when set): k_map1 phases
                               // skipped to price them: 2 entry-list gathers, 4 filter/order/candidate
                               // writes, 8 hash writes, 16 base loads (codes left as they are),
                               // 32 windows after the first
    // multi-k map by passes (k_map1 pass mode; the final pass merges): per k slot i and read r, the
    // entries of the read's count table at that k that meet that k's need (tid << 8 | count):
    // kcnt[i * n + r] of them at ktab[(i * TS + j) * n + r], and the need itself (min(ceil(fraction
    // * max), 255); 0: the k slot does not filter) at kcnt[(nk + i) * n + r]
    uint32_t* ktab;
    uint8_t* kcnt;
    // wide direct tables (DESIGN.md "Index"): entry h of k slot i is 8 words at wdir[i] + 8h,
    // [n, t0..t6] for lists of n <= 7 transcripts, [0x80000000 | list offset, t0..t6] for longer
    // ones (the rest at lists[offset + 8..]), n = 0 for no key; h >= wdir_len[i] is a miss.
    // wide = 1: lofs holds the sketch's hashes themselves (k_count3 only)
    // Compact tables (wide = 3): the same 8-word entries, one per key, placed by a minimal
    // perfect hash (cmp_slot below) in wdir_len[i] slots; wpil[i] holds one 16-bit pilot per
    // bucket of keys (wnb[i] buckets, hash seed wseed[i]). Entry: [key, t0 | F << 22, t1 .. t6],
    // F = n (1..7), 8 for a longer list (t0..t6 inline, the list at lists[offset]: offset bits
    // 0-31 in bits 22-31 of words 4, 5, 6 and 22-23 of word 7), 0 for an empty slot.
    const uint16_t* wpil[SKQ_MAX_K];
    uint32_t wnb[SKQ_MAX_K];
    uint32_t wseed[SKQ_MAX_K];
    int wide;
    const uint32_t* wdir[SKQ_MAX_K];
    uint64_t wdir_len[SKQ_MAX_K];
    // chained tables (k_map1 TAB = 3 over wide entries, 4 over compact ones): a
    // 128-B entry per possible key up to chain_len (TAB 4: per present key, at the key's compact
    // slot) of 8 uint4 each (layout CHN_* below): the key's own record, then records of
    // keys that follow it along the transcripts (nearest first), each naming the key's WHOLE
    // postings list as a set of the entry's transcripts, so one 128-B request settles a run of a
    // read's retained hashes
    const uint32_t* chain[SKQ_MAX_K];  // per k slot (null: none for that slot)
    uint64_t chain_len[SKQ_MAX_K];
};

// records the message returned by skq_last_error(); returns code (skq_capi.hip)
int set_error(int code, const char* msg);
// session facts for skq_ingest (skq_capi.hip)
int session_device(const skq_session* s);
uint64_t session_max_reads(const skq_session* s);

// host: one sequence's retained hashes at k in position order (repeats kept; ntHash's window
// rules: windows holding a byte outside ACGTUacgtu skipped) (skq_tables.cpp)
void sketch_positions(const uint8_t* s, uint64_t len, uint32_t k, uint32_t thr, std::vector<uint32_t>& out);
// Chained entries (ChainParams::chain), CHAIN_WORDS words each:
//   words 0-3         per entry id q (0..7): the records whose list holds it, a 16-bit set in half
//                     q & 1 of word q >> 1 (a record's count is its key's; an id's is the records')
//   words 4-11        the entry's transcript ids (up to CHN_TIDS, each once)
//   words 12-27       records: key ^ CHN_KEY_LIMIT, the entry's own key first (unused: 0, which
//                     decodes to the key 0x0FFFFFFF no retained hash reaches: keys < CHN_KEY_LIMIT).
//                     Word 12 CHN_LONG: the key's own list holds more than CHN_TIDS transcripts (the
//                     entry holds nothing: lookups go to the wide entries); word 12 zero: no such key
//   word 28           the entry's own key ^ CHN_KEY_LIMIT (entries at compact slots: a slot asked for
//                     a key it does not hold answers "no such key"); words 29-31 unused
constexpr uint32_t CHAIN_WORDS = 32;  // chained entry: 128 B
constexpr uint32_t CHN_KEYS = 16, CHN_TIDS = 8;
constexpr uint32_t CHN_W_SET = 0, CHN_W_TID = 4, CHN_W_KEY = 12, CHN_W_SELF = 28;
constexpr uint32_t CHN_LONG = 0x80000000u;  // (decodes to 0x8FFFFFFF: neither a hash nor the sort's padding)
constexpr uint32_t CHN_KEY_LIMIT = 0x0FFFFFFFu;
// host: ascending sort with threads (skq_tables.cpp)
void parallel_sort_u64(std::vector<uint64_t>& v, int threads);
// host: tables from (key << 32 | tid) words per distinct k (consumed; duplicates removed)
int tables_from_words(uint32_t ntables, const uint32_t* ks, std::vector<uint64_t>* words, skq_tables** out);
// host: tables taking over ready CSR arrays per distinct k (moved from)
int tables_from_csr(uint32_t ntables, const uint32_t* ks, std::vector<uint32_t>* keys, std::vector<uint64_t>* offs,
                    std::vector<uint32_t>* tids, skq_tables** out);

// launchers (skq_kernels.hip)
int launch_sketch(const SketchParams& p, void* stream);
// (grid: workgroups walking the list; the list length is on the device)
int launch_sketch_slow(const SketchParams& p, void* stream, unsigned grid = 2048);
// fused sketch + chain (k_map1: quant mode, one k slot, wide tables, hcap 16 or 32; -4 otherwise)
int launch_map1(const SketchParams& p, const ChainParams& cp, void* stream);
// fused sketch + chain for 2..4 k slots (wide or compact tables) by passes: k_map1 in pass mode
// for each k slot (p.kslot; a raw capacity `cap` of 16 or 32 hashes, at most the hashes' layout
// stride p.hcap); the last (final_pass) merges the per-k tables, filters, orders and bins
int launch_map1_pass(const SketchParams& p, const ChainParams& cp, uint32_t cap, bool final_pass, void* stream);
// the same passes in one launch (k_mapk: every workgroup runs the k slots in turn; one capacity for
// all of them, and every k slot chained or none: -5 otherwise)
int launch_mapk(const SketchParams& p, const ChainParams& cp, uint32_t cap, void* stream);
int launch_probe(const ChainParams& p, void* stream);  // k_probe
int launch_count(const ChainParams& p, void* stream);  // k_count<nk>
int launch_chain_slow(const ChainParams& p, void* stream, unsigned grid = 2048);
// k_sketch_slow then k_chain_slow per read in one launch, over the chain list p.ovf2 (the fused
// map's tail behind k_slow_wave: the reads still flagged ST_SLOW1 are re-sketched first)
// (zero_next: control words zeroed on the way, for the next batch; null: none)
int launch_general_slow(const SketchParams& sp, const ChainParams& p, void* stream, unsigned grid = 256,
                        uint32_t* zero_next = nullptr);
// the wave slow path behind k_map1 and its passes (wide or compact tables, <= 4 k slots; -4 otherwise):
// the listed reads it cannot take go on to ovf3 (C_OVF3) and ovf4 (C_OVF4)
int launch_slow_wave(const SketchParams& p, const ChainParams& cp, uint32_t* ovf3, uint32_t* ovf4, void* stream);
int launch_fold_totals(uint64_t* acc, uint64_t* reads, uint64_t* score, uint32_t ntx, void* stream);
// per-transcript totals of the batch's final candidates into p.tx_acc (k_bin + k_bin_sum), then
// launch_fold_totals adds them into p.tx_reads / p.tx_score with atomics (commuting with the slow
// paths' direct adds)
// (binned = 1: the count kernel already wrote the bins; only k_bin_sum runs). Returns 0, < 0 on a
// failure. The sums land in p.tx_acc, packed (reads << 40 | score): k_fold_totals unpacks them
// (beside_map: on the side stream, beside the next batch's map: kernels sized to start in the LDS a
// retiring map workgroup frees)
int launch_bin(const ChainParams& p, int binned, void* stream, bool beside_map);
// whether launch_count's kernel bins the totals itself (k_count3 with p.bin_nb > 0)
bool count_bins(const ChainParams& p);
int launch_dir_scatter(uint32_t* dir, const uint32_t* keys, const uint32_t* vals, uint64_t n, void* stream);
// fills wide entries wdir[keys[j]] from the postings lists at lists[vals[j]]
int launch_wdir_scatter(uint32_t* wdir, const uint32_t* keys, const uint32_t* vals, const uint32_t* lists,
                        uint64_t n, void* stream);

#ifdef __HIPCC__
#define SKQ_HD __host__ __device__
#else
#define SKQ_HD
#endif
SKQ_HD inline uint32_t home_bucket(uint32_t key, uint32_t nbuckets) {
    return (uint32_t)(((uint64_t)(uint32_t)(key * HASH_MUL) * nbuckets) >> 32);
}

// Compact tables: key -> bucket (a 16-bit pilot each) -> slot. mix is murmur3's 32-bit finaliser
// (a bijection); scale maps a 32-bit hash onto [0, n) by its high bits.
SKQ_HD inline uint32_t cmp_mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
SKQ_HD inline uint32_t cmp_scale(uint32_t h, uint64_t n) { return (uint32_t)(((uint64_t)h * n) >> 32); }
SKQ_HD inline uint32_t cmp_key_hash(uint32_t key, uint32_t seed) { return cmp_mix(key ^ seed); }
SKQ_HD inline uint32_t cmp_slot(uint32_t kh, uint32_t pilot, uint64_t nslots) {
    return cmp_scale(cmp_mix(kh ^ (pilot * 0x9E3779B1u)), nslots);
}
constexpr uint32_t CMP_LONG = 8;  // F of an entry whose list continues at lists[offset]
size_t sketch_lds_bytes(uint32_t nk, uint32_t tile_chunks, uint32_t hcap, bool nthash);
// SketchParams::stash: words per wave (codes, then 2 words of bad bits per 64 chunks), whole lines
SKQ_HD inline uint32_t stash_stride(uint32_t tile_chunks) {
    return (((tile_chunks + 1) & ~1u) + 2 * ((tile_chunks + 63) / 64) + 15) & ~15u;
}

// 33-bit ntHash lane (bits 0..32 of ntHash's split rotate evolve on their own)
constexpr uint64_t M33 = (1ull << 33) - 1;
inline uint64_t rot33(uint64_t x, unsigned d) {
    d %= 33;
    return d ? (((x << d) | (x >> (33 - d))) & M33) : x;
}
// seed33 by 2-bit code: ((ascii >> 1) & 3): A=0, C=1, T=2, G=3
constexpr uint64_t SEED33[4] = {0x195c60474ull, 0x162a02b4cull, 0x14be24456ull, 0x082572324ull};

}  // namespace skq
