/*
 * skq.h — C ABI of the MI355X-native FracMinHash sketch + sparse-chain hot path.
 *
 * Plain C: pointers, sizes, int status codes (0 = ok, < 0 = error, message via
 * skq_last_error()); no exceptions and no C++/HIP/torch types cross this boundary. Streams are
 * passed as `void*` (a hipStream_t, or NULL for the null stream).
 *
 * What each entry point replaces in the reference (Codfishz/Sketch-for-RNA-seq @ 2025-04-18):
 *   skq_index_create        build_kmer_to_transcript_map's result, made device-resident
 *                           (include/sketch.h:59, src/sketch.cpp:51-74; consumed at
 *                           src/sparse_chaining.cpp:51-62)
 *   skq_sketch              createSketch_FracMinhash_direct over a batch of reads, plus the
 *                           read filters of process_fastq_single_pass
 *                           (include/sketch.h:47, src/sketch.cpp:24-39; src/main.cpp:132-144)
 *   skq_chain               sparse_chain (include/sparse_chaining.h:35-42,
 *                           src/sparse_chaining.cpp:29-115)
 *   skq_map                 skq_sketch + skq_chain (the quant hot path, src/main.cpp:181-185)
 *   skq_chain_sketches      sparse_chain on caller-provided read sketches (drop-in wrapper path)
 * The C++ drop-in signatures (kmer.h, sketch.h, sparse_chaining.h) are thin wrappers over these
 * (sketch-for-rna-seq_amd/csrc/dropin.cpp); INTEGRATION.md shows the bindings.
 *
 * Threading: one skq_session per host thread / stream; an skq_index may be shared by sessions
 * on its device. All device pointers must live on the index's device.
 */
#ifndef SKQ_H
#define SKQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SKQ_MAX_K 8 /* distinct k-mer lengths per index (the reference allows any list) */

/* per-read status (low 2 bits; higher bits are internal flags) */
#define SKQ_READ_OK 0      /* sketched and chained                                        */
#define SKQ_READ_INVALID 1 /* a byte outside uppercase ACGT: dropped (src/main.cpp:132)  */
#define SKQ_READ_SHORT 2   /* shorter than the largest k: dropped (src/main.cpp:136-138) */
#define SKQ_STATUS_MASK 3

typedef struct skq_index skq_index;
typedef struct skq_session skq_session;

const char* skq_last_error(void);
int skq_version(void);
int skq_device_count(void);

/* One k: an inverted index in CSR form, host memory. keys ascending and unique; tids of key j
 * are tids[offs[j] .. offs[j+1]), ascending and unique (a transcript appears at most once per
 * (k, hash): sketches are sets). */
typedef struct {
    uint32_t k;
    uint64_t nkeys;
    const uint32_t* keys;
    const uint64_t* offs; /* nkeys + 1 */
    const uint32_t* tids;
} skq_kmer_table;

/* Upload an index to `device`. `ks[0..nk)` is the k list in CLI order (duplicates allowed, as in
 * the reference); tables[] holds one entry per DISTINCT k (any order). */
int skq_index_create(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks,
                     uint32_t ntables, const skq_kmer_table* tables, skq_index** out);
int skq_index_free(skq_index* idx);
/* device bytes held, total postings, longest postings list */
int skq_index_stats(const skq_index* idx, uint64_t* device_bytes, uint64_t* npostings,
                    uint32_t* max_list);
/* Probe structure of an index (DESIGN.md "Index"); results are identical in every mode:
 *   3 = wide direct tables: a 32-B entry per possible key holding the key's postings list (up to
 *       7 transcripts inline); the sketch does not probe, the count kernel gathers one entry per
 *       retained hash. 32 B x (largest key + 1) per k; only for indexes of <= 2^22 transcripts.
 *   1 = direct tables: a 4-B list offset per possible key, gathered by the sketch kernel.
 *   2 = rank tables (SKQ_PROBE=rank): 16-B blocks of 32 keys, gathered by the sketch kernel.
 *   0 = the bucket table only (k_probe).
 * The first that fits SKQ_DIRECT_MB (environment, MiB, default 49152; 0 disables all but the
 * bucket table) and half the free device memory is built; SKQ_PROBE = wide | dir | rank forces
 * one kind. */
int skq_index_direct(const skq_index* ix);
/* skq_index_create plus, for an index of one k whose transcripts are given (seqs[seq_offs[t] ..
 * seq_offs[t+1]), the sequences the tables were built from, sketched at `threshold`), chained
 * tables: per possible key a 128-B entry holding its postings list and those of the keys that
 * follow it along the transcripts (nearest first, whole lists). skq_map then settles a read's
 * retained hashes with one entry request plus one per hash the entry does not hold (2.6 instead
 * of 6 at cfg3); results are identical (a record is used only for its exact key).
 * Built only with SKQ_CHAIN=1 in the environment (27.5 GB at cfg3; 11 % slower than the wide
 * tables after round 3's write-request changes);
 * otherwise, and for other indexes: as skq_index_create. */
int skq_index_create_chained(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks, uint32_t ntables,
                             const skq_kmer_table* tables, const uint8_t* seqs, const uint64_t* seq_offs,
                             uint32_t nseq, uint32_t threshold, skq_index** out);
/* 0: no chained tables; else 1 + the mean successor records per entry */
double skq_index_chained(const skq_index* ix);
/* the chained tables' host build: seconds this index spent building entries (0 when it took them
 * from another device's build of the same tables), and the host peak of one k slot's build (bytes) */
int skq_index_chain_build(const skq_index* ix, double* host_seconds, uint64_t* host_peak_bytes);

/* A session owns the device workspace for batches of up to max_reads reads of at most
 * max_len bases each (longer reads are still handled exactly, by the slow path). Indexes of
 * 2-4 k add, on the first skq_map, the passes' per-k tables (nk * 64 + 2 * nk B per read) and
 * the first pass's image of the bases (about a quarter of the bases' bytes). */
int skq_session_create(skq_index* idx, uint64_t max_reads, uint32_t max_len, skq_session** out);
/* (max_reads < 2^24: per-batch transcript totals are packed into 24-bit read counts) */
int skq_session_free(skq_session* s);

/* Reads: ASCII bytes on the device; read r is d_reads[d_offs[r] .. d_offs[r+1]). With
 * d_offs == NULL every read is `fixed_len` bytes (read r at r * fixed_len). max_len bounds the
 * read length of this batch (reads above it, or above 256, take the slow path).
 * threshold = (uint32_t)(UINT32_MAX * fraction) — skq_threshold(). */
int skq_sketch(skq_session* s, const uint8_t* d_reads, const uint64_t* d_offs, uint32_t fixed_len,
               uint64_t n_reads, uint32_t max_len, uint32_t threshold, void* stream);
/* createSketch_FracMinhash_direct semantics (include/sketch.h:47, src/sketch.cpp:24-39) on
 * arbitrary sequences, e.g. transcripts or the C++ drop-in: no sequence is rejected (every
 * status is SKQ_READ_OK), windows holding a byte outside ACGTUacgtu are skipped as ntHash skips
 * them, lowercase hashes like uppercase and U like T, and a k longer than the sequence gives an
 * empty set for that k. Same layout and session results as skq_sketch. */
int skq_sketch_seqs(skq_session* s, const uint8_t* d_seqs, const uint64_t* d_offs, uint32_t fixed_len,
                    uint64_t n_seqs, uint32_t max_len, uint32_t threshold, void* stream);
/* One sequence per call, for per-sequence callers: the reference calls
 * createSketch_FracMinhash_direct once per transcript per k (src/main.cpp:79) and once per read
 * per k (src/main.cpp:143-144), and the C++ drop-in (include/dropin/sketch.h, kmer.h) serves those
 * calls here. skq_sketch_seqs semantics for one sequence; the bytes go through pinned host memory
 * the device maps to a resident single-workgroup server (launched by the first call, gone after
 * 2 ms without one, relaunched by the next), no launch or stream synchronisation per call: the
 * caller spins on a mapped completion word. hashes receives up to cap of
 * the retained windows' hashes (unordered; a hash retained at two windows appears twice: the
 * caller's set removes repeats), *count how many there are. Handles are not thread-safe; one per
 * host thread. max_len only sizes the first buffers (longer sequences grow them). */
typedef struct skq_sketcher skq_sketcher;
int skq_sketcher_create(int device, uint64_t max_len, skq_sketcher** out);
int skq_sketcher_run(skq_sketcher* h, const char* seq, uint64_t len, uint32_t k, uint32_t threshold,
                     uint32_t* hashes, uint64_t cap, uint64_t* count);
int skq_sketcher_free(skq_sketcher* h);

/* Chain the session's current sketches; `fraction` as sparse_chain's (0.9 in quant).
 * accumulate != 0 adds each read's candidates into the per-transcript totals. */
int skq_chain(skq_session* s, double fraction, int accumulate, void* stream);
int skq_map(skq_session* s, const uint8_t* d_reads, const uint64_t* d_offs, uint32_t fixed_len,
            uint64_t n_reads, uint32_t max_len, uint32_t threshold, double fraction,
            int accumulate, void* stream);

/* Chain caller-provided sketches (device arrays): read r's sketch at k slot i is
 * d_hashes[d_hash_offs[r*nk+i] .. +d_hash_cnt[r*nk+i]). present[r*nk+i] == 0 marks a k the
 * read has no sketch for (skipped, src/sparse_chaining.cpp:55-58); NULL = all present. */
int skq_chain_sketches(skq_session* s, uint64_t n_reads, const uint32_t* d_hashes,
                       const uint64_t* d_hash_offs, const uint32_t* d_hash_cnt,
                       const uint8_t* d_present, double fraction, int accumulate, void* stream);

uint32_t skq_threshold(double fraction);

/* Device-resident results of the last call (valid until the next call on the session), in
 * structure-of-arrays layout (n = n_reads of the call, so a wave's accesses are contiguous):
 * hashes, hash_layout 0 (padded rows; skq_sketch): read r, k slot i: c = hash_cnt[i*n + r]; if
 *   c <= hcap the sorted set is hashes[(i*hcap + j)*n + r] for j < c; otherwise it is
 *   hash_ext[hashes[i*hcap*n + r] + j].
 * hashes, hash_layout 1 (per-wave packed; skq_map's fused kernels, which then write whole 64-B
 *   lines): c = hash_cnt[i*n + r]; if c & 0x80000000 the set is a run in hash_ext at
 *   x = (c & 0xFFFFFF) * 8: hash_ext[x] hashes at hash_ext[x + 2 ..], and (c >> 24) & 0x7F is the
 *   read's share of its wave's region (the count the pass that sketched it first packed there);
 *   otherwise its c hashes are at hashes[i*hcap*n + (r & ~63)*hcap + o .. + c), o = the summed
 *   shares (counts, or the marks' shares) of reads (r & ~63) .. r - 1 at k slot i.
 *   skq_session_export gives either layout as flat arrays.
 * candidates (sorted by score desc, tid asc), cand_layout 0 (padded rows): c = cand_cnt[r]; if
 *   c <= ccap candidate j is (cand_tid[j*n + r], cand_score[j*n + r]); otherwise the (tid, score)
 *   pairs are at cand_ext[2*(cand_tid[r] + j)], cand_ext[2*(cand_tid[r] + j) + 1].
 * candidates, cand_layout 1 (per-wave packed; skq_map's fused kernels): c = cand_cnt[r]; if
 *   c & 0x80000000 they are a run of pairs at x = c & 0x7FFFFFFF: cand_ext[2x] of them, pair j at
 *   cand_ext[2(x + 1 + j)], cand_ext[2(x + 1 + j) + 1]; otherwise candidate j is the word
 *   cand_tid[(r & ~63)*ccap + o + j] = tid | score << 22, o = the summed counts of reads
 *   (r & ~63) .. r - 1 that are not runs (cand_score unused).
 * After skq_chain_sketches, hash_cnt/hashes are not the session's (the caller's inputs). */
typedef struct {
    uint64_t n_reads;
    uint32_t nk;
    uint32_t hcap;
    uint32_t ccap;
    uint32_t ntx;
    const uint8_t* status;
    const uint32_t* hash_cnt;
    const uint32_t* hashes;
    const uint32_t* hash_ext;
    const uint32_t* cand_cnt;
    const uint32_t* cand_tid;
    const uint32_t* cand_score;
    const uint32_t* cand_ext;
    const uint64_t* tx_reads; /* per transcript: reads listing it as a candidate (accumulated) */
    const uint64_t* tx_score; /* per transcript: sum of those reads' scores (accumulated)      */
    uint32_t hash_layout;     /* 0: padded rows, 1: per-wave packed (above)                     */
    uint32_t cand_layout;     /* 0: padded rows, 1: per-wave packed (above)                     */
    /* (fused maps of 4M+ reads run their whole tail — slow paths and totals — on the session's
     * own side stream, which the launch stream does not wait for: skq_session_results blocks the
     * host until that work is done, and folds the batch's packed per-transcript sums into
     * tx_reads / tx_score on the stream the last batch's tail ran on, so they are current once
     * the caller's stream is synchronized; skq_session_totals waits for it all on the caller's
     * stream instead) */
} skq_results;
int skq_session_results(skq_session* s, skq_results* out);

/* Waits for the session's work on `stream` and reports device-side capacity errors
 * (slow-path workspace exhausted). 0 = ok. */
int skq_session_check(skq_session* s, void* stream);

/* Zero the per-transcript totals. */
int skq_session_reset_totals(skq_session* s, void* stream);

/* Copy results to host memory in packed CSR form (reads in batch order):
 * hash_offs[n*nk+1] / hashes[total]; cand_offs[n+1] / cand_tid / cand_score.
 * Pass NULL arrays to query sizes first (*n_hashes, *n_cands are always written). */
int skq_session_export(skq_session* s, uint8_t* status, uint64_t* hash_offs, uint32_t* hashes,
                       uint64_t* cand_offs, uint32_t* cand_tid, uint32_t* cand_score,
                       uint64_t* n_hashes, uint64_t* n_cands);
/* Copy the per-transcript totals (ntx each) to host or device memory. */
int skq_session_totals(skq_session* s, uint64_t* tx_reads, uint64_t* tx_score, int to_device,
                       void* stream);
/* The same snapshot into device memory without holding `stream` behind the batch's tail: after
 * `stream`'s work so far (the previous snapshot's consumer, e.g. an all-reduce), the totals are
 * folded and copied on the stream the last batch's tail runs on, in order with the tails, and
 * `stream` waits for the copy. The launch stream's next map does not wait for any of it (bench.py
 * --gpus N: the per-step all-reduce of the totals overlaps the next map). */
int skq_session_totals_async(skq_session* s, uint64_t* d_reads, uint64_t* d_score, void* stream);

/* ---- FASTQ ingest on the GPU (process_fastq_single_pass's reader, src/main.cpp:113-148) ------
 * The FASTQ text itself goes to the device: a reader thread pulls the file into pinned staging
 * buffers (io_threads parallel preads, <= 0 = 16, at most 64) and copies chunks of about chunk_bytes (0 = 64 MiB) to HBM
 * on its own stream, up to three chunks ahead; the GPU splits them into records with the reader's rules
 * (a line starting with '@' opens a record whose id is the rest of that line; the next three
 * lines are sequence, '+' and quality, whatever they hold; other lines between records are
 * skipped) and the batch goes through skq_map. Records are numbered in file order from 0. */
typedef struct skq_ingest skq_ingest;
int skq_ingest_open(skq_session* s, const char* path, uint64_t chunk_bytes, int io_threads, skq_ingest** out);
/* The records whose header line starts in [lo, hi) of the file (line starts, e.g. from
 * skq_fastq_split), the reader's state at lo given: one part of a file mapped on several devices.
 * Records are numbered from 0 within the part. */
int skq_ingest_open_range(skq_session* s, const char* path, uint64_t lo, uint64_t hi, uint32_t entry_state,
                          uint64_t chunk_bytes, int io_threads, skq_ingest** out);
/* The next batch (at most the session's max_reads records): parse if needed, sketch + chain on
 * `stream`. Results are the session's, as after skq_map; *n = records in the batch (0 at the end
 * of the file), numbered from *first. Every record is in the batch: status marks the reads the
 * reference drops (invalid / shorter than the largest k). */
int skq_ingest_map(skq_ingest* g, uint32_t threshold, double fraction, int accumulate, void* stream,
                   uint64_t* n, uint64_t* first);
uint64_t skq_ingest_records(const skq_ingest* g);
/* After the last batch: kept[r] = 1 for the record that the reference keeps for its id, the last
 * one with status SKQ_READ_OK (src/main.cpp:147); kept holds skq_ingest_records() bytes. */
int skq_ingest_finish(skq_ingest* g, uint8_t* kept);
/* The parts of one file, in file order, each finished with its own kept array: clears
 * kept[p][r] where a later part keeps a record of the same id, so that across the parts only the
 * last valid record of every id stays (src/main.cpp:147). */
int skq_ingest_supersede(skq_ingest* const* parts, uint32_t nparts, uint8_t* const* kept);
/* id of a record (the header line after '@'), pointing into the mapped file */
int skq_ingest_id(const skq_ingest* g, uint64_t ordinal, const char** id, uint64_t* len);
int skq_ingest_close(skq_ingest* g);

/* ---- EM and assignment on the GPU (estimate_isoform_abundance_em / assign_reads_to_isoforms,
 * src/isoform_assignment.cpp:9-97) ----------------------------------------------------------
 * An skq_em_set holds one device's share of the reads' candidate lists. Reads are appended in order
 * (from a session's device results, or from host CSR arrays); skq_em_select optionally keeps only
 * some of them (the reads the reference's EM sees). Every kept read counts in R, with or without
 * candidates (homologous_segments.size(), :55).
 * One device: skq_em_run + skq_em_assign_host. Several devices (one process each, read-sharded):
 * every rank runs skq_em_estep on its share, the caller sums post[ntx] over ranks (all-reduce),
 * and every rank runs skq_em_mstep with the global R; the rounds are then identical on all ranks.
 * Posterior sums are formed in a fixed order (bitwise reproducible run to run); the reference's
 * own order is unordered_map iteration order, so parity is to a relative tolerance. */
typedef struct skq_em_set skq_em_set;
int skq_em_create(int device, uint32_t ntx, skq_em_set** out);
int skq_em_free(skq_em_set* em);
/* append nreads reads: read r's candidates are cand_tid/cand_score[cand_offs[r] .. cand_offs[r+1]) */
int skq_em_add(skq_em_set* em, uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
               const uint32_t* cand_score);
/* append every read of the session's last batch, in batch order (device to device; synchronous) */
int skq_em_add_session(skq_em_set* em, skq_session* s, void* stream);
/* reads appended so far */
uint64_t skq_em_size(const skq_em_set* em);
/* keep[r] != 0 selects appended read r (skq_em_size() bytes, host); once, after the last add */
int skq_em_select(skq_em_set* em, const uint8_t* keep);
/* R: the selected reads (all appended reads without skq_em_select) */
uint64_t skq_em_reads(const skq_em_set* em);
/* device arrays of ntx doubles: pi = 1/ntx (:17-20) */
int skq_em_init(skq_em_set* em, double* d_pi, void* stream);
/* post[t] = sum over this share's reads with den = sum(pi * score) > 1e-10 of pi[t] * score / den */
int skq_em_estep(skq_em_set* em, const double* d_pi, double* d_post, void* stream);
/* pi[t] = (post[t] + (double)(0.01f / (float)total_reads)) + (double)0.01f; *change (host, may be
 * NULL) = sum of |new - old| — synchronous when change is requested */
int skq_em_mstep(skq_em_set* em, double* d_pi, const double* d_post, uint64_t total_reads, double* change,
                 void* stream);
/* one device: the whole loop (stops after the round whose change < convergence); pi (host, ntx) */
int skq_em_run(skq_em_set* em, int max_iterations, double convergence, double* pi, int* iterations);
/* assign_reads_to_isoforms: counts[t] = sum of pi[t] * score / total over this share's reads with
 * total > 0; assigned[t] = 1 where such a read lists t (device arrays) */
int skq_em_assign(skq_em_set* em, const double* d_pi, double* d_counts, uint8_t* d_assigned, void* stream);
/* the same with host arrays; pi NULL = the pi skq_em_run left on the device */
int skq_em_assign_host(skq_em_set* em, const double* pi, double* counts, uint8_t* assigned);

/* Device memory helpers (for hosts without their own allocator). */
int skq_malloc(int device, size_t bytes, void** out);
int skq_free(void* p);
int skq_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int skq_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int skq_stream_sync(void* stream);

/* Kernel timing: with timing enabled, every skq_sketch / skq_chain call records HIP events on
 * its stream around its fast kernel. skq_session_kernel_time waits for them and returns the
 * summed milliseconds and launch count of one kind since the last query (then forgets them).
 * kind: 0 = k_sketch, 1 = k_probe, 2 = k_count, 3 = per-transcript totals (k_bin + k_bin_sum +
 * k_fold_totals). Used by bench.py for the roofline figure. */
int skq_session_enable_timing(skq_session* s, int enable);
/* Development: device buffer of 8 uint64 per wave of the fused map kernel that receives the
 * wave's phase clocks (s_memtime); NULL turns it off. Not needed by users. */
int skq_session_set_stamps(skq_session* s, void* d_stamps);
int skq_session_kernel_time(skq_session* s, int kind, double* total_ms, uint64_t* launches);
/* Reads of the last batch that took the slow sketch / slow chain path (synchronous). */
int skq_session_slow_reads(skq_session* s, uint32_t* sketch_slow, uint32_t* chain_slow);
/* The same, and (fused map) the reads the wave slow path handed on to the general slow paths:
 * counts[0..3] = sketch slow, chain slow, then second-level sketch, chain (synchronous). */
int skq_session_slow_counts(skq_session* s, uint32_t* counts);

#ifdef __cplusplus
}
#endif
#endif
