/*
 * oracle.h — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline. The product (libskq.so, the skq CLI) never links it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - the rolling hash is pinned by ntHash's own constant tables, read as data from the
 *     reference's prebuilt binary (tests/golden/nthash_tables.json) and by the known-answer
 *     vectors of SURVEY.md §8c;
 *   - the chain (sparse_chain), EM, assignment and is_valid_sequence are pinned against the
 *     reference's OWN code: /root/reference/src/{sparse_chaining,data_io,isoform_assignment}.cpp
 *     compile unmodified here (oracle/ref.mk -> oracle/_ref/libref.so, harness
 *     oracle/ref_harness.cpp) and tests/test_ref_pinned.py compares them with this file;
 *   - the record rules are pinned by the edge-case fixture of SURVEY.md §8c (tests/golden/edge/).
 *   Only the reference's kmer.cpp / sketch.cpp / main.cpp are unbuildable here: they need the
 *   absent third-party ntHash library, and no stand-in for it is written.
 *
 * Third-party algorithm restated: bcgsc ntHash >= 2.3 (not vendored in the reference, version
 * not pinned by its build; identified from symbols in build/test):
 *   fwd(s_0..s_{k-1}) = XOR_i srol^{k-1-i}(SEED[s_i]) on 64 bits, with the split rotate
 *   srol(x) = ((x << 1) & ~(1<<33)) | (bit63 -> bit33) | (bit32 -> bit0); windows containing a
 *   base whose seed is 0 (N and anything outside ACGTUacgtu) are skipped.
 */
#ifndef SKQ_ORACLE_H
#define SKQ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ntHash 64-bit seed of byte c (0 = invalid). */
uint64_t orc_seed(unsigned char c);
/* one split-rotate step of ntHash (srol). */
uint64_t orc_srol(uint64_t x);

/* ntHash NtHash(seq, 1, k) + roll()/get_forward_hash() loop: writes the 64-bit forward hash and
 * the window start of every window free of invalid bases, in order. Returns the count, or
 * (size_t)-1 for the argument errors ntHash rejects (k == 0 or len < k). */
size_t orc_nthash_fwd(const char* seq, size_t len, unsigned k, uint64_t* out_hash, size_t* out_pos);

/* (uint32_t)(UINT32_MAX * fraction) — src/sketch.cpp:25-26 */
uint32_t orc_threshold(double fraction);

/* is_valid_sequence — src/data_io.cpp:17-34: only uppercase A, C, G, T. Empty is valid. */
int orc_is_valid_sequence(const char* seq, size_t len);

/* createSketch_FracMinhash_direct — src/sketch.cpp:24-39. Writes the retained hash SET in
 * ascending order (the reference's unordered_set has no order). out needs len-k+1 slots.
 * Returns the count or (size_t)-1 on len < k. */
size_t orc_sketch(const char* seq, size_t len, unsigned k, uint32_t threshold, uint32_t* out);

/* extract_and_hash_kmers_nthash — src/kmer.cpp:19-35 (no threshold). Same output contract. */
size_t orc_all_hashes(const char* seq, size_t len, unsigned k, uint32_t* out);

/* ---- inverted index: build_kmer_to_transcript_map (src/sketch.cpp:51-74) ----------------- */
typedef struct orc_index orc_index;

/* Builds the oracle index from transcript sequences (concatenated bytes + offsets, tids are
 * positions 0..ntx-1). Restates build_and_save_index (src/main.cpp:66-85): a transcript
 * shorter than ANY k is skipped entirely; every other transcript is sketched at every k. */
orc_index* orc_index_build(unsigned nk, const unsigned* ks, uint32_t ntx, const char* seqs,
                           const uint64_t* offs, uint32_t threshold);
/* Builds from explicit postings: per k, npairs (hash, tid) pairs (any order, duplicates of a
 * (hash, tid) pair are removed since sketches are sets). */
orc_index* orc_index_from_pairs(unsigned nk, const unsigned* ks, uint32_t ntx,
                                const uint64_t* npairs, const uint32_t* const* hashes,
                                const uint32_t* const* tids);
void orc_index_free(orc_index*);
/* number of distinct keys / postings at k index i */
uint64_t orc_index_nkeys(const orc_index*, unsigned i);
uint64_t orc_index_npost(const orc_index*, unsigned i);
/* CSR export at k index i: keys ascending (nkeys), offs (nkeys+1), tids ascending per key. */
void orc_index_export(const orc_index*, unsigned i, uint32_t* keys, uint64_t* offs, uint32_t* tids);

/* ---- sparse_chain (src/sparse_chaining.cpp:29-115) for ONE read -------------------------- */
/* hashes[i]/nh[i]: the read's sketch at k index i (a set; any order). present[i] = 0 means the
 * read has no sketch for that k (skipped, :55-58). Output candidates sorted by score desc, then
 * tid asc (the reference sort is unstable, :108-109: only this normalised order is comparable).
 * Returns the number of candidates, or (size_t)-1 if cap is too small. */
size_t orc_chain_read(const orc_index* idx, const uint32_t* const* hashes, const uint32_t* nh,
                      const int* present, double fraction, uint32_t* out_tid,
                      uint32_t* out_score, size_t cap);

/* orc_chain_read over a batch of sketches (CSR: read r, k slot i at hash_offs[r*nk+i]); candidates
 * as CSR (cand_offs[n+1]). Returns 0, -1 when cap is too small. */
int orc_chain_batch(const orc_index* idx, uint64_t n, const uint64_t* hash_offs, const uint32_t* hashes,
                    double fraction, uint64_t* cand_offs, uint32_t* cand_tid, uint32_t* cand_score,
                    uint64_t cap);

/* ---- whole hot path over a batch of read sequences -------------------------------------- */
enum { ORC_OK = 0, ORC_INVALID = 1, ORC_SHORT = 2 };
/* Per read r (bytes reads[offs[r] .. offs[r+1])): status (process_fastq_single_pass filters,
 * src/main.cpp:132-138), per k sketch (hash_cnt[r*nk+i], hashes at (r*nk+i)*hcap), candidates
 * (cand_cnt[r], tid/score at r*ccap). Returns 0, or -1 if a cap is exceeded. */
int orc_map_batch(const orc_index* idx, const uint8_t* reads, const uint64_t* offs, uint64_t n,
                  uint32_t threshold, double fraction, uint8_t* status, uint32_t* hash_cnt,
                  uint32_t* hashes, uint32_t hcap, uint32_t* cand_cnt, uint32_t* cand_tid,
                  uint32_t* cand_score, uint32_t ccap);

/* The same without outputs (CPU-baseline timing): returns the total candidate count. */
uint64_t orc_map_batch_count(const orc_index* idx, const uint8_t* reads, const uint64_t* offs,
                             uint64_t n, uint32_t threshold, double fraction);

/* The quant hot path from FASTQ bytes (src/main.cpp:107-151, :181-185), for bench.py's CPU
 * baseline: the reference's record machine over fq[0..len) (sequential, as the reference),
 * then per record is_valid_sequence + length filter + every k's sketch + sparse_chain on
 * nthreads threads over contiguous record ranges, then the id map (the last valid record of an
 * id is kept, :147). At most max_records records. Optional outputs (NULL = skipped), record
 * order, layouts as orc_map_batch: status, hash_cnt/hashes (hcap per (record, k)),
 * cand_cnt/cand_tid/cand_score (ccap per record); kept[n] (1 = the record kept for its id);
 * tx_reads/tx_score[ntx]: candidate reads and summed scores per transcript over the kept
 * records. Returns 0; -1 if a cap is exceeded; -2 if totals were asked for without per-record
 * lists and the file has duplicate ids. */
int orc_fastq_map(const orc_index* idx, const char* fq, uint64_t len, uint32_t threshold, double fraction,
                  int nthreads, uint64_t max_records, uint64_t* n_records, uint8_t* status, uint32_t* hash_cnt,
                  uint32_t* hashes, uint32_t hcap, uint32_t* cand_cnt, uint32_t* cand_tid, uint32_t* cand_score,
                  uint32_t ccap, uint8_t* kept, uint64_t* tx_reads, uint64_t* tx_score);

/* Per-read digests of a batch of fixed-length reads (bases[r*L .. (r+1)*L)), for per-read parity
 * at full batch sizes where keeping every record's outputs would not fit: for read r,
 *   digest[r] = item(0xA5, 0, status) + SUM_{k slot i, j < hash_cnt} item(i + 1, j, hash_j)
 *             + SUM_{j < cand_cnt} (item(0xC0, j, tid_j) + item(0xD0, j, score_j))   (mod 2^64),
 *   item(tag, j, v) = splitmix64-finaliser((tag << 56) ^ (j << 32) ^ v),
 * hashes ascending per k slot, candidates by score desc then tid asc (orc_map_batch's outputs).
 * So two results agree iff (with overwhelming probability) every read's status, retained-hash sets
 * and candidate list agree, read by read. tx_reads / tx_score (optional): the per-transcript totals.
 * nthreads over contiguous read ranges. Returns 0, -1 on a failure. (tests/digest.py restates the
 * digest over an skq export.) */
int orc_map_digest(const orc_index* idx, const uint8_t* bases, uint32_t L, uint64_t n, uint32_t threshold,
                   double fraction, int nthreads, uint64_t* digest, uint64_t* tx_reads, uint64_t* tx_score);

/* EM over the reads' candidate lists (src/isoform_assignment.cpp:9-65): pi starts uniform over
 * the ntx transcripts; E-step per read in order, posterior = pi*score * (1/denominator) when the
 * denominator exceeds 1e-10; M-step pi = (posterior_sum + 0.01f/R) + 0.01f (float pseudocount,
 * R = reads including those without candidates); stop after max_iterations or when the summed
 * absolute change drops below convergence. Returns the iterations run. */
int orc_em(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
           const uint32_t* cand_score, uint32_t ntx, int max_iterations, double convergence,
           double* pi);
/* assign_reads_to_isoforms (src/isoform_assignment.cpp:67-97) */
void orc_assign(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
                const uint32_t* cand_score, uint32_t ntx, const double* pi, double* counts,
                uint8_t* assigned);

#ifdef __cplusplus
}
#endif
#endif
