/*
 * skq_host.h — C ABI of the host-side pieces around the hot path: the inverted-index builder,
 * FASTA/FASTQ readers that keep the reference's record rules, the reference's legacy binary
 * index format, and the EM / assignment / CSV stage downstream of sparse_chain.
 *
 * What each entry point replaces in the reference (Codfishz/Sketch-for-RNA-seq @ 2025-04-18):
 *   skq_tables_build     build_and_save_index's sketch loop + build_kmer_to_transcript_map
 *                        (src/main.cpp:66-85, src/sketch.cpp:51-74), multi-threaded, dense ids
 *   skq_fasta_load       load_fasta (src/data_io.cpp:47-80)
 *   skq_fastq_*          process_fastq_single_pass's record reader (src/main.cpp:113-148)
 *   skq_legacy_index_*   save_index / load_index (src/data_io.cpp:165-304)
 *   skq_em / skq_assign  estimate_isoform_abundance_em / assign_reads_to_isoforms
 *                        (src/isoform_assignment.cpp:9-97)
 *   skq_csv_write        output_to_csv (src/data_io.cpp:133-152)
 */
#ifndef SKQ_HOST_H
#define SKQ_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "skq.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- inverted index (host CSR, one table per distinct k) ---------------------------------- */
typedef struct skq_tables skq_tables;

/* Sketch every transcript (sequences seqs[offs[t] .. offs[t+1]), dense ids t) at every k of
 * ks[0..nk) and invert. A transcript shorter than ANY k is left out entirely
 * (src/main.cpp:66-75). Bases are hashed as ntHash does: lowercase like uppercase, U like T,
 * windows holding any other byte skipped. nthreads <= 0: hardware concurrency. */
int skq_tables_build(uint32_t ntx, const uint8_t* seqs, const uint64_t* offs, uint32_t nk,
                     const uint32_t* ks, uint32_t threshold, int nthreads, skq_tables** out);
/* The same tables built on the GPU (host arrays in; transcripts sketched by one workgroup each,
 * one radix sort per k): identical output to skq_tables_build. */
int skq_tables_build_gpu(int device, uint32_t ntx, const uint8_t* seqs, const uint64_t* offs,
                         uint32_t nk, const uint32_t* ks, uint32_t threshold, skq_tables** out);
/* from (hash, tid) pairs per distinct k (duplicates removed) */
int skq_tables_from_pairs(uint32_t ntables, const uint32_t* ks, const uint64_t* npairs,
                          const uint32_t* const* hashes, const uint32_t* const* tids,
                          skq_tables** out);
uint32_t skq_tables_count(const skq_tables* t);
/* view of table i (pointers valid while t lives) */
int skq_tables_get(const skq_tables* t, uint32_t i, skq_kmer_table* out);
int skq_tables_free(skq_tables* t);

/* convenience: upload built tables; ks = the k list in CLI order */
int skq_index_from_tables(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks,
                          const skq_tables* t, skq_index** out);
/* the same with the chained tables (skq_index_create_chained) from the transcripts' sequences in
 * tx (the tables' transcripts, dense ids in tx order), sketched at threshold; tx without
 * sequences (null, or names only): as skq_index_from_tables */
struct skq_seqs;
int skq_index_from_tables_chained(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks,
                                  const skq_tables* t, const struct skq_seqs* tx, uint32_t threshold,
                                  skq_index** out);

/* Single-sequence sketch on the host, used on the index side (transcripts): sorted unique
 * retained hashes, ntHash semantics. out needs len-k+1 slots. Returns the count, or -1 if
 * k == 0 or len < k. (The quant path and the C++ drop-in sketch on the GPU: skq_sketch,
 * skq_sketch_seqs.) */
int64_t skq_host_sketch(const uint8_t* seq, uint64_t len, uint32_t k, uint32_t threshold,
                        uint32_t* out);

/* ---- sequences: FASTA (load_fasta, src/data_io.cpp:47-80) ------------------------------- */
typedef struct skq_seqs skq_seqs;
/* Transcripts in file order. The id is the header up to the first space; the first record of an
 * id wins; every record but the last is kept only if it is uppercase A/C/G/T (the last one is
 * kept unvalidated, as the reference does); blank lines are skipped. */
int skq_fasta_load(const char* path, skq_seqs** out);
uint64_t skq_seqs_count(const skq_seqs* s);
/* flat views: sequence i = seq_bytes[seq_offs[i] .. seq_offs[i+1]), name i likewise */
int skq_seqs_view(const skq_seqs* s, const uint8_t** seq_bytes, const uint64_t** seq_offs,
                  const char** name_bytes, const uint64_t** name_offs);
int skq_seqs_free(skq_seqs* s);

/* ---- reads: FASTQ (process_fastq_single_pass's reader, src/main.cpp:113-148) -------------- */
typedef struct skq_fastq skq_fastq;
int skq_fastq_open(const char* path, skq_fastq** out);
/* Next batch of up to max_reads records in file order (every record: the sketch kernel's status
 * applies the reference's filter). bytes/offs stay valid until the next call; records are
 * numbered from *first_ordinal. *n == 0 at the end of the file. */
int skq_fastq_next(skq_fastq* q, uint64_t max_reads, uint64_t* n, const uint8_t** bytes,
                   const uint64_t** offs, uint64_t* first_ordinal);
/* Report the status of records first .. first+n-1; then skq_fastq_kept(ordinal) is 1 for the
 * record kept for its id: the last one with status SKQ_READ_OK (src/main.cpp:147). */
int skq_fastq_mark(skq_fastq* q, uint64_t first, uint64_t n, const uint8_t* status);
int skq_fastq_kept(const skq_fastq* q, uint64_t ordinal);
uint64_t skq_fastq_records(const skq_fastq* q);
int skq_fastq_id(const skq_fastq* q, uint64_t ordinal, const char** id, uint64_t* len);
int skq_fastq_close(skq_fastq* q);
/* Split a FASTQ file into `parts` byte ranges for several devices (skq_ingest_open_range):
 * offs[0] = 0, offs[parts] = file size, the rest at line starts near equal shares; states[p] is
 * the reader's record-machine state (0 between records, 1-3 inside one, src/main.cpp:119-129)
 * at offs[p], exact: worked out from the lines before the split point, going back until every
 * possible earlier state has converged (a few lines in any FASTQ; the whole prefix at worst). */
int skq_fastq_split(const char* path, uint32_t parts, uint64_t* offs, uint32_t* states);

/* ---- the legacy binary index (save_index / load_index, src/data_io.cpp:165-304) ------------ */
typedef struct skq_legacy_index skq_legacy_index;
/* k list (CLI order), every transcript (id, sequence, length field 0), then per distinct k the
 * key -> transcript-id lists; native endian, size_t = u64, unsigned = u32. */
int skq_legacy_index_write(const char* path, uint32_t nk, const uint32_t* ks, const skq_seqs* tx,
                           const skq_tables* tables);
/* Dense transcript ids follow the file's transcript order. */
int skq_legacy_index_read(const char* path, skq_legacy_index** out);
int skq_legacy_index_view(const skq_legacy_index* ix, uint32_t* nk, const uint32_t** ks,
                          const skq_seqs** tx, const skq_tables** tables);
int skq_legacy_index_free(skq_legacy_index* ix);
/* Compact sidecar `<legacy_path>.skq` (CSR tables + names, no sequences), stamped with the legacy
 * file's size and mtime; written by the CLI's index mode after the legacy file. */
int skq_sidecar_write(const char* legacy_path, uint32_t nk, const uint32_t* ks, const skq_seqs* tx,
                      const skq_tables* tables);
/* quant's loader: the sidecar when present and its stamp matches, else skq_legacy_index_read.
 * From the sidecar the transcripts carry names only (empty sequences). *from_sidecar (may be
 * NULL) tells which. */
int skq_index_open(const char* path, skq_legacy_index** out, int* from_sidecar);

/* ---- EM, assignment, CSV (src/isoform_assignment.cpp:9-97, src/data_io.cpp:133-152) ------- */
/* Reads' candidates in CSR form (cand_offs[nreads+1]); every read counts in R, including reads
 * without candidates. pi[ntx] out (not normalised, as in the reference); *iterations out. */
int skq_em(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
           const uint32_t* cand_score, uint32_t ntx, int max_iterations, double convergence,
           int nthreads, double* pi, int* iterations);
/* The EM round split for read-sharded drivers (skq/dist.py; the GPU forms are skq_em_estep /
 * skq_em_mstep in skq.h): post[ntx] = posterior sums of these reads under pi; then, with post
 * summed over all shards, pi = (post + (double)(0.01f / R)) + (double)0.01f, *change = sum |d pi|.
 * (skq_em_estep_host runs on the calling thread; nthreads is reserved.) */
int skq_em_estep_host(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
                      const uint32_t* cand_score, uint32_t ntx, const double* pi, int nthreads,
                      double* post);
int skq_em_mstep_host(uint32_t ntx, double* pi, const double* post, uint64_t total_reads,
                      double* change);
/* counts[ntx]: expected reads per transcript; assigned[ntx] = 1 where a read contributed. */
int skq_assign(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
               const uint32_t* cand_score, uint32_t ntx, const double* pi, double* counts,
               uint8_t* assigned);
/* "Name,NumReads,EM_Abundance", one row per assigned transcript, values printed like %g. */
int skq_csv_write(const char* path, const skq_seqs* tx, const double* counts,
                  const uint8_t* assigned, const double* pi);

#ifdef __cplusplus
}
#endif
#endif
