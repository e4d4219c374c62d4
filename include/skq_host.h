/*
 * skq_host.h — C ABI of the host-side pieces around the hot path: the inverted-index builder,
 * FASTA/FASTQ readers that keep the reference's record rules, the reference's legacy binary
 * index format, and the EM / assignment / CSV stage downstream of sparse_chain.
 *
 * What each entry point replaces in the reference (Codfishz/Sketch-for-RNA-seq @ 2025-04-18):
 *   skq_tables_build     build_and_save_index's sketch loop + build_kmer_to_transcript_map
 *                        (src/main.cpp:66-85, src/sketch.cpp:51-74), multi-threaded, dense ids
 *   skq_fasta_load       load_fasta (src/data_io.cpp:47-80)
 *   skq_fastq_load       process_fastq_single_pass's record reader (src/main.cpp:113-148)
 *   skq_legacy_index_*   save_index / load_index (src/data_io.cpp:165-304)
 *   skq_em / skq_assign  estimate_isoform_abundance_em / assign_reads_to_isoforms
 *                        (src/isoform_assignment.cpp:9-97)
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

/* Single-sequence sketch on the host (the drop-in createSketch_FracMinhash_direct for one
 * transcript-sized sequence): sorted unique retained hashes. out needs len-k+1 slots.
 * Returns the count, or -1 if k == 0 or len < k. */
int64_t skq_host_sketch(const uint8_t* seq, uint64_t len, uint32_t k, uint32_t threshold,
                        uint32_t* out);

#ifdef __cplusplus
}
#endif
#endif
