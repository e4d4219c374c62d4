// Drop-in for the reference's include/kmer.h:21. Runs on the GPU through skq_sketch_seqs.
#ifndef KMER_H
#define KMER_H

#include <cstdint>
#include <string>
#include <unordered_set>

// Every (uint32_t) ntHash forward hash of `sequence` at length k (windows holding a byte
// outside ACGTUacgtu skipped). Throws std::runtime_error("Sequence length is shorter than
// k-mer length") when sequence.size() < k, as src/kmer.cpp does.
std::unordered_set<uint32_t> extract_and_hash_kmers_nthash(const std::string& sequence, int k);

#endif  // KMER_H
