// Drop-in for the reference's include/sparse_chaining.h:35-42. The vote runs on the GPU
// (skq_index_create + skq_chain_sketches); results per read are sorted by score descending and,
// where scores tie, by transcript id ascending (the reference's std::sort leaves ties unordered).
#ifndef SPARSE_CHAINING_H
#define SPARSE_CHAINING_H

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "data_io.h"
#include "sketch.h"

std::unordered_map<std::string, std::vector<std::pair<std::string, int>>> sparse_chain(
    const std::unordered_map<std::string, MultiKmerSketch>& read_sketches,
    const std::unordered_map<unsigned,
                             std::unordered_map<uint32_t, std::vector<std::pair<std::string, const std::unordered_set<uint32_t>*>>>>&
        kmer_to_transcripts,
    const std::unordered_map<std::string, Transcript>& transcripts,
    const std::vector<unsigned>& kmer_lengths,
    double fraction);

#endif  // SPARSE_CHAINING_H
