// Drop-in for the reference's include/sketch.h (types :15-33, functions :47 and :59).
#ifndef SKETCHING_H
#define SKETCHING_H

#include <cstdint>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

using SketchType = std::unordered_set<uint32_t>;
using TranscriptMapping = std::unordered_map<uint32_t, std::vector<std::pair<std::string, const SketchType*>>>;

struct MultiKmerSketch {
    std::unordered_map<unsigned, SketchType> sketches;
};

// FracMinHash: the set of (uint32_t) ntHash forward hashes <= (uint32_t)(UINT32_MAX * fraction)
// (src/sketch.cpp:24-39). Runs on the GPU (skq_sketch_seqs). A sequence shorter than k throws
// std::length_error (the reference's reserve(len - k + 1) would underflow).
std::unordered_set<uint32_t> createSketch_FracMinhash_direct(const std::string& sequence, int k, double fraction);

// k -> hash -> [(transcript id, pointer to that transcript's sketch at k)] (src/sketch.cpp:51-74).
// The pointers point into `transcript_sketches`, which must outlive the result.
std::unordered_map<unsigned, TranscriptMapping> build_kmer_to_transcript_map(
    const std::unordered_map<std::string, MultiKmerSketch>& transcript_sketches);

#endif  // SKETCHING_H
