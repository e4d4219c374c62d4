// Drop-in for the reference's include/data_io.h (types :17-43, functions :51-115): the same
// names, members and signatures, so a reference translation unit compiles unchanged with
// -I include/dropin ahead of its own include/. The definitions are in libskq.so
// (csrc/skq_dropin.cpp, over the host IO of csrc/skq_io.cpp); a build that keeps the reference's
// own src/data_io.cpp links that instead (its definitions take precedence over the library's).
#ifndef DATA_IO_H
#define DATA_IO_H

#include <cstdint>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

using SketchType = std::unordered_set<uint32_t>;
using TranscriptMapping = std::unordered_map<uint32_t, std::vector<std::pair<std::string, const SketchType*>>>;

struct Transcript {
    std::string id;
    std::string sequence;
    int length;
};

struct Read {
    std::string id;
    std::string sequence;
    std::string quality;
};

// true iff every byte is one of 'A' 'C' 'G' 'T' (src/data_io.cpp:17-34)
bool is_valid_sequence(const std::string& sequence);

// id = header up to the first space; the first record of an id wins; records that are not
// uppercase ACGT are dropped except the last one; Transcript::length is 0 (src/data_io.cpp:47-80).
// Throws std::runtime_error("Could not open FASTA file: ...").
std::unordered_map<std::string, Transcript> load_fasta(const std::string& fasta_file);

// 4-line records; a read whose sequence is not uppercase ACGT is dropped, the last record of an id
// wins; prints "Actual number of reads: N" (src/data_io.cpp:94-117; no caller in the reference).
std::unordered_map<std::string, Read> load_fastq(const std::string& fastq_file);

// "Name,NumReads,EM_Abundance", one row per transcript present in both maps, in the transcripts
// map's order, values as an ostream prints doubles (src/data_io.cpp:133-152).
void output_to_csv(const std::string& filename,
                   const std::unordered_map<std::string, double>& read_counts,
                   const std::unordered_map<std::string, double>& pi,
                   const std::unordered_map<std::string, Transcript>& transcripts);

// The reference's binary index (src/data_io.cpp:165-220 / :233-304): native endian, size_t = u64,
// unsigned = u32; an unopenable path prints to stderr and returns (as the reference does).
void save_index(const std::string& index_output_path,
                std::vector<unsigned>& kmer_lengths,
                const std::unordered_map<unsigned, TranscriptMapping>& kmer_to_transcripts,
                const std::unordered_map<std::string, Transcript>& transcripts);

void load_index(const std::string& index_path,
                std::vector<unsigned>& kmer_lengths,
                std::unordered_map<unsigned, TranscriptMapping>& kmer_to_transcripts,
                std::unordered_map<std::string, Transcript>& transcripts);

#endif  // DATA_IO_H
