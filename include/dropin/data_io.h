// Drop-in for the reference's include/data_io.h types used on the sketch/chain path
// (include/data_io.h:17-43 and :51): same names, same members, same meaning.
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

#endif  // DATA_IO_H
