// Exercises the reference's C++ signatures (include/dropin/*.h, linked against libskq.so) the
// way src/main.cpp calls them, on inputs given as text. Output is canonical text that
// tests/test_dropin.py compares with the oracle.
//   input : lines "T <id> <seq>" (transcripts), "R <id> <seq>" (reads), "K <k,k,...>"
//   output: "S <id> <k> <sorted hashes...>" for every transcript sketch,
//           "A <id> <k> <n>" (extract_and_hash_kmers_nthash size), "V <id> <0|1>" (validity),
//           "C <read id> <tid:score ...>" per read, in the drop-in's order
#include <algorithm>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "kmer.h"
#include "sketch.h"
#include "sparse_chaining.h"

int main() {
    std::vector<std::pair<std::string, std::string>> tx, rd;
    std::vector<unsigned> ks;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string tag, a, b;
        in >> tag >> a;
        std::getline(in >> std::ws, b);
        if (tag == "T") tx.emplace_back(a, b);
        else if (tag == "R") rd.emplace_back(a, b);
        else if (tag == "K") {
            std::stringstream ss(a);
            std::string x;
            while (std::getline(ss, x, ',')) ks.push_back((unsigned)std::stoul(x));
        }
    }
    const double fraction = (double)0.05f;  // src/main.cpp:43
    std::unordered_map<std::string, MultiKmerSketch> tsk;
    std::unordered_map<std::string, Transcript> transcripts;
    for (const auto& [id, seq] : tx) {
        transcripts[id] = Transcript{id, seq, 0};
        for (unsigned k : ks) {
            if (seq.size() < k) continue;
            tsk[id].sketches[k] = createSketch_FracMinhash_direct(seq, (int)k, fraction);
            std::vector<uint32_t> v(tsk[id].sketches[k].begin(), tsk[id].sketches[k].end());
            std::sort(v.begin(), v.end());
            std::cout << "S " << id << " " << k;
            for (uint32_t h : v) std::cout << " " << h;
            std::cout << "\n";
            std::cout << "A " << id << " " << k << " " << extract_and_hash_kmers_nthash(seq, (int)k).size() << "\n";
        }
    }
    const auto index = build_kmer_to_transcript_map(tsk);
    std::unordered_map<std::string, MultiKmerSketch> rsk;
    for (const auto& [id, seq] : rd) {
        std::cout << "V " << id << " " << (is_valid_sequence(seq) ? 1 : 0) << "\n";
        if (!is_valid_sequence(seq)) continue;
        bool ok = true;
        for (unsigned k : ks) ok &= seq.size() >= k;
        if (!ok) continue;
        for (unsigned k : ks) rsk[id].sketches[k] = createSketch_FracMinhash_direct(seq, (int)k, fraction);
    }
    const auto chains = sparse_chain(rsk, index, transcripts, ks, 0.9);
    for (const auto& [id, seq] : rd) {
        auto it = chains.find(id);
        if (it == chains.end()) continue;
        std::cout << "C " << id;
        for (const auto& [t, s] : it->second) std::cout << " " << t << ":" << s;
        std::cout << "\n";
    }
    try {
        (void)extract_and_hash_kmers_nthash("ACG", 5);
        std::cout << "E none\n";
    } catch (const std::runtime_error& e) {
        std::cout << "E " << e.what() << "\n";
    }
    return 0;
}
