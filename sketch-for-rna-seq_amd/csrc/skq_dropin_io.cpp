// skq_dropin_io.cpp — the rest of the reference's host surface that src/main.cpp calls
// (include/data_io.h:51-115, include/isoform_assignment.h:24-44), so the reference's own CLI
// links against libskq.so alone (tests/test_dropin_ref.py). Same signatures,
// same observable behaviour (messages, error handling, duplicate-id rules); the containers are
// the reference's. The EM and the assignment sum in a fixed order (reads in the map's order,
// candidates in list order) where the reference follows unordered_map order for the posterior
// sums, so pi and the counts agree with it to rounding (tests: rtol 1e-9).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "dropin/data_io.h"
#include "dropin/isoform_assignment.h"
#include "skq_host.h"

namespace {

// binary reader over a FILE*: a short read marks the stream failed and later reads return zeros,
// as the reference's std::ifstream::read leaves its targets on a truncated file
struct BinIn {
    FILE* f;
    bool ok = true;
    template <typename T>
    T get() {
        T v{};
        if (ok && std::fread(&v, sizeof v, 1, f) != 1) ok = false;
        return ok ? v : T{};
    }
    std::string str(size_t n) {
        std::string s(n, '\0');
        if (ok && n && std::fread(&s[0], 1, n, f) != n) ok = false;
        return s;
    }
};

struct BinOut {
    FILE* f;
    template <typename T>
    void put(const T& v) {
        std::fwrite(&v, sizeof v, 1, f);
    }
    void str(const std::string& s) {
        put<size_t>(s.size());
        if (!s.empty()) std::fwrite(s.data(), 1, s.size(), f);
    }
};

}  // namespace

// src/data_io.cpp:47-80 through skq_fasta_load (the same record rules: first id wins, every record
// but the last validated, id up to the first space); Transcript::length is 0 as in the reference
// (its moved-from sequence's size)
std::unordered_map<std::string, Transcript> load_fasta(const std::string& fasta_file) {
    skq_seqs* s = nullptr;
    if (skq_fasta_load(fasta_file.c_str(), &s) != 0) throw std::runtime_error("Could not open FASTA file: " + fasta_file);
    const uint8_t* bytes = nullptr;
    const uint64_t *offs = nullptr, *noffs = nullptr;
    const char* names = nullptr;
    skq_seqs_view(s, &bytes, &offs, &names, &noffs);
    std::unordered_map<std::string, Transcript> out;
    const uint64_t n = skq_seqs_count(s);
    out.reserve(n);
    for (uint64_t t = 0; t < n; ++t) {
        std::string id(names + noffs[t], noffs[t + 1] - noffs[t]);
        std::string seq(reinterpret_cast<const char*>(bytes) + offs[t], offs[t + 1] - offs[t]);
        out.emplace(id, Transcript{id, std::move(seq), 0});
    }
    skq_seqs_free(s);
    return out;
}

// src/data_io.cpp:94-117
std::unordered_map<std::string, Read> load_fastq(const std::string& fastq_file) {
    std::ifstream in(fastq_file);
    if (!in) throw std::runtime_error("Could not open FASTQ file: " + fastq_file);
    std::unordered_map<std::string, Read> reads;
    std::string line;
    int count = 0;
    while (std::getline(in, line)) {
        if (line.empty() || line[0] != '@') continue;
        Read r;
        r.id = line.substr(1);
        std::getline(in, r.sequence);
        std::getline(in, line);
        std::getline(in, r.quality);
        ++count;
        if (is_valid_sequence(r.sequence)) reads[r.id] = r;
    }
    std::cout << "Actual number of reads: " << count << std::endl;
    return reads;
}

// src/data_io.cpp:133-152 (the ostream's default double formatting: 6 significant digits)
void output_to_csv(const std::string& filename, const std::unordered_map<std::string, double>& read_counts,
                   const std::unordered_map<std::string, double>& pi,
                   const std::unordered_map<std::string, Transcript>& transcripts) {
    std::ofstream out(filename);
    if (!out.is_open()) throw std::runtime_error("Could not open file for writing: " + filename);
    out << "Name,NumReads,EM_Abundance\n";
    for (const auto& kv : transcripts) {
        const auto c = read_counts.find(kv.first);
        const auto p = pi.find(kv.first);
        if (c != read_counts.end() && p != pi.end()) out << kv.first << "," << c->second << "," << p->second << "\n";
    }
}

// src/data_io.cpp:165-220: k list; transcripts (id, sequence, length); per k the key -> id lists
void save_index(const std::string& index_output_path, std::vector<unsigned>& kmer_lengths,
                const std::unordered_map<unsigned, TranscriptMapping>& kmer_to_transcripts,
                const std::unordered_map<std::string, Transcript>& transcripts) {
    FILE* f = std::fopen(index_output_path.c_str(), "wb");
    if (!f) {
        std::cerr << "Error: Unable to open file for writing: " << index_output_path << std::endl;
        return;
    }
    BinOut w{f};
    w.put<size_t>(kmer_lengths.size());
    for (unsigned k : kmer_lengths) w.put<unsigned>(k);
    w.put<size_t>(transcripts.size());
    for (const auto& kv : transcripts) {
        w.str(kv.first);
        w.str(kv.second.sequence);
        w.put<int>(kv.second.length);
    }
    w.put<size_t>(kmer_to_transcripts.size());
    for (const auto& km : kmer_to_transcripts) {
        w.put<unsigned>(km.first);
        w.put<size_t>(km.second.size());
        for (const auto& kv : km.second) {
            w.put<uint32_t>(kv.first);
            w.put<size_t>(kv.second.size());
            for (const auto& pr : kv.second) w.str(pr.first);
        }
    }
    std::fclose(f);
    std::cout << "Index saved to " << index_output_path << std::endl;
}

// src/data_io.cpp:233-304: a later transcript of the same id replaces an earlier one
// (transcripts[id] = ...), sketch pointers come back null; an unopenable path prints and returns
void load_index(const std::string& index_path, std::vector<unsigned>& kmer_lengths,
                std::unordered_map<unsigned, TranscriptMapping>& kmer_to_transcripts,
                std::unordered_map<std::string, Transcript>& transcripts) {
    FILE* f = std::fopen(index_path.c_str(), "rb");
    if (!f) {
        std::cerr << "Error: Unable to open file for reading: " << index_path << std::endl;
        return;
    }
    std::vector<char> buf(1 << 22);
    std::setvbuf(f, buf.data(), _IOFBF, buf.size());
    BinIn r{f};
    const size_t nk = r.get<size_t>();
    kmer_lengths.resize(nk);
    for (size_t i = 0; i < nk; ++i) kmer_lengths[i] = r.get<unsigned>();
    const size_t ntx = r.get<size_t>();
    transcripts.clear();
    for (size_t t = 0; t < ntx; ++t) {
        std::string id = r.str(r.get<size_t>());
        std::string seq = r.str(r.get<size_t>());
        const int length = r.get<int>();
        transcripts[id] = Transcript{id, std::move(seq), length};
    }
    const size_t nmaps = r.get<size_t>();
    kmer_to_transcripts.clear();
    for (size_t m = 0; m < nmaps; ++m) {
        const unsigned k = r.get<unsigned>();
        const size_t nkeys = r.get<size_t>();
        TranscriptMapping map;
        map.reserve(nkeys);
        for (size_t j = 0; j < nkeys; ++j) {
            const uint32_t key = r.get<uint32_t>();
            const size_t np = r.get<size_t>();
            std::vector<std::pair<std::string, const SketchType*>> v;
            v.reserve(np);
            for (size_t q = 0; q < np; ++q) v.emplace_back(r.str(r.get<size_t>()), nullptr);
            map[key] = std::move(v);
        }
        kmer_to_transcripts[k] = std::move(map);
    }
    std::fclose(f);
    std::cout << "Index loaded from " << index_path << std::endl;
}

namespace {

// sparse_chain's results in CSR form over dense ids: ids [0, T) are `transcripts` (their map
// order), candidates naming anything else get ids past them (the reference's pi[...] inserts
// such a name with 0 at its first E-step, src/isoform_assignment.cpp:37)
struct Dense {
    std::vector<std::string> names;
    std::unordered_map<std::string, uint32_t> id;
    std::vector<uint64_t> offs{0};
    std::vector<uint32_t> tid, score;
    uint32_t T = 0;
    Dense(const std::unordered_map<std::string, std::vector<std::pair<std::string, int>>>& hs,
          const std::unordered_map<std::string, Transcript>& transcripts) {
        id.reserve(transcripts.size());
        for (const auto& kv : transcripts) {
            id.emplace(kv.first, (uint32_t)names.size());
            names.push_back(kv.first);
        }
        T = (uint32_t)names.size();
        for (const auto& rd : hs) {
            for (const auto& c : rd.second) {
                auto it = id.find(c.first);
                if (it == id.end()) {
                    it = id.emplace(c.first, (uint32_t)names.size()).first;
                    names.push_back(c.first);
                }
                tid.push_back(it->second);
                score.push_back((uint32_t)c.second);
            }
            offs.push_back(tid.size());
        }
    }
};

}  // namespace

// src/isoform_assignment.cpp:9-68: pi = 1/T over the transcripts, then rounds of E-step (posterior
// sums of every read with a positive denominator) and M-step (post + (double)(0.01f / R) +
// (double)0.01f over every name in pi), stopping when sum |d pi| < the threshold
std::unordered_map<std::string, double> estimate_isoform_abundance_em(
    const std::unordered_map<std::string, std::vector<std::pair<std::string, int>>>& homologous_segments,
    const std::unordered_map<std::string, Transcript>& transcripts, int max_iterations, double convergence_threshold) {
    Dense d(homologous_segments, transcripts);
    const uint32_t N = (uint32_t)d.names.size();
    std::vector<double> pi(N, 0.0), post(N);
    for (uint32_t t = 0; t < d.T; ++t) pi[t] = 1.0 / (double)transcripts.size();
    const uint64_t R = homologous_segments.size();
    for (int it = 0; it < max_iterations; ++it) {
        double change = 0;
        if (skq_em_estep_host(R, d.offs.data(), d.tid.data(), d.score.data(), N, pi.data(), 1, post.data()) ||
            skq_em_mstep_host(N, pi.data(), post.data(), R, &change))
            throw std::runtime_error(std::string("skq EM: ") + skq_last_error());
        if (change < convergence_threshold) break;
    }
    std::unordered_map<std::string, double> out;
    out.reserve(N);
    // names the reference's pi never holds: candidates of reads it skips are still inserted by
    // its E-step lookup, so every name seen is in pi, as here
    for (uint32_t t = 0; t < N; ++t) out.emplace(d.names[t], pi[t]);
    return out;
}

// src/isoform_assignment.cpp:70-97: per read, its candidates' pi * score shares (names absent
// from pi are skipped); a transcript gets a row once any read with a positive total names it
std::unordered_map<std::string, double> assign_reads_to_isoforms(
    const std::unordered_map<std::string, std::vector<std::pair<std::string, int>>>& homologous_segments,
    const std::unordered_map<std::string, double>& pi, const std::unordered_map<std::string, Transcript>& /*unused*/) {
    std::unordered_map<std::string, double> counts;
    std::vector<const double*> p;
    for (const auto& rd : homologous_segments) {
        double total = 0;
        p.clear();
        for (const auto& c : rd.second) {
            const auto it = pi.find(c.first);
            p.push_back(it == pi.end() ? nullptr : &it->second);
            if (p.back()) total += *p.back() * c.second;
        }
        if (!(total > 0.0)) continue;
        size_t q = 0;
        for (const auto& c : rd.second) {
            const double* pv = p[q++];
            if (pv) counts[c.first] += (*pv * c.second) / total;
        }
    }
    return counts;
}
