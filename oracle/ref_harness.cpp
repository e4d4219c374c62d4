// ref_harness.cpp — TEST INFRASTRUCTURE ONLY. A C-ABI shim over the reference's own code,
// compiled UNMODIFIED from /root/reference/src/{sparse_chaining,data_io,isoform_assignment}.cpp
// (recipe: oracle/ref.mk, output oracle/_ref/libref.so). It lets the CPU tests pin the oracle's
// chain / EM / assignment / index-format / FASTA / CSV legs against the reference itself.
//
// The reference's kmer.cpp, sketch.cpp and main.cpp need the third-party ntHash library, which the
// image lacks; they are not built (no stand-in is written for ntHash). The hashing leg is pinned
// by ntHash's own tables instead (tests/golden/nthash_tables.json).
//
// Conventions: transcripts are named by the caller (names[t]) or "t<t>"; reads are "r<r>". The
// reference's containers are unordered, so every output is put in a canonical order here:
// candidates by score desc, then tid asc (std::sort in src/sparse_chaining.cpp:108-109 is
// unstable, so only this normalised order is comparable); dumps sorted by id / key.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "data_io.h"
#include "isoform_assignment.h"
#include "sparse_chaining.h"

namespace {

using KMap = std::unordered_map<unsigned, TranscriptMapping>;

struct RefIndex {
    std::vector<std::string> names;
    std::unordered_map<std::string, uint32_t> tid_of;
    KMap map;
    std::unordered_map<std::string, Transcript> transcripts;
};

std::string tname(uint32_t t) { return "t" + std::to_string(t); }

double g_chain_seconds = 0;  // wall time of the last ref_chain's sparse_chain call alone

}  // namespace

extern "C" {

// kmer_to_transcripts from CSR tables (per k: keys ascending, offs, tids) — the structure
// build_kmer_to_transcript_map (src/sketch.cpp:51-74) returns; the sketch pointers stay null,
// as after load_index (src/data_io.cpp:295). names may be null ("t<i>").
void* ref_index_new(uint32_t ntx, const char* const* names, unsigned nk, const unsigned* ks,
                    const uint64_t* nkeys, const uint32_t* const* keys, const uint64_t* const* offs,
                    const uint32_t* const* tids) {
    auto* ix = new RefIndex();
    ix->names.resize(ntx);
    for (uint32_t t = 0; t < ntx; ++t) {
        ix->names[t] = names ? std::string(names[t]) : tname(t);
        ix->tid_of[ix->names[t]] = t;
        ix->transcripts[ix->names[t]] = Transcript{ix->names[t], std::string(), 0};
    }
    for (unsigned i = 0; i < nk; ++i) {
        TranscriptMapping& m = ix->map[ks[i]];
        for (uint64_t j = 0; j < nkeys[i]; ++j) {
            auto& v = m[keys[i][j]];
            for (uint64_t q = offs[i][j]; q < offs[i][j + 1]; ++q) v.emplace_back(ix->names[tids[i][q]], nullptr);
        }
    }
    return ix;
}

void ref_index_free(void* h) { delete static_cast<RefIndex*>(h); }

// seconds the last ref_chain spent inside sparse_chain itself (container set-up excluded)
double ref_chain_seconds(void) { return g_chain_seconds; }

// sparse_chain (src/sparse_chaining.cpp:29-115) over a batch. Read r's sketch at k slot i is
// hashes[hash_offs[r*nk+i] .. hash_offs[r*nk+i+1]); present[r*nk+i] == 0 leaves that k out of the
// read's MultiKmerSketch (null present: all present). kmer_lengths = ks (may name a k the index
// lacks). Output CSR: cand_offs[n+1]; returns 0, or -1 when cap is too small.
int ref_chain(void* h, uint64_t n, unsigned nk, const unsigned* ks, const uint64_t* hash_offs,
              const uint32_t* hashes, const uint8_t* present, double fraction, uint64_t* cand_offs,
              uint32_t* cand_tid, uint32_t* cand_score, uint64_t cap) {
    auto* ix = static_cast<RefIndex*>(h);
    std::unordered_map<std::string, MultiKmerSketch> reads;
    for (uint64_t r = 0; r < n; ++r) {
        MultiKmerSketch ms;
        for (unsigned i = 0; i < nk; ++i) {
            const uint64_t e = r * nk + i;
            if (present && !present[e]) continue;
            SketchType& s = ms.sketches[ks[i]];
            for (uint64_t q = hash_offs[e]; q < hash_offs[e + 1]; ++q) s.insert(hashes[q]);
        }
        reads["r" + std::to_string(r)] = std::move(ms);
    }
    std::vector<unsigned> kl(ks, ks + nk);
    const auto t0 = std::chrono::steady_clock::now();
    const auto res = sparse_chain(reads, ix->map, ix->transcripts, kl, fraction);
    g_chain_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t o = 0;
    cand_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        auto it = res.find("r" + std::to_string(r));
        std::vector<std::pair<int, uint32_t>> c;  // (score, tid)
        if (it != res.end())
            for (const auto& [name, score] : it->second) c.emplace_back(score, ix->tid_of.at(name));
        std::sort(c.begin(), c.end(), [](const auto& a, const auto& b) {
            return a.first != b.first ? a.first > b.first : a.second < b.second;
        });
        if (o + c.size() > cap) return -1;
        for (const auto& [score, t] : c) {
            cand_tid[o] = t;
            cand_score[o] = (uint32_t)score;
            ++o;
        }
        cand_offs[r + 1] = o;
    }
    return 0;
}

// estimate_isoform_abundance_em + assign_reads_to_isoforms (src/isoform_assignment.cpp:9-97)
// over reads' candidate lists (CSR; a read with no candidates is still a read, as in quant's
// homologous_segments). pi[ntx], counts[ntx], assigned[ntx] (1 where the reference's
// weighted_read_counts has the transcript) out.
void ref_em_assign(uint64_t n, const uint64_t* cand_offs, const uint32_t* cand_tid, const uint32_t* cand_score,
                   uint32_t ntx, int max_iterations, double convergence, double* pi, double* counts,
                   uint8_t* assigned) {
    std::unordered_map<std::string, Transcript> transcripts;
    for (uint32_t t = 0; t < ntx; ++t) transcripts[tname(t)] = Transcript{tname(t), std::string(), 0};
    std::unordered_map<std::string, std::vector<std::pair<std::string, int>>> hs;
    for (uint64_t r = 0; r < n; ++r) {
        auto& v = hs["r" + std::to_string(r)];
        for (uint64_t q = cand_offs[r]; q < cand_offs[r + 1]; ++q) v.emplace_back(tname(cand_tid[q]), (int)cand_score[q]);
    }
    const auto p = estimate_isoform_abundance_em(hs, transcripts, max_iterations, convergence);
    const auto c = assign_reads_to_isoforms(hs, p, transcripts);
    for (uint32_t t = 0; t < ntx; ++t) {
        auto a = p.find(tname(t));
        pi[t] = a == p.end() ? -1.0 : a->second;
        auto b = c.find(tname(t));
        counts[t] = b == c.end() ? 0.0 : b->second;
        assigned[t] = b != c.end();
    }
}

// output_to_csv (src/data_io.cpp:133-152) for transcripts t0..t<ntx-1> named names[t]; rows
// exist where assigned[t] (weighted_read_counts has the id) — pi holds every transcript.
int ref_output_csv(const char* path, uint32_t ntx, const char* const* names, const double* counts,
                   const uint8_t* assigned, const double* pi) {
    std::unordered_map<std::string, double> rc, p;
    std::unordered_map<std::string, Transcript> transcripts;
    for (uint32_t t = 0; t < ntx; ++t) {
        transcripts[names[t]] = Transcript{names[t], std::string(), 0};
        p[names[t]] = pi[t];
        if (assigned[t]) rc[names[t]] = counts[t];
    }
    try {
        output_to_csv(path, rc, p, transcripts);
    } catch (...) {
        return -1;
    }
    return 0;
}

int ref_is_valid_sequence(const char* s, uint64_t len) { return is_valid_sequence(std::string(s, len)) ? 1 : 0; }

// load_fasta (src/data_io.cpp:47-80), dumped sorted by id as "id\tsequence\tlength\n".
int ref_load_fasta_dump(const char* path, const char* out) {
    std::unordered_map<std::string, Transcript> tx;
    try {
        tx = load_fasta(path);
    } catch (...) {
        return -1;
    }
    std::vector<std::string> ids;
    for (const auto& kv : tx) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    std::ofstream f(out, std::ios::binary);
    for (const auto& id : ids) f << id << '\t' << tx[id].sequence << '\t' << tx[id].length << '\n';
    return 0;
}

// save_index (src/data_io.cpp:165-221) from CSR tables and transcripts (names, sequences; the
// length field 0 as after load_fasta's emplace of a moved-from string).
int ref_save_index(const char* path, unsigned nk, const unsigned* ks, uint32_t ntx, const char* const* names,
                   const char* seqs, const uint64_t* seq_offs, const uint64_t* nkeys, const uint32_t* const* keys,
                   const uint64_t* const* offs, const uint32_t* const* tids) {
    auto* ix = static_cast<RefIndex*>(ref_index_new(ntx, names, nk, ks, nkeys, keys, offs, tids));
    for (uint32_t t = 0; t < ntx; ++t)
        ix->transcripts[names[t]] = Transcript{names[t], std::string(seqs + seq_offs[t], seq_offs[t + 1] - seq_offs[t]), 0};
    std::vector<unsigned> kl(ks, ks + nk);
    save_index(path, kl, ix->map, ix->transcripts);
    delete ix;
    return 0;
}

// load_index (src/data_io.cpp:233-304), dumped canonically: "K k1 k2 ...\n", then per transcript
// sorted by id "T id\tsequence\tlength\n", then per k (ascending) per key (ascending)
// "M k key id1 id2 ...\n" with the ids sorted.
int ref_load_index_dump(const char* path, const char* out) {
    std::vector<unsigned> kl;
    KMap map;
    std::unordered_map<std::string, Transcript> tx;
    load_index(path, kl, map, tx);
    std::ofstream f(out, std::ios::binary);
    f << "K";
    for (unsigned k : kl) f << ' ' << k;
    f << '\n';
    std::vector<std::string> ids;
    for (const auto& kv : tx) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    for (const auto& id : ids) f << "T " << id << '\t' << tx[id].sequence << '\t' << tx[id].length << '\n';
    std::vector<unsigned> mk;
    for (const auto& kv : map) mk.push_back(kv.first);
    std::sort(mk.begin(), mk.end());
    for (unsigned k : mk) {
        const auto& m = map[k];
        std::vector<uint32_t> keys;
        for (const auto& kv : m) keys.push_back(kv.first);
        std::sort(keys.begin(), keys.end());
        for (uint32_t key : keys) {
            std::vector<std::string> v;
            for (const auto& pr : m.at(key)) v.push_back(pr.first);
            std::sort(v.begin(), v.end());
            f << "M " << k << ' ' << key;
            for (const auto& s : v) f << ' ' << s;
            f << '\n';
        }
    }
    return 0;
}

}  // extern "C"
