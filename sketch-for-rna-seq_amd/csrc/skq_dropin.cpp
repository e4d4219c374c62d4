// skq_dropin.cpp — the reference's C++ sketch / chain signatures (include/dropin/*.h) on top of
// the C ABI. These exist so a caller of the reference can relink unchanged; they convert the
// string-keyed containers to dense arrays, run the HIP path, and convert back. Per-sequence calls
// cannot amortise a launch: batch through skq_sketch / skq_map for throughput.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "dropin/data_io.h"
#include "dropin/kmer.h"
#include "dropin/sketch.h"
#include "dropin/sparse_chaining.h"
#include "skq.h"

namespace {

void check(int rc) {
    if (rc != 0) throw std::runtime_error(std::string("skq: ") + skq_last_error());
}

int device() {
    const char* e = std::getenv("SKQ_DEVICE");
    return e ? std::atoi(e) : 0;
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int dev = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) skq_free(p);
    }
    void ensure(size_t n) {
        n = std::max<size_t>(n, 16);
        if (n <= cap) return;
        if (p) skq_free(p);
        p = nullptr;
        cap = 0;
        check(skq_malloc(dev, n, &p));
        cap = n;
    }
    void put(const void* src, size_t n) {
        ensure(n);
        if (n) check(skq_memcpy_h2d(p, src, n, nullptr));
    }
};

// one per-call sketcher for every k (skq_sketcher_run: pinned mapped buffers, one kernel, one
// synchronisation per call), behind the drop-in's single-threaded contract
std::mutex g_mu;
skq_sketcher* g_sk = nullptr;
std::vector<uint32_t> g_buf;

// at exit the resident server is told to leave and waited for (registered after the HIP runtime
// initialised, so it runs before the runtime's own teardown)
void free_sketcher() {
    std::lock_guard<std::mutex> lock(g_mu);
    if (g_sk) skq_sketcher_free(g_sk);
    g_sk = nullptr;
}

std::unordered_set<uint32_t> gpu_sketch(const std::string& seq, int k, uint32_t threshold) {
    std::lock_guard<std::mutex> lock(g_mu);
    if (!g_sk) {
        check(skq_sketcher_create(device(), 4096, &g_sk));
        std::atexit(free_sketcher);
    }
    const uint64_t nw = seq.size() >= (size_t)k ? seq.size() - (size_t)k + 1 : 0;
    if (g_buf.size() < nw + 1) g_buf.resize(nw + 1);
    uint64_t n = 0;
    check(skq_sketcher_run(g_sk, seq.data(), seq.size(), (uint32_t)k, threshold, g_buf.data(), nw, &n));
    return std::unordered_set<uint32_t>(g_buf.begin(), g_buf.begin() + (ptrdiff_t)std::min<uint64_t>(n, nw));
}

}  // namespace

bool is_valid_sequence(const std::string& sequence) {
    for (unsigned char c : sequence)
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T') return false;
    return true;
}

std::unordered_set<uint32_t> extract_and_hash_kmers_nthash(const std::string& sequence, int k) {
    if (k <= 0) throw std::runtime_error("k-mer length must be positive");
    if (sequence.size() < (size_t)k) throw std::runtime_error("Sequence length is shorter than k-mer length");
    return gpu_sketch(sequence, k, 0xFFFFFFFFu);
}

std::unordered_set<uint32_t> createSketch_FracMinhash_direct(const std::string& sequence, int k, double fraction) {
    if (k <= 0) throw std::runtime_error("k-mer length must be positive");
    if (sequence.size() < (size_t)k) throw std::length_error("createSketch_FracMinhash_direct: sequence shorter than k");
    return gpu_sketch(sequence, k, skq_threshold(fraction));
}

std::unordered_map<unsigned, TranscriptMapping> build_kmer_to_transcript_map(
    const std::unordered_map<std::string, MultiKmerSketch>& transcript_sketches) {
    std::unordered_map<unsigned, TranscriptMapping> out;
    for (const auto& [id, multi] : transcript_sketches)
        for (const auto& [k, sketch] : multi.sketches) {
            TranscriptMapping& m = out[k];
            for (uint32_t h : sketch) m[h].emplace_back(id, &sketch);
        }
    return out;
}

std::unordered_map<std::string, std::vector<std::pair<std::string, int>>> sparse_chain(
    const std::unordered_map<std::string, MultiKmerSketch>& read_sketches,
    const std::unordered_map<unsigned,
                             std::unordered_map<uint32_t, std::vector<std::pair<std::string, const std::unordered_set<uint32_t>*>>>>&
        kmer_to_transcripts,
    const std::unordered_map<std::string, Transcript>& /*transcripts: unused, as in the reference*/,
    const std::vector<unsigned>& kmer_lengths, double fraction) {
    std::unordered_map<std::string, std::vector<std::pair<std::string, int>>> result;
    if (read_sketches.empty()) return result;
    if (kmer_lengths.empty() || kmer_lengths.size() > SKQ_MAX_K)
        throw std::runtime_error("sparse_chain: 1..SKQ_MAX_K k-mer lengths supported");
    const uint32_t nk = (uint32_t)kmer_lengths.size();

    // dense transcript ids in name order (so equal scores come out in name order)
    std::vector<std::string> names;
    for (const auto& [k, map] : kmer_to_transcripts)
        for (const auto& [h, posts] : map)
            for (const auto& pr : posts) names.push_back(pr.first);
    std::sort(names.begin(), names.end());
    names.erase(std::unique(names.begin(), names.end()), names.end());
    std::unordered_map<std::string, uint32_t> tid;
    tid.reserve(names.size());
    for (uint32_t t = 0; t < names.size(); ++t) tid.emplace(names[t], t);

    // CSR table per distinct k of the index that the caller asks for (a k missing from the index
    // is skipped, src/sparse_chaining.cpp:51-58)
    std::vector<uint32_t> tks;
    for (unsigned k : kmer_lengths)
        if (kmer_to_transcripts.count(k) && std::find(tks.begin(), tks.end(), k) == tks.end()) tks.push_back(k);
    std::vector<std::vector<uint32_t>> keys(tks.size()), tids(tks.size());
    std::vector<std::vector<uint64_t>> offs(tks.size());
    std::vector<skq_kmer_table> tables(tks.size());
    for (size_t t = 0; t < tks.size(); ++t) {
        const auto& map = kmer_to_transcripts.at(tks[t]);
        std::vector<uint32_t> ks_sorted;
        ks_sorted.reserve(map.size());
        for (const auto& [h, posts] : map) ks_sorted.push_back(h);
        std::sort(ks_sorted.begin(), ks_sorted.end());
        offs[t].push_back(0);
        for (uint32_t h : ks_sorted) {
            std::vector<uint32_t> ids;
            for (const auto& pr : map.at(h)) ids.push_back(tid.at(pr.first));
            std::sort(ids.begin(), ids.end());
            ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
            keys[t].push_back(h);
            tids[t].insert(tids[t].end(), ids.begin(), ids.end());
            offs[t].push_back(tids[t].size());
        }
        tables[t] = skq_kmer_table{tks[t], (uint64_t)keys[t].size(), keys[t].data(), offs[t].data(), tids[t].data()};
    }
    std::vector<uint32_t> ks(kmer_lengths.begin(), kmer_lengths.end());
    skq_index* ix = nullptr;
    check(skq_index_create(device(), (uint32_t)names.size(), nk, ks.data(), (uint32_t)tables.size(), tables.data(), &ix));
    std::unique_ptr<skq_index, int (*)(skq_index*)> ixg(ix, skq_index_free);

    // reads in batches: per (read, k) sorted hashes, counts, and a present flag (a k missing
    // from the read's sketch is skipped)
    std::vector<const std::string*> rid;
    std::vector<const MultiKmerSketch*> rsk;
    for (const auto& [id, ms] : read_sketches) {
        rid.push_back(&id);
        rsk.push_back(&ms);
    }
    const uint64_t B = std::min<uint64_t>(rid.size(), 1u << 20);
    skq_session* s = nullptr;
    check(skq_session_create(ix, B, 256, &s));
    std::unique_ptr<skq_session, int (*)(skq_session*)> sg(s, skq_session_free);
    DevBuf dh, doff, dcnt, dpres;
    for (int* d : {&dh.dev, &doff.dev, &dcnt.dev, &dpres.dev}) *d = device();
    for (uint64_t r0 = 0; r0 < rid.size(); r0 += B) {
        const uint64_t n = std::min<uint64_t>(B, rid.size() - r0);
        std::vector<uint32_t> hashes, cnt(n * nk);
        std::vector<uint64_t> ho(n * nk + 1);
        std::vector<uint8_t> pres(n * nk);
        for (uint64_t r = 0; r < n; ++r)
            for (uint32_t i = 0; i < nk; ++i) {
                ho[r * nk + i] = hashes.size();
                auto it = rsk[r0 + r]->sketches.find(ks[i]);
                if (it == rsk[r0 + r]->sketches.end()) continue;
                pres[r * nk + i] = 1;
                const size_t at = hashes.size();
                hashes.insert(hashes.end(), it->second.begin(), it->second.end());
                std::sort(hashes.begin() + (ptrdiff_t)at, hashes.end());
                cnt[r * nk + i] = (uint32_t)(hashes.size() - at);
            }
        ho[n * nk] = hashes.size();
        dh.put(hashes.data(), hashes.size() * 4);
        doff.put(ho.data(), ho.size() * 8);
        dcnt.put(cnt.data(), cnt.size() * 4);
        dpres.put(pres.data(), pres.size());
        check(skq_chain_sketches(s, n, static_cast<const uint32_t*>(dh.p), static_cast<const uint64_t*>(doff.p),
                                 static_cast<const uint32_t*>(dcnt.p), static_cast<const uint8_t*>(dpres.p), fraction,
                                 0, nullptr));
        uint64_t nh = 0, nc = 0;
        check(skq_session_export(s, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &nh, &nc));
        std::vector<uint64_t> co(n + 1);
        std::vector<uint32_t> ct(nc + 1), cs(nc + 1);
        check(skq_session_export(s, nullptr, nullptr, nullptr, co.data(), ct.data(), cs.data(), &nh, &nc));
        for (uint64_t r = 0; r < n; ++r) {
            auto& v = result[*rid[r0 + r]];  // reads without hits map to an empty list
            for (uint64_t c = co[r]; c < co[r + 1]; ++c) v.emplace_back(names[ct[c]], (int)cs[c]);
        }
    }
    return result;
}
