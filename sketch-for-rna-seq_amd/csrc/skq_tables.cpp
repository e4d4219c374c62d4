// skq_tables.cpp — host-side inverted-index builder (C ABI in include/skq_host.h).
//
// Restates build_and_save_index's sketch loop and build_kmer_to_transcript_map
// (reference src/main.cpp:66-85, src/sketch.cpp:51-74) with dense transcript ids instead of
// string keys: transcripts are sketched in parallel (one std::thread per slice), each emits
// (hash << 32 | tid) words per k, and one sort per k yields the CSR (keys ascending, tids
// ascending per key).
//
// The rolling hash here is the 33-bit lane of ntHash's forward hash (bits 0..32 of the split
// rotate evolve on their own, and the reference keeps only bits 0..31), with ntHash's rule for
// bases outside ACGTU/acgtu: every window containing one is skipped.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "skq_host.h"
#include "skq_internal.h"

struct skq_tables {
    struct T {
        uint32_t k;
        std::vector<uint32_t> keys;
        std::vector<uint64_t> offs;
        std::vector<uint32_t> tids;
    };
    std::vector<T> t;
};

namespace {

int hfail(int code, const char* msg) { return skq::set_error(code, msg); }

// byte -> 2-bit code for ntHash-valid bases (A/a 0, C/c 1, T/t/U/u 2, G/g 3), 4 = skipped
struct CodeTable {
    uint8_t c[256];
    CodeTable() {
        std::memset(c, 4, sizeof c);
        c['A'] = c['a'] = 0;
        c['C'] = c['c'] = 1;
        c['T'] = c['t'] = c['U'] = c['u'] = 2;
        c['G'] = c['g'] = 3;
    }
};
const CodeTable kCodes;

// retained hashes of one sequence at one k, appended to out (unsorted, may repeat)
void sketch_into(const uint8_t* s, uint64_t len, uint32_t k, uint32_t thr, const uint64_t* rk,
                 std::vector<uint32_t>& out) {
    if (len < k) return;
    uint64_t h = 0;
    uint64_t run = 0;  // valid bases ending at the current position
    for (uint64_t p = 0; p < len; ++p) {
        const uint8_t c = kCodes.c[s[p]];
        if (c == 4) {
            run = 0;
            h = 0;
            continue;
        }
        ++run;
        h = ((h << 1) | (h >> 32)) & skq::M33;
        h ^= skq::SEED33[c];
        if (run > k) h ^= rk[kCodes.c[s[p - k]]];
        if (run >= k && (uint32_t)h <= thr) out.push_back((uint32_t)h);
    }
}

void sort_unique(std::vector<uint32_t>& v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
}

}  // namespace

namespace skq {
void sketch_positions(const uint8_t* s, uint64_t len, uint32_t k, uint32_t thr, std::vector<uint32_t>& out) {
    uint64_t rk[4];
    for (int c = 0; c < 4; ++c) rk[c] = rot33(SEED33[c], k);
    sketch_into(s, len, k, thr, rk, out);
}

// Sorts ascending with up to `threads` threads: sorted chunks, then rounds of pairwise merges.
// Input that is already sorted (the product's own index files) costs one pass.
void parallel_sort_u64(std::vector<uint64_t>& v, int threads) {
    if (std::is_sorted(v.begin(), v.end())) return;
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    const uint64_t n = v.size();
    int P = 1;
    while (P * 2 <= threads && n / (uint64_t)(P * 2) >= (1u << 16)) P *= 2;
    std::vector<uint64_t> cut(P + 1);
    for (int i = 0; i <= P; ++i) cut[i] = n * (uint64_t)i / (uint64_t)P;
    {
        std::vector<std::thread> pool;
        for (int i = 0; i < P; ++i)
            pool.emplace_back([&, i] { std::sort(v.begin() + (ptrdiff_t)cut[i], v.begin() + (ptrdiff_t)cut[i + 1]); });
        for (auto& t : pool) t.join();
    }
    for (int w = 1; w < P; w *= 2) {
        std::vector<std::thread> pool;
        for (int i = 0; i + w < P; i += 2 * w) {
            const uint64_t a = cut[i], m = cut[i + w], b = cut[std::min(i + 2 * w, P)];
            pool.emplace_back([&v, a, m, b] {
                std::inplace_merge(v.begin() + (ptrdiff_t)a, v.begin() + (ptrdiff_t)m, v.begin() + (ptrdiff_t)b);
            });
        }
        for (auto& t : pool) t.join();
    }
}
}  // namespace skq

namespace {

void finalize(skq_tables::T& T, std::vector<uint64_t>& words) {
    skq::parallel_sort_u64(words, 0);
    words.erase(std::unique(words.begin(), words.end()), words.end());
    T.tids.resize(words.size());
    T.keys.clear();
    T.offs.clear();
    for (uint64_t j = 0; j < words.size(); ++j) {
        const uint32_t key = (uint32_t)(words[j] >> 32);
        if (j == 0 || key != T.keys.back()) {
            T.keys.push_back(key);
            T.offs.push_back(j);
        }
        T.tids[j] = (uint32_t)words[j];
    }
    T.offs.push_back(words.size());
}

}  // namespace

extern "C" {

int64_t skq_host_sketch(const uint8_t* seq, uint64_t len, uint32_t k, uint32_t threshold, uint32_t* out) {
    if (k == 0 || len < k) return -1;
    uint64_t rk[4];
    for (int c = 0; c < 4; ++c) rk[c] = skq::rot33(skq::SEED33[c], k);
    std::vector<uint32_t> v;
    sketch_into(seq, len, k, threshold, rk, v);
    sort_unique(v);
    std::copy(v.begin(), v.end(), out);
    return (int64_t)v.size();
}

int skq_tables_build(uint32_t ntx, const uint8_t* seqs, const uint64_t* offs, uint32_t nk, const uint32_t* ks,
                     uint32_t threshold, int nthreads, skq_tables** out) {
    if (!out) return hfail(-1, "out is null");
    *out = nullptr;
    if (nk == 0 || nk > SKQ_MAX_K) return hfail(-1, "k list must hold 1..SKQ_MAX_K entries");
    std::vector<uint32_t> dk;  // distinct ks, first-seen order
    uint32_t maxk = 0;
    for (uint32_t i = 0; i < nk; ++i) {
        if (ks[i] == 0) return hfail(-1, "k must be greater than 0");
        maxk = std::max(maxk, ks[i]);
        if (std::find(dk.begin(), dk.end(), ks[i]) == dk.end()) dk.push_back(ks[i]);
    }
    int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::max(1, std::min<int>(nt, (int)std::max<uint32_t>(1, ntx / 64 + 1)));
    const size_t nd = dk.size();
    std::vector<std::vector<std::vector<uint64_t>>> part(nt, std::vector<std::vector<uint64_t>>(nd));
    std::vector<std::thread> th;
    for (int w = 0; w < nt; ++w) {
        th.emplace_back([&, w] {
            std::vector<uint64_t> rk(nd * 4);
            for (size_t d = 0; d < nd; ++d)
                for (int c = 0; c < 4; ++c) rk[d * 4 + c] = skq::rot33(skq::SEED33[c], dk[d]);
            std::vector<uint32_t> buf;
            const uint64_t a = (uint64_t)ntx * w / nt, b = (uint64_t)ntx * (w + 1) / nt;
            for (uint64_t t = a; t < b; ++t) {
                const uint64_t len = offs[t + 1] - offs[t];
                if (len < maxk) continue;  // shorter than some k: not indexed (src/main.cpp:66-75)
                for (size_t d = 0; d < nd; ++d) {
                    buf.clear();
                    sketch_into(seqs + offs[t], len, dk[d], threshold, &rk[d * 4], buf);
                    sort_unique(buf);
                    for (uint32_t h : buf) part[w][d].push_back(((uint64_t)h << 32) | t);
                }
            }
        });
    }
    for (auto& x : th) x.join();
    auto* T = new skq_tables();
    T->t.resize(nd);
    std::vector<std::thread> fin;
    for (size_t d = 0; d < nd; ++d) {
        fin.emplace_back([&, d] {
            std::vector<uint64_t> words;
            size_t tot = 0;
            for (int w = 0; w < nt; ++w) tot += part[w][d].size();
            words.reserve(tot);
            for (int w = 0; w < nt; ++w) {
                words.insert(words.end(), part[w][d].begin(), part[w][d].end());
                std::vector<uint64_t>().swap(part[w][d]);
            }
            T->t[d].k = dk[d];
            finalize(T->t[d], words);
        });
    }
    for (auto& x : fin) x.join();
    *out = T;
    return 0;
}

int skq_tables_from_pairs(uint32_t ntables, const uint32_t* ks, const uint64_t* npairs,
                          const uint32_t* const* hashes, const uint32_t* const* tids, skq_tables** out) {
    if (!out) return hfail(-1, "out is null");
    auto* T = new skq_tables();
    T->t.resize(ntables);
    for (uint32_t d = 0; d < ntables; ++d) {
        std::vector<uint64_t> words(npairs[d]);
        for (uint64_t j = 0; j < npairs[d]; ++j) words[j] = ((uint64_t)hashes[d][j] << 32) | tids[d][j];
        T->t[d].k = ks[d];
        finalize(T->t[d], words);
    }
    *out = T;
    return 0;
}

}  // extern "C"

int skq::tables_from_words(uint32_t ntables, const uint32_t* ks, std::vector<uint64_t>* words, skq_tables** out) {
    if (!out) return hfail(-1, "out is null");
    auto* T = new skq_tables();
    T->t.resize(ntables);
    for (uint32_t d = 0; d < ntables; ++d) {
        T->t[d].k = ks[d];
        finalize(T->t[d], words[d]);
        std::vector<uint64_t>().swap(words[d]);
    }
    *out = T;
    return 0;
}

int skq::tables_from_csr(uint32_t ntables, const uint32_t* ks, std::vector<uint32_t>* keys,
                         std::vector<uint64_t>* offs, std::vector<uint32_t>* tids, skq_tables** out) {
    if (!out) return hfail(-1, "out is null");
    auto* T = new skq_tables();
    T->t.resize(ntables);
    for (uint32_t d = 0; d < ntables; ++d) {
        T->t[d].k = ks[d];
        T->t[d].keys = std::move(keys[d]);
        T->t[d].offs = std::move(offs[d]);
        T->t[d].tids = std::move(tids[d]);
    }
    *out = T;
    return 0;
}

extern "C" {

uint32_t skq_tables_count(const skq_tables* t) { return t ? (uint32_t)t->t.size() : 0; }

int skq_tables_get(const skq_tables* t, uint32_t i, skq_kmer_table* o) {
    if (!t || !o || i >= t->t.size()) return hfail(-1, "bad table index");
    const auto& T = t->t[i];
    o->k = T.k;
    o->nkeys = T.keys.size();
    o->keys = T.keys.data();
    o->offs = T.offs.data();
    o->tids = T.tids.data();
    return 0;
}

int skq_tables_free(skq_tables* t) {
    delete t;
    return 0;
}

int skq_index_from_tables(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks, const skq_tables* t,
                          skq_index** out) {
    if (!t) return hfail(-1, "null tables");
    std::vector<skq_kmer_table> v(t->t.size());
    for (uint32_t i = 0; i < v.size(); ++i) skq_tables_get(t, i, &v[i]);
    return skq_index_create(device, ntx, nk, ks, (uint32_t)v.size(), v.data(), out);
}

int skq_index_from_tables_chained(int device, uint32_t ntx, uint32_t nk, const uint32_t* ks, const skq_tables* t,
                                  const skq_seqs* tx, uint32_t threshold, skq_index** out) {
    if (!t) return hfail(-1, "null tables");
    std::vector<skq_kmer_table> v(t->t.size());
    for (uint32_t i = 0; i < v.size(); ++i) skq_tables_get(t, i, &v[i]);
    const uint8_t* bytes = nullptr;
    const uint64_t* offs = nullptr;
    const uint64_t n = tx ? skq_seqs_count(tx) : 0;
    if (tx) skq_seqs_view(tx, &bytes, &offs, nullptr, nullptr);
    if (!tx || n == 0 || offs[n] == 0)  // (no sequences: nothing to chain)
        return skq_index_create(device, ntx, nk, ks, (uint32_t)v.size(), v.data(), out);
    return skq_index_create_chained(device, ntx, nk, ks, (uint32_t)v.size(), v.data(), bytes, offs, (uint32_t)n,
                                    threshold, out);
}

}  // extern "C"
