// skq_io.cpp — host pieces around the hot path, with the reference's record rules:
//   FASTA loading (load_fasta, src/data_io.cpp:47-80), a streaming FASTQ reader over mmap
//   (process_fastq_single_pass's reader, src/main.cpp:113-148), the legacy binary index
//   (save_index / load_index, src/data_io.cpp:165-304), EM + assignment
//   (src/isoform_assignment.cpp:9-97) and the CSV writer (src/data_io.cpp:133-152).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "skq_host.h"
#include "skq_internal.h"

namespace {

int fail(int code, const std::string& msg) { return skq::set_error(code, msg.c_str()); }

bool valid_acgt(std::string_view s) {
    for (unsigned char c : s)
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T') return false;
    return true;
}

// read-only mapping of a whole file
struct MappedFile {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    int open(const char* path) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) return fail(-4, std::string("could not open ") + path);
        struct stat st {};
        if (fstat(fd, &st) != 0) return fail(-4, std::string("could not stat ") + path);
        n = (size_t)st.st_size;
        if (n) {
            void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m == MAP_FAILED) return fail(-4, std::string("could not map ") + path);
            madvise(m, n, MADV_SEQUENTIAL);
            p = static_cast<const char*>(m);
        }
        return 0;
    }
    ~MappedFile() {
        if (p) munmap(const_cast<char*>(p), n);
        if (fd >= 0) ::close(fd);
    }
};

// std::getline on the mapping: the line at *pos (without '\n'); false at end of data
bool next_line(const char* p, size_t n, size_t& pos, std::string_view& line) {
    if (pos >= n) return false;
    const void* nl = memchr(p + pos, '\n', n - pos);
    const size_t end = nl ? (size_t)(static_cast<const char*>(nl) - p) : n;
    line = std::string_view(p + pos, end - pos);
    pos = nl ? end + 1 : n;
    return true;
}

}  // namespace

// ---- sequences (FASTA) ----------------------------------------------------------------------

struct skq_seqs {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs{0};
    std::vector<char> names;
    std::vector<uint64_t> name_offs{0};
    void add(std::string_view name, std::string_view seq) {
        names.insert(names.end(), name.begin(), name.end());
        name_offs.push_back(names.size());
        bytes.insert(bytes.end(), seq.begin(), seq.end());
        offs.push_back(bytes.size());
    }
};

extern "C" {

int skq_fasta_load(const char* path, skq_seqs** out) {
    if (!path || !out) return fail(-1, "null argument");
    *out = nullptr;
    MappedFile f;
    if (int rc = f.open(path)) return rc;
    auto* s = new skq_seqs();
    std::unordered_map<std::string, bool> seen;  // first occurrence of an id wins (emplace)
    std::string id, seq;
    bool have = false;
    auto flush = [&](bool last) {
        // every record but the last is kept only if valid (src/data_io.cpp:62-64, :73-75)
        if (!have || (!last && !valid_acgt(seq))) return;
        if (seen.emplace(id, true).second) s->add(id, seq);
    };
    size_t pos = 0;
    std::string_view line;
    while (next_line(f.p, f.n, pos, line)) {
        if (line.empty()) continue;
        if (line[0] == '>') {
            flush(false);
            // the id ends at the first space (substr(1, find(' ') - 1))
            const size_t sp = line.find(' ');
            id.assign(line.substr(1, sp == std::string_view::npos ? std::string_view::npos : sp - 1));
            seq.clear();
            have = !id.empty();
        } else {
            seq.append(line.data(), line.size());
        }
    }
    flush(true);
    *out = s;
    return 0;
}

uint64_t skq_seqs_count(const skq_seqs* s) { return s ? s->offs.size() - 1 : 0; }

int skq_seqs_view(const skq_seqs* s, const uint8_t** seq_bytes, const uint64_t** seq_offs, const char** name_bytes,
                  const uint64_t** name_offs) {
    if (!s) return fail(-1, "null sequences");
    if (seq_bytes) *seq_bytes = s->bytes.data();
    if (seq_offs) *seq_offs = s->offs.data();
    if (name_bytes) *name_bytes = s->names.data();
    if (name_offs) *name_offs = s->name_offs.data();
    return 0;
}

int skq_seqs_free(skq_seqs* s) {
    delete s;
    return 0;
}

}  // extern "C"

// ---- FASTQ ----------------------------------------------------------------------------------

struct skq_fastq {
    MappedFile f;
    size_t pos = 0;
    uint64_t records = 0;
    std::vector<uint64_t> id_at;   // per record: offset of the id in the mapping
    std::vector<uint32_t> id_len;
    std::vector<uint8_t> batch;    // bases of the current batch, contiguous
    std::vector<uint64_t> offs;
    std::unordered_map<std::string_view, uint64_t> last_ok;  // id -> last record marked OK
};

extern "C" {

// the record machine over the lines of t[a, b) (a and b line starts) from state s
// (src/main.cpp:119-129: between records a line starting with '@' opens one, any other line is
// skipped; the sequence, '+' and quality lines are taken whatever they hold)
static uint32_t fastq_run(const char* t, uint64_t a, uint64_t b, uint32_t s) {
    while (a < b) {
        s = s == 0 ? (t[a] == '@' ? 1u : 0u) : (s + 1) & 3u;
        const void* nl = std::memchr(t + a, '\n', (size_t)(b - a));
        a = nl ? (uint64_t)(static_cast<const char*>(nl) - t) + 1 : b;
    }
    return s;
}

int skq_fastq_split(const char* path, uint32_t parts, uint64_t* offs, uint32_t* states) {
    if (!path || !offs || !states || parts == 0) return skq::set_error(-1, "null argument or no parts");
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return skq::set_error(-2, (std::string("Could not open FASTQ file: ") + path).c_str());
    struct stat st {};
    if (fstat(fd, &st) != 0) {
        ::close(fd);
        return skq::set_error(-2, "Could not stat FASTQ file");
    }
    const uint64_t n = (uint64_t)st.st_size;
    const char* t = nullptr;
    if (n) {
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            ::close(fd);
            return skq::set_error(-2, "FASTQ mmap failed");
        }
        t = static_cast<const char*>(m);
    }
    auto line_start_at_or_after = [&](uint64_t x) -> uint64_t {
        if (x == 0 || x >= n) return std::min(x, n);
        const void* nl = std::memchr(t + x - 1, '\n', (size_t)(n - x + 1));
        return nl ? (uint64_t)(static_cast<const char*>(nl) - t) + 1 : n;
    };
    offs[0] = 0;
    states[0] = 0;
    for (uint32_t p = 1; p < parts; ++p) {
        uint64_t b = line_start_at_or_after(n / parts * p);
        b = std::max(b, offs[p - 1]);
        offs[p] = b;
        // the state at b: from a line start W bytes back, all four states run forward; when they
        // agree at b that is the state whatever it was there; else go back further (from the file
        // start the state is exactly 0)
        uint32_t s = 0;
        for (uint64_t W = 1 << 12;; W <<= 2) {
            if (W >= b) {
                s = fastq_run(t, 0, b, 0);
                break;
            }
            const uint64_t a = line_start_at_or_after(b - W);
            const uint32_t s0 = fastq_run(t, a, b, 0);
            if (fastq_run(t, a, b, 1) == s0 && fastq_run(t, a, b, 2) == s0 && fastq_run(t, a, b, 3) == s0) {
                s = s0;
                break;
            }
        }
        states[p] = s;
    }
    offs[parts] = n;
    if (t) munmap(const_cast<char*>(t), n);
    ::close(fd);
    return 0;
}

int skq_fastq_open(const char* path, skq_fastq** out) {
    if (!path || !out) return fail(-1, "null argument");
    *out = nullptr;
    auto* q = new skq_fastq();
    if (int rc = q->f.open(path)) {
        delete q;
        return rc;
    }
    *out = q;
    return 0;
}

// Records as std::getline sees them (src/main.cpp:120-129): a line starting with '@' opens a
// record whose id is the rest of that line; the next line is the sequence, then '+' and the
// quality line. Lines that do not start with '@' between records are skipped. No filtering here:
// the sketch kernel marks invalid and short reads (status), and skq_fastq_mark / skq_fastq_kept
// apply "the last valid record of an id wins" (src/main.cpp:147).
int skq_fastq_next(skq_fastq* q, uint64_t max_reads, uint64_t* n, const uint8_t** bytes, const uint64_t** offs,
                   uint64_t* first_ordinal) {
    if (!q || !n) return fail(-1, "null argument");
    q->batch.clear();
    q->offs.assign(1, 0);
    if (first_ordinal) *first_ordinal = q->records;
    uint64_t got = 0;
    std::string_view line, seq, skip;
    while (got < max_reads && next_line(q->f.p, q->f.n, q->pos, line)) {
        if (line.empty() || line[0] != '@') continue;
        if (!next_line(q->f.p, q->f.n, q->pos, seq)) seq = std::string_view();
        next_line(q->f.p, q->f.n, q->pos, skip);  // '+'
        next_line(q->f.p, q->f.n, q->pos, skip);  // quality
        q->id_at.push_back((uint64_t)(line.data() + 1 - q->f.p));
        q->id_len.push_back((uint32_t)(line.size() - 1));
        q->batch.insert(q->batch.end(), seq.begin(), seq.end());
        q->offs.push_back(q->batch.size());
        ++q->records;
        ++got;
    }
    *n = got;
    if (bytes) *bytes = q->batch.data();
    if (offs) *offs = q->offs.data();
    return 0;
}

// status[i] of records first .. first + n - 1 (SKQ_READ_OK = kept by the reference's filter)
int skq_fastq_mark(skq_fastq* q, uint64_t first, uint64_t n, const uint8_t* status) {
    if (!q || (n && !status)) return fail(-1, "null argument");
    if (first + n > q->records) return fail(-1, "records out of range");
    for (uint64_t i = 0; i < n; ++i) {
        if ((status[i] & SKQ_STATUS_MASK) != SKQ_READ_OK) continue;
        const uint64_t r = first + i;
        q->last_ok[std::string_view(q->f.p + q->id_at[r], q->id_len[r])] = r;
    }
    return 0;
}

// 1 if record `ordinal` is the one kept for its id (the last record marked OK), else 0
int skq_fastq_kept(const skq_fastq* q, uint64_t ordinal) {
    if (!q || ordinal >= q->records) return 0;
    auto it = q->last_ok.find(std::string_view(q->f.p + q->id_at[ordinal], q->id_len[ordinal]));
    return it != q->last_ok.end() && it->second == ordinal ? 1 : 0;
}

uint64_t skq_fastq_records(const skq_fastq* q) { return q ? q->records : 0; }

int skq_fastq_id(const skq_fastq* q, uint64_t ordinal, const char** id, uint64_t* len) {
    if (!q || ordinal >= q->records) return fail(-1, "record out of range");
    if (id) *id = q->f.p + q->id_at[ordinal];
    if (len) *len = q->id_len[ordinal];
    return 0;
}

int skq_fastq_close(skq_fastq* q) {
    delete q;
    return 0;
}

}  // extern "C"

// ---- legacy index (src/data_io.cpp:165-304) ---------------------------------------------------

namespace {

struct Writer {
    FILE* f;
    bool ok = true;
    void raw(const void* p, size_t n) { ok &= fwrite(p, 1, n, f) == n; }
    void u64(uint64_t v) { raw(&v, 8); }
    void u32(uint32_t v) { raw(&v, 4); }
    void str(const char* p, uint64_t n) {
        u64(n);
        raw(p, n);
    }
};

struct Reader {
    const char* p;
    size_t n, at = 0;
    bool ok = true;
    bool raw(void* dst, size_t k) {
        if (!ok || at + k > n) return ok = false;
        memcpy(dst, p + at, k);
        at += k;
        return true;
    }
    uint64_t u64() {
        uint64_t v = 0;
        raw(&v, 8);
        return v;
    }
    uint32_t u32() {
        uint32_t v = 0;
        raw(&v, 4);
        return v;
    }
    std::string_view str() {
        const uint64_t k = u64();
        if (!ok || at + k > n) {
            ok = false;
            return {};
        }
        std::string_view s(p + at, k);
        at += k;
        return s;
    }
};

}  // namespace

struct skq_legacy_index {
    std::vector<uint32_t> ks;  // as saved (CLI order)
    skq_seqs tx;               // transcripts in file order
    skq_tables* tables = nullptr;
    ~skq_legacy_index() { skq_tables_free(tables); }
};

extern "C" {

// Writes the reference's format: k list; every transcript (id, sequence, length field 0 — the
// reference's load_fasta leaves length 0); then per distinct k the key -> transcript-id lists.
// Keys ascending and ids in table order (the reference writes unordered_map order: the bytes
// differ, the content is the same).
int skq_legacy_index_write(const char* path, uint32_t nk, const uint32_t* ks, const skq_seqs* tx,
                           const skq_tables* tables) {
    if (!path || !tx || !tables || (nk && !ks)) return fail(-1, "null argument");
    FILE* f = fopen(path, "wb");
    if (!f) return fail(-4, std::string("could not open for writing: ") + path);
    Writer w{f};
    w.u64(nk);
    for (uint32_t i = 0; i < nk; ++i) w.u32(ks[i]);
    const uint64_t ntx = skq_seqs_count(tx);
    w.u64(ntx);
    for (uint64_t t = 0; t < ntx; ++t) {
        w.str(tx->names.data() + tx->name_offs[t], tx->name_offs[t + 1] - tx->name_offs[t]);
        w.str(reinterpret_cast<const char*>(tx->bytes.data()) + tx->offs[t], tx->offs[t + 1] - tx->offs[t]);
        w.u32(0);
    }
    const uint32_t nt = skq_tables_count(tables);
    w.u64(nt);
    for (uint32_t i = 0; i < nt; ++i) {
        skq_kmer_table v{};
        skq_tables_get(tables, i, &v);
        w.u32(v.k);
        w.u64(v.nkeys);
        for (uint64_t j = 0; j < v.nkeys; ++j) {
            w.u32(v.keys[j]);
            w.u64(v.offs[j + 1] - v.offs[j]);
            for (uint64_t q = v.offs[j]; q < v.offs[j + 1]; ++q) {
                const uint32_t t = v.tids[q];
                w.str(tx->names.data() + tx->name_offs[t], tx->name_offs[t + 1] - tx->name_offs[t]);
            }
        }
    }
    const bool ok = w.ok && fclose(f) == 0;
    return ok ? 0 : fail(-4, std::string("write failed: ") + path);
}

// ---- compact sidecar -----------------------------------------------
// `<legacy>.skq`, written by `index` next to the reference's file: the same content in CSR form
// (k list, transcript names, per distinct k keys / offsets / dense ids; no sequences, which
// quant does not use), stamped with the legacy file's size and mtime. skq_index_open loads it
// with a few large copies instead of parsing 1.3 GB of length-prefixed strings, and falls back
// to the legacy file whenever the stamp does not match.
namespace {

constexpr char kSidecarMagic[8] = {'S', 'K', 'Q', 'I', 'D', 'X', '0', '2'};  // 02: with sequences

std::string sidecar_path(const char* legacy) { return std::string(legacy) + ".skq"; }

bool file_stamp(const char* path, uint64_t& size, int64_t& mtime_ns) {
    struct stat st {};
    if (stat(path, &st) != 0) return false;
    size = (uint64_t)st.st_size;
    mtime_ns = (int64_t)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec;
    return true;
}

}  // namespace

extern "C" {

int skq_sidecar_write(const char* legacy_path, uint32_t nk, const uint32_t* ks, const skq_seqs* tx,
                      const skq_tables* tables) {
    if (!legacy_path || !tx || !tables || (nk && !ks)) return fail(-1, "null argument");
    uint64_t lsize = 0;
    int64_t lmtime = 0;
    if (!file_stamp(legacy_path, lsize, lmtime)) return fail(-4, std::string("no legacy index at ") + legacy_path);
    const std::string out = sidecar_path(legacy_path);
    const std::string tmp = out + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return fail(-4, std::string("could not open for writing: ") + tmp);
    Writer w{f};
    w.raw(kSidecarMagic, 8);
    w.u64(lsize);
    w.u64((uint64_t)lmtime);
    w.u64(nk);
    for (uint32_t i = 0; i < nk; ++i) w.u32(ks[i]);
    const uint64_t ntx = skq_seqs_count(tx);
    w.u64(ntx);
    w.u64(tx->names.size());
    w.raw(tx->names.data(), tx->names.size());
    w.raw(tx->name_offs.data(), (ntx + 1) * 8);
    // the sequences (quant's chained tables follow the transcripts: skq_index_create_chained)
    w.u64(tx->bytes.size());
    w.raw(tx->bytes.data(), tx->bytes.size());
    w.raw(tx->offs.data(), (ntx + 1) * 8);
    const uint32_t nt = skq_tables_count(tables);
    w.u64(nt);
    for (uint32_t i = 0; i < nt; ++i) {
        skq_kmer_table v{};
        skq_tables_get(tables, i, &v);
        w.u32(v.k);
        w.u64(v.nkeys);
        w.u64(v.offs[v.nkeys]);
        w.raw(v.keys, v.nkeys * 4);
        w.raw(v.offs, (v.nkeys + 1) * 8);
        w.raw(v.tids, v.offs[v.nkeys] * 4);
    }
    const bool ok = w.ok && fclose(f) == 0 && rename(tmp.c_str(), out.c_str()) == 0;
    if (!ok) std::remove(tmp.c_str());
    return ok ? 0 : fail(-4, std::string("write failed: ") + out);
}

}  // extern "C"

// Reads the format back: dense transcript ids follow the transcripts' order in the file; a
// posting naming a transcript that is not in the file gets a new id past them (name kept).
int skq_legacy_index_read(const char* path, skq_legacy_index** out) {
    if (!path || !out) return fail(-1, "null argument");
    *out = nullptr;
    MappedFile f;
    if (int rc = f.open(path)) return rc;
    Reader r{f.p, f.n};
    auto* ix = new skq_legacy_index();
    const uint64_t nk = r.u64();
    if (nk > SKQ_MAX_K * 64ull) r.ok = false;
    for (uint64_t i = 0; r.ok && i < nk; ++i) ix->ks.push_back(r.u32());
    const uint64_t ntx = r.u64();
    std::unordered_map<std::string_view, uint32_t> id;
    for (uint64_t t = 0; r.ok && t < ntx; ++t) {
        const std::string_view name = r.str();
        const std::string_view seq = r.str();
        (void)r.u32();  // length field
        if (!r.ok) break;
        if (id.emplace(name, (uint32_t)skq_seqs_count(&ix->tx)).second) ix->tx.add(name, seq);
    }
    // postings: one sequential walk records where each posting's name is (cheap: lengths only);
    // the name -> id lookups then run on all cores (the map is only read), and the rare names
    // that are not transcripts of the file get ids afterwards, in file order
    const uint64_t nmaps = r.u64();
    std::vector<uint32_t> tks;
    std::vector<std::vector<uint64_t>> words;  // per map: (key << 32 | tid)
    std::vector<std::vector<uint64_t>> at;     // per map: file offset of each posting's name
    for (uint64_t m = 0; r.ok && m < nmaps; ++m) {
        tks.push_back(r.u32());
        words.emplace_back();
        at.emplace_back();
        const uint64_t nkeys = r.u64();
        for (uint64_t j = 0; r.ok && j < nkeys; ++j) {
            const uint32_t key = r.u32();
            const uint64_t np = r.u64();
            for (uint64_t q = 0; r.ok && q < np; ++q) {
                at.back().push_back(r.at);
                (void)r.str();
                words.back().push_back((uint64_t)key << 32);
            }
        }
    }
    if (r.ok) {
        const int P = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        for (size_t m = 0; m < words.size(); ++m) {
            std::vector<uint64_t>& wv = words[m];
            const std::vector<uint64_t>& av = at[m];
            const uint64_t n = wv.size();
            auto resolve = [&](uint64_t lo, uint64_t hi) {
                for (uint64_t i = lo; i < hi; ++i) {
                    Reader q{f.p, f.n, (size_t)av[i]};
                    auto it = id.find(q.str());
                    wv[i] |= it == id.end() ? 0xFFFFFFFFull : (uint64_t)it->second;
                }
            };
            if (n < (1u << 16) || P == 1) {
                resolve(0, n);
            } else {
                std::vector<std::thread> pool;
                for (int w = 0; w < P; ++w) pool.emplace_back(resolve, n * w / P, n * (w + 1) / P);
                for (auto& t : pool) t.join();
            }
            for (uint64_t i = 0; i < n; ++i) {
                if ((uint32_t)wv[i] != 0xFFFFFFFFu) continue;
                Reader q{f.p, f.n, (size_t)av[i]};
                const std::string_view name = q.str();
                auto it = id.find(name);
                uint32_t t;
                if (it == id.end()) {  // keep unknown names addressable
                    t = (uint32_t)skq_seqs_count(&ix->tx);
                    ix->tx.add(name, std::string_view());
                    id.emplace(name, t);  // (a view into the mapping: stable while it lives)
                } else {
                    t = it->second;
                }
                wv[i] = (wv[i] & ~0xFFFFFFFFull) | t;
            }
        }
    }
    if (!r.ok) {
        delete ix;
        return fail(-5, std::string("truncated or malformed index: ") + path);
    }
    at.clear();
    if (int rc = skq::tables_from_words((uint32_t)tks.size(), tks.data(), words.data(), &ix->tables)) {
        delete ix;
        return rc;
    }
    *out = ix;
    return 0;
}

int skq_legacy_index_view(const skq_legacy_index* ix, uint32_t* nk, const uint32_t** ks, const skq_seqs** tx,
                          const skq_tables** tables) {
    if (!ix) return fail(-1, "null index");
    if (nk) *nk = (uint32_t)ix->ks.size();
    if (ks) *ks = ix->ks.data();
    if (tx) *tx = &ix->tx;
    if (tables) *tables = ix->tables;
    return 0;
}

int skq_legacy_index_free(skq_legacy_index* ix) {
    delete ix;
    return 0;
}

// quant's loader: the sidecar when its stamp matches the legacy file, else the legacy file
int skq_index_open(const char* path, skq_legacy_index** out, int* from_sidecar) {
    if (!path || !out) return fail(-1, "null argument");
    *out = nullptr;
    if (from_sidecar) *from_sidecar = 0;
    uint64_t lsize = 0;
    int64_t lmtime = 0;
    const std::string sp = sidecar_path(path);
    if (file_stamp(path, lsize, lmtime) && access(sp.c_str(), R_OK) == 0) {
        MappedFile f;
        if (f.open(sp.c_str()) == 0) {
            Reader r{f.p, f.n};
            char magic[8] = {};
            r.raw(magic, 8);
            const uint64_t sz = r.u64(), mt = r.u64();
            if (r.ok && !std::memcmp(magic, kSidecarMagic, 8) && sz == lsize && (int64_t)mt == lmtime) {
                auto* ix = new skq_legacy_index();
                const uint64_t nk = r.u64();
                if (nk > SKQ_MAX_K * 64ull) r.ok = false;
                for (uint64_t i = 0; r.ok && i < nk; ++i) ix->ks.push_back(r.u32());
                const uint64_t ntx = r.u64(), nb = r.u64();
                if (r.ok && nb <= f.n && ntx < f.n) {
                    ix->tx.names.resize(nb);
                    r.raw(ix->tx.names.data(), nb);
                    ix->tx.name_offs.resize(ntx + 1);
                    r.raw(ix->tx.name_offs.data(), (ntx + 1) * 8);
                    const uint64_t sb = r.u64();
                    if (r.ok && sb <= f.n) {
                        ix->tx.bytes.resize(sb);
                        r.raw(ix->tx.bytes.data(), sb);
                        ix->tx.offs.resize(ntx + 1);
                        r.raw(ix->tx.offs.data(), (ntx + 1) * 8);
                        r.ok = r.ok && ix->tx.offs[0] == 0 && ix->tx.offs[ntx] == sb;
                        // (never decreasing: the chained tables' builder sketches offs[u] .. offs[u+1])
                        for (uint32_t u = 0; r.ok && u < ntx; ++u) r.ok = ix->tx.offs[u] <= ix->tx.offs[u + 1];
                    } else {
                        r.ok = false;
                    }
                } else {
                    r.ok = false;
                }
                const uint64_t nt = r.u64();
                if (nt > SKQ_MAX_K * 64ull) r.ok = false;
                std::vector<uint32_t> tks;
                std::vector<std::vector<uint32_t>> K, T;
                std::vector<std::vector<uint64_t>> O;
                for (uint64_t i = 0; r.ok && i < nt; ++i) {
                    tks.push_back(r.u32());
                    const uint64_t nkeys = r.u64(), np = r.u64();
                    if (!r.ok || nkeys > f.n || np > f.n) {
                        r.ok = false;
                        break;
                    }
                    std::vector<uint32_t> keys(nkeys), tids(np);
                    std::vector<uint64_t> offs(nkeys + 1);
                    r.raw(keys.data(), nkeys * 4);
                    r.raw(offs.data(), (nkeys + 1) * 8);
                    r.raw(tids.data(), np * 4);
                    bool mono = r.ok && offs[0] == 0 && offs[nkeys] == np;
                    for (uint64_t j = 0; mono && j < nkeys; ++j) mono = offs[j] <= offs[j + 1];
                    if (!mono) {
                        r.ok = false;
                        break;
                    }
                    K.push_back(std::move(keys));
                    O.push_back(std::move(offs));
                    T.push_back(std::move(tids));
                }
                if (r.ok && skq::tables_from_csr((uint32_t)tks.size(), tks.data(), K.data(), O.data(), T.data(),
                                                 &ix->tables) == 0) {
                    *out = ix;
                    if (from_sidecar) *from_sidecar = 1;
                    return 0;
                }
                delete ix;
            }
        }
    }
    return skq_legacy_index_read(path, out);
}

// ---- EM, assignment (src/isoform_assignment.cpp:9-97), CSV (src/data_io.cpp:133-152) ---------

int skq_em(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid, const uint32_t* cand_score,
           uint32_t ntx, int max_iterations, double convergence, int nthreads, double* pi, int* iterations) {
    if (!pi || (nreads && (!cand_offs || !cand_tid || !cand_score))) return fail(-1, "null argument");
    if (ntx == 0) return 0;
    for (uint32_t t = 0; t < ntx; ++t) pi[t] = 1.0 / ntx;  // uniform start (:17-20)
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
    nthreads = (int)std::min<uint64_t>((uint64_t)nthreads, std::max<uint64_t>(1, nreads / 65536 + 1));
    std::vector<std::vector<double>> part(nthreads, std::vector<double>(ntx));
    const double probability_epsilon = 1e-10;  // (:30)
    // the pseudocount is a float (:55-58): (posterior + 0.01f / R) + 0.01f
    const float pseudocount = 0.01f;
    const float pc_per_read = pseudocount / (float)nreads;  // (R = 0: inf, as the reference)
    int it = 0;
    for (; it < max_iterations; ++it) {
        auto estep = [&](int w) {
            std::vector<double>& acc = part[w];
            std::fill(acc.begin(), acc.end(), 0.0);
            const uint64_t a = nreads * w / nthreads, b = nreads * (w + 1) / nthreads;
            for (uint64_t r = a; r < b; ++r) {
                double den = 0.0;
                for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c) den += pi[cand_tid[c]] * (double)cand_score[c];
                if (den > probability_epsilon) {
                    const double inv = 1.0 / den;
                    for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c)
                        acc[cand_tid[c]] += pi[cand_tid[c]] * (double)cand_score[c] * inv;
                }
            }
        };
        std::vector<std::thread> pool;
        for (int w = 1; w < nthreads; ++w) pool.emplace_back(estep, w);
        estep(0);
        for (auto& th : pool) th.join();
        double change = 0.0;  // M-step (:53-62)
        for (uint32_t t = 0; t < ntx; ++t) {
            double post = 0.0;
            for (int w = 0; w < nthreads; ++w) post += part[w][t];
            const double np = post + (double)pc_per_read + (double)pseudocount;
            change += std::fabs(np - pi[t]);
            pi[t] = np;
        }
        if (change < convergence) {
            ++it;
            break;
        }
    }
    if (iterations) *iterations = it;
    return 0;
}

// One E-step on the host (the reads' posterior sums, read order): the CPU side of the multi-rank
// EM loop (skq/dist.py), used where there is no GPU (gloo tests).
int skq_em_estep_host(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
                      const uint32_t* cand_score, uint32_t ntx, const double* pi, int nthreads, double* post) {
    (void)nthreads;
    if (!pi || !post || (nreads && (!cand_offs || !cand_tid || !cand_score))) return fail(-1, "null argument");
    std::fill(post, post + ntx, 0.0);
    for (uint64_t r = 0; r < nreads; ++r) {
        double den = 0.0;
        for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c) {
            if (cand_tid[c] >= ntx) return fail(-1, "candidate transcript id out of range");
            den += pi[cand_tid[c]] * (double)cand_score[c];
        }
        if (den > 1e-10) {
            const double inv = 1.0 / den;
            for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c)
                post[cand_tid[c]] += pi[cand_tid[c]] * (double)cand_score[c] * inv;
        }
    }
    return 0;
}

// The M-step (src/isoform_assignment.cpp:53-60) on host arrays; returns sum |new - old| in *change.
int skq_em_mstep_host(uint32_t ntx, double* pi, const double* post, uint64_t total_reads, double* change) {
    if (!pi || !post || !change) return fail(-1, "null argument");
    const float pc = 0.01f;
    const double a = (double)(pc / (float)total_reads), b = (double)pc;  // (R = 0: inf, as the reference)
    double ch = 0.0;
    for (uint32_t t = 0; t < ntx; ++t) {
        const double np = post[t] + a + b;
        ch += std::fabs(np - pi[t]);
        pi[t] = np;
    }
    *change = ch;
    return 0;
}

int skq_assign(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid, const uint32_t* cand_score,
               uint32_t ntx, const double* pi, double* counts, uint8_t* assigned) {
    if (!pi || !counts || (nreads && (!cand_offs || !cand_tid || !cand_score))) return fail(-1, "null argument");
    std::fill(counts, counts + ntx, 0.0);
    if (assigned) std::fill(assigned, assigned + ntx, 0);
    for (uint64_t r = 0; r < nreads; ++r) {
        double total = 0.0;
        for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c) total += pi[cand_tid[c]] * cand_score[c];
        if (!(total > 0.0)) continue;
        for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c) {
            counts[cand_tid[c]] += (pi[cand_tid[c]] * cand_score[c]) / total;
            if (assigned) assigned[cand_tid[c]] = 1;
        }
    }
    return 0;
}

// "Name,NumReads,EM_Abundance" then one row per transcript that received reads, values as a
// default std::ostream prints a double (6 significant digits, %g)
int skq_csv_write(const char* path, const skq_seqs* tx, const double* counts, const uint8_t* assigned,
                  const double* pi) {
    if (!path || !tx || !counts || !assigned || !pi) return fail(-1, "null argument");
    FILE* f = fopen(path, "w");
    if (!f) return fail(-4, std::string("Could not open file for writing: ") + path);
    fputs("Name,NumReads,EM_Abundance\n", f);
    const uint64_t n = skq_seqs_count(tx);
    for (uint64_t t = 0; t < n; ++t) {
        if (!assigned[t]) continue;
        fwrite(tx->names.data() + tx->name_offs[t], 1, tx->name_offs[t + 1] - tx->name_offs[t], f);
        fprintf(f, ",%g,%g\n", counts[t], pi[t]);
    }
    return fclose(f) == 0 ? 0 : fail(-4, std::string("write failed: ") + path);
}

}  // extern "C"
