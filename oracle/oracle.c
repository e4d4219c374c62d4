/*
 * oracle.c — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Written for clarity, not speed: full 64-bit ntHash state (the product kernels use only the
 * 33-bit lane), sorted pair arrays + binary search for the index, qsort-based counting.
 * Every function cites the reference file:line it restates.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- ntHash (third party, bcgsc ntHash >= 2.3) ----------------------------------------- */
uint64_t orc_seed(unsigned char c) {
    switch (c) {
    case 'A': case 'a': return 0x3c8bfbb395c60474ULL;
    case 'C': case 'c': return 0x3193c18562a02b4cULL;
    case 'G': case 'g': return 0x20323ed082572324ULL;
    case 'T': case 't': case 'U': case 'u': return 0x295549f54be24456ULL;
    default: return 0; /* SEED_N: base is skipped */
    }
}

uint64_t orc_srol(uint64_t x) {
    uint64_t wrap = ((x & 0x8000000000000000ULL) >> 30) | ((x & 0x100000000ULL) >> 32);
    return ((x << 1) & 0xFFFFFFFDFFFFFFFFULL) | wrap;
}

static uint64_t srol_n(uint64_t x, unsigned d) {
    while (d--) x = orc_srol(x);
    return x;
}

/* NtHash(seq, 1, k) then `while (roll()) get_forward_hash()` as called at src/sketch.cpp:31-33
 * and src/kmer.cpp:26-30. init() skips past the last invalid base of the window; roll() with an
 * invalid incoming base jumps pos += k and re-inits. */
size_t orc_nthash_fwd(const char* seq, size_t len, unsigned k, uint64_t* out_hash, size_t* out_pos) {
    if (k == 0 || len < k) return (size_t)-1;
    /* srol^k(SEED[c]) of the outgoing base, for the four distinct non-zero seeds (the roll's
     * third term), computed once per call instead of k rotations per window */
    static const unsigned char acgt[4] = {'A', 'C', 'G', 'T'};
    uint64_t seed4[4], rolk4[4];
    for (int b = 0; b < 4; ++b) {
        seed4[b] = orc_seed(acgt[b]);
        rolk4[b] = srol_n(seed4[b], k);
    }
    size_t pos = 0, n = 0;
    int initialized = 0;
    uint64_t fwd = 0;
    for (;;) {
        int need_init = !initialized;
        if (initialized) {
            if (pos >= len - k) break;
            if (orc_seed((unsigned char)seq[pos + k]) == 0) {
                pos += k;
                need_init = 1;
            } else {
                const uint64_t so = orc_seed((unsigned char)seq[pos]);
                uint64_t rk = 0;
                for (int b = 0; b < 4; ++b)
                    if (so == seed4[b]) rk = rolk4[b]; /* = srol_n(so, k) */
                fwd = orc_srol(fwd) ^ orc_seed((unsigned char)seq[pos + k]) ^ rk;
                ++pos;
            }
        }
        if (need_init) {
            for (;;) {
                if (pos > len - k) break;
                long bad = -1;
                for (long i = (long)k - 1; i >= 0; --i)
                    if (orc_seed((unsigned char)seq[pos + i]) == 0) { bad = i; break; }
                if (bad < 0) break;
                pos += (size_t)bad + 1;
            }
            if (pos > len - k) break;
            fwd = 0;
            for (unsigned i = 0; i < k; ++i) fwd = orc_srol(fwd) ^ orc_seed((unsigned char)seq[pos + i]);
            initialized = 1;
        }
        if (out_hash) out_hash[n] = fwd;
        if (out_pos) out_pos[n] = pos;
        ++n;
    }
    return n;
}

/* src/sketch.cpp:25-26 — the caller passes (double)0.05f from src/main.cpp:43,110 */
uint32_t orc_threshold(double fraction) {
    const uint32_t H = 0xFFFFFFFFu;
    return (uint32_t)(H * fraction);
}

/* src/data_io.cpp:17-34 */
int orc_is_valid_sequence(const char* seq, size_t len) {
    for (size_t i = 0; i < len; ++i) {
        char c = seq[i];
        if (c != 'A' && c != 'T' && c != 'C' && c != 'G') return 0;
    }
    return 1;
}

static int cmp_u32(const void* a, const void* b) {
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

static size_t sort_unique_u32(uint32_t* v, size_t n) {
    if (n == 0) return 0;
    if (n <= 32) { /* insertion sort: a read's retained set is a handful of values */
        for (size_t i = 1; i < n; ++i) {
            uint32_t x = v[i];
            size_t j = i;
            for (; j > 0 && v[j - 1] > x; --j) v[j] = v[j - 1];
            v[j] = x;
        }
    } else {
        qsort(v, n, sizeof(uint32_t), cmp_u32);
    }
    size_t m = 1;
    for (size_t i = 1; i < n; ++i)
        if (v[i] != v[m - 1]) v[m++] = v[i];
    return m;
}

static size_t hashes_filtered(const char* seq, size_t len, unsigned k, uint64_t thr, uint32_t* out) {
    if (k == 0 || len < k) return (size_t)-1;
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * (len - k + 1));
    size_t n = orc_nthash_fwd(seq, len, k, h, NULL), m = 0;
    for (size_t i = 0; i < n; ++i) {
        uint32_t v = (uint32_t)h[i]; /* uint32_t hash_value = nth.get_forward_hash(); */
        if ((uint64_t)v <= thr) out[m++] = v;
    }
    free(h);
    return sort_unique_u32(out, m);
}

/* src/sketch.cpp:24-39 */
size_t orc_sketch(const char* seq, size_t len, unsigned k, uint32_t threshold, uint32_t* out) {
    return hashes_filtered(seq, len, k, threshold, out);
}

/* src/kmer.cpp:19-35 */
size_t orc_all_hashes(const char* seq, size_t len, unsigned k, uint32_t* out) {
    return hashes_filtered(seq, len, k, 0xFFFFFFFFull, out);
}

/* ---- inverted index (src/sketch.cpp:51-74) --------------------------------------------- */
typedef struct { uint32_t hash, tid; } pair_t;

struct orc_index {
    unsigned nk;
    unsigned ks[64];
    uint32_t ntx;
    uint64_t npairs[64];
    pair_t* pairs[64]; /* sorted by (hash, tid), unique */
    uint64_t nkeys[64];
};

static int cmp_pair(const void* a, const void* b) {
    const pair_t* x = (const pair_t*)a;
    const pair_t* y = (const pair_t*)b;
    if (x->hash != y->hash) return x->hash < y->hash ? -1 : 1;
    return x->tid < y->tid ? -1 : x->tid > y->tid;
}

static void finalize_k(orc_index* ix, unsigned i) {
    pair_t* p = ix->pairs[i];
    uint64_t n = ix->npairs[i];
    if (n) qsort(p, n, sizeof(pair_t), cmp_pair);
    uint64_t m = 0, keys = 0;
    for (uint64_t j = 0; j < n; ++j) {
        if (m && p[m - 1].hash == p[j].hash && p[m - 1].tid == p[j].tid) continue;
        if (!m || p[m - 1].hash != p[j].hash) ++keys;
        p[m++] = p[j];
    }
    ix->npairs[i] = m;
    ix->nkeys[i] = keys;
}

orc_index* orc_index_build(unsigned nk, const unsigned* ks, uint32_t ntx, const char* seqs,
                           const uint64_t* offs, uint32_t threshold) {
    if (nk == 0 || nk > 64) return NULL;
    orc_index* ix = (orc_index*)calloc(1, sizeof(orc_index));
    ix->nk = nk;
    ix->ntx = ntx;
    memcpy(ix->ks, ks, nk * sizeof(unsigned));
    uint64_t cap[64];
    for (unsigned i = 0; i < nk; ++i) {
        cap[i] = 1024;
        ix->pairs[i] = (pair_t*)malloc(cap[i] * sizeof(pair_t));
    }
    uint64_t maxlen = 0;
    for (uint32_t t = 0; t < ntx; ++t)
        if (offs[t + 1] - offs[t] > maxlen) maxlen = offs[t + 1] - offs[t];
    uint32_t* buf = (uint32_t*)malloc(sizeof(uint32_t) * (maxlen + 1));
    for (uint32_t t = 0; t < ntx; ++t) {
        const char* s = seqs + offs[t];
        size_t len = offs[t + 1] - offs[t];
        int ok = 1; /* src/main.cpp:66-75: skip if shorter than any k */
        for (unsigned i = 0; i < nk; ++i)
            if (len < ks[i]) ok = 0;
        if (!ok) continue;
        for (unsigned i = 0; i < nk; ++i) { /* src/main.cpp:78-80 */
            size_t m = orc_sketch(s, len, ks[i], threshold, buf);
            if (ix->npairs[i] + m > cap[i]) {
                while (ix->npairs[i] + m > cap[i]) cap[i] *= 2;
                ix->pairs[i] = (pair_t*)realloc(ix->pairs[i], cap[i] * sizeof(pair_t));
            }
            for (size_t j = 0; j < m; ++j) {
                ix->pairs[i][ix->npairs[i]].hash = buf[j];
                ix->pairs[i][ix->npairs[i]].tid = t;
                ix->npairs[i]++;
            }
        }
    }
    free(buf);
    for (unsigned i = 0; i < nk; ++i) finalize_k(ix, i);
    return ix;
}

orc_index* orc_index_from_pairs(unsigned nk, const unsigned* ks, uint32_t ntx,
                                const uint64_t* npairs, const uint32_t* const* hashes,
                                const uint32_t* const* tids) {
    if (nk == 0 || nk > 64) return NULL;
    orc_index* ix = (orc_index*)calloc(1, sizeof(orc_index));
    ix->nk = nk;
    ix->ntx = ntx;
    memcpy(ix->ks, ks, nk * sizeof(unsigned));
    for (unsigned i = 0; i < nk; ++i) {
        ix->npairs[i] = npairs[i];
        ix->pairs[i] = (pair_t*)malloc((npairs[i] + 1) * sizeof(pair_t));
        for (uint64_t j = 0; j < npairs[i]; ++j) {
            ix->pairs[i][j].hash = hashes[i][j];
            ix->pairs[i][j].tid = tids[i][j];
        }
        finalize_k(ix, i);
    }
    return ix;
}

void orc_index_free(orc_index* ix) {
    if (!ix) return;
    for (unsigned i = 0; i < ix->nk; ++i) free(ix->pairs[i]);
    free(ix);
}

uint64_t orc_index_nkeys(const orc_index* ix, unsigned i) { return ix->nkeys[i]; }
uint64_t orc_index_npost(const orc_index* ix, unsigned i) { return ix->npairs[i]; }

void orc_index_export(const orc_index* ix, unsigned i, uint32_t* keys, uint64_t* offs, uint32_t* tids) {
    uint64_t kk = 0;
    const pair_t* p = ix->pairs[i];
    for (uint64_t j = 0; j < ix->npairs[i]; ++j) {
        if (j == 0 || p[j].hash != p[j - 1].hash) {
            keys[kk] = p[j].hash;
            offs[kk] = j;
            ++kk;
        }
        tids[j] = p[j].tid;
    }
    offs[kk] = ix->npairs[i];
}

/* first pair with hash >= h */
static uint64_t lower_bound(const pair_t* p, uint64_t n, uint32_t h) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (p[mid].hash < h) lo = mid + 1; else hi = mid;
    }
    return lo;
}

/* ---- sparse_chain for one read (src/sparse_chaining.cpp:42-111) ------------------------ */
typedef struct { uint32_t tid, ki; } hit_t;

static int cmp_hit(const void* a, const void* b) {
    const hit_t* x = (const hit_t*)a;
    const hit_t* y = (const hit_t*)b;
    if (x->tid != y->tid) return x->tid < y->tid ? -1 : 1;
    return x->ki < y->ki ? -1 : x->ki > y->ki;
}

typedef struct { uint32_t tid, score; } cand_t;

static int cmp_cand(const void* a, const void* b) {
    const cand_t* x = (const cand_t*)a;
    const cand_t* y = (const cand_t*)b;
    if (x->score != y->score) return x->score > y->score ? -1 : 1; /* :108-109 score desc */
    return x->tid < y->tid ? -1 : x->tid > y->tid;               /* normalised tie order */
}

/* `nq` k-lengths are the read's kmer_lengths list (in quant: the index's list, src/main.cpp:178),
 * index slot qi corresponds to ix->ks[qi]. */
static size_t chain_core(const orc_index* ix, const uint32_t* const* hashes, const uint32_t* nh,
                         const int* present, double fraction, uint32_t* out_tid,
                         uint32_t* out_score, size_t cap) {
    const unsigned nq = ix->nk;
    size_t nhits = 0;
    for (unsigned i = 0; i < nq; ++i) {
        if (!present[i]) continue;
        for (uint32_t j = 0; j < nh[i]; ++j) {
            const pair_t* p = ix->pairs[i];
            uint64_t a = lower_bound(p, ix->npairs[i], hashes[i][j]);
            while (a < ix->npairs[i] && p[a].hash == hashes[i][j]) { ++nhits; ++a; }
        }
    }
    hit_t* hits = (hit_t*)malloc(sizeof(hit_t) * (nhits + 1));
    size_t h = 0;
    for (unsigned i = 0; i < nq; ++i) { /* :48-73 count matches per (transcript, k) */
        if (!present[i]) continue;
        for (uint32_t j = 0; j < nh[i]; ++j) {
            const pair_t* p = ix->pairs[i];
            uint64_t a = lower_bound(p, ix->npairs[i], hashes[i][j]);
            for (; a < ix->npairs[i] && p[a].hash == hashes[i][j]; ++a) {
                hits[h].tid = p[a].tid;
                hits[h].ki = i;
                ++h;
            }
        }
    }
    if (h) qsort(hits, h, sizeof(hit_t), cmp_hit);
    /* distinct transcripts with their count vectors */
    size_t ndist = 0;
    for (size_t a = 0; a < h; ++a)
        if (a == 0 || hits[a].tid != hits[a - 1].tid) ++ndist;
    uint32_t* ctid = (uint32_t*)malloc(sizeof(uint32_t) * (ndist + 1));
    int* cnt = (int*)calloc((ndist + 1) * nq, sizeof(int));
    size_t d = 0;
    for (size_t a = 0; a < h; ++a) {
        if (a == 0 || hits[a].tid != hits[a - 1].tid) ctid[d++] = hits[a].tid;
        cnt[(d - 1) * nq + hits[a].ki]++;
    }
    int maxc[64] = {0}; /* :76-82 */
    for (size_t t = 0; t < ndist; ++t)
        for (unsigned i = 0; i < nq; ++i)
            if (cnt[t * nq + i] > maxc[i]) maxc[i] = cnt[t * nq + i];
    double thr[64]; /* :84-87 */
    for (unsigned i = 0; i < nq; ++i) thr[i] = fraction * maxc[i];
    cand_t* cands = (cand_t*)malloc(sizeof(cand_t) * (ndist + 1));
    size_t nc = 0;
    for (size_t t = 0; t < ndist; ++t) { /* :89-105 */
        int meets = 1, score = 0;
        for (unsigned i = 0; i < nq; ++i) {
            if (cnt[t * nq + i] < thr[i]) { meets = 0; break; }
            score += cnt[t * nq + i];
        }
        if (meets) { cands[nc].tid = ctid[t]; cands[nc].score = (uint32_t)score; ++nc; }
    }
    if (nc) qsort(cands, nc, sizeof(cand_t), cmp_cand);
    size_t ret = nc;
    if (nc > cap) ret = (size_t)-1;
    else
        for (size_t c = 0; c < nc; ++c) { out_tid[c] = cands[c].tid; out_score[c] = cands[c].score; }
    free(hits);
    free(ctid);
    free(cnt);
    free(cands);
    return ret;
}

size_t orc_chain_read(const orc_index* ix, const uint32_t* const* hashes, const uint32_t* nh,
                      const int* present, double fraction, uint32_t* out_tid,
                      uint32_t* out_score, size_t cap) {
    return chain_core(ix, hashes, nh, present, fraction, out_tid, out_score, cap);
}

/* sparse_chain over a batch of sketches in CSR form (read r, k slot i: hashes[hash_offs[r*nk+i] ..
 * hash_offs[r*nk+i+1])), every k present; candidates out as CSR. The CPU-baseline calibration
 * (tools/cpu_calibrate.py) times this against the reference's own sparse_chain on the same
 * sketches. Returns 0, or -1 when cap is too small. */
int orc_chain_batch(const orc_index* ix, uint64_t n, const uint64_t* hash_offs, const uint32_t* hashes,
                    double fraction, uint64_t* cand_offs, uint32_t* cand_tid, uint32_t* cand_score,
                    uint64_t cap) {
    const unsigned nk = ix->nk;
    const uint32_t* hp[64];
    uint32_t nh[64];
    int present[64];
    uint64_t o = 0;
    cand_offs[0] = 0;
    for (uint64_t r = 0; r < n; ++r) {
        for (unsigned i = 0; i < nk; ++i) {
            hp[i] = hashes + hash_offs[r * nk + i];
            nh[i] = (uint32_t)(hash_offs[r * nk + i + 1] - hash_offs[r * nk + i]);
            present[i] = 1;
        }
        size_t c = chain_core(ix, hp, nh, present, fraction, cand_tid + o, cand_score + o, cap - o);
        if (c == (size_t)-1) return -1;
        o += c;
        cand_offs[r + 1] = o;
    }
    return 0;
}

/* ---- batch: process_fastq_single_pass filters (src/main.cpp:132-144) + sparse_chain ----- */
static int map_one(const orc_index* ix, const uint8_t* s, size_t len, uint32_t threshold,
                   double fraction, uint8_t* status, uint32_t* hcnt, uint32_t* hout, uint32_t hcap,
                   uint32_t* ccnt, uint32_t* ctid, uint32_t* cscore, uint32_t ccap, uint32_t* scratch) {
    unsigned maxk = 0;
    for (unsigned i = 0; i < ix->nk; ++i)
        if (ix->ks[i] > maxk) maxk = ix->ks[i];
    for (unsigned i = 0; i < ix->nk; ++i) hcnt[i] = 0;
    *ccnt = 0;
    if (!orc_is_valid_sequence((const char*)s, len)) { *status = ORC_INVALID; return 0; }
    if (len < maxk) { *status = ORC_SHORT; return 0; }
    *status = ORC_OK;
    const uint32_t* hp[64];
    int present[64];
    for (unsigned i = 0; i < ix->nk; ++i) {
        uint32_t* dst = scratch + (size_t)i * (len + 1);
        size_t m = orc_sketch((const char*)s, len, ix->ks[i], threshold, dst);
        if (hout && m > hcap) return -1;
        hcnt[i] = (uint32_t)m;
        if (hout) memcpy(hout + (size_t)i * hcap, dst, m * sizeof(uint32_t));
        hp[i] = dst;
        present[i] = 1;
    }
    size_t nc = chain_core(ix, hp, hcnt, present, fraction, ctid, cscore, ccap);
    if (nc == (size_t)-1) return -1;
    *ccnt = (uint32_t)nc;
    return 0;
}

int orc_map_batch(const orc_index* ix, const uint8_t* reads, const uint64_t* offs, uint64_t n,
                  uint32_t threshold, double fraction, uint8_t* status, uint32_t* hash_cnt,
                  uint32_t* hashes, uint32_t hcap, uint32_t* cand_cnt, uint32_t* cand_tid,
                  uint32_t* cand_score, uint32_t ccap) {
    uint64_t maxlen = 0;
    for (uint64_t r = 0; r < n; ++r)
        if (offs[r + 1] - offs[r] > maxlen) maxlen = offs[r + 1] - offs[r];
    uint32_t* scratch = (uint32_t*)malloc(sizeof(uint32_t) * (maxlen + 1) * ix->nk + 4);
    int rc = 0;
    for (uint64_t r = 0; r < n && rc == 0; ++r)
        rc = map_one(ix, reads + offs[r], offs[r + 1] - offs[r], threshold, fraction, status + r,
                     hash_cnt + r * ix->nk, hashes + r * ix->nk * hcap, hcap, cand_cnt + r,
                     cand_tid + r * ccap, cand_score + r * ccap, ccap, scratch);
    free(scratch);
    return rc;
}

uint64_t orc_map_batch_count(const orc_index* ix, const uint8_t* reads, const uint64_t* offs,
                             uint64_t n, uint32_t threshold, double fraction) {
    uint64_t maxlen = 0, total = 0;
    for (uint64_t r = 0; r < n; ++r)
        if (offs[r + 1] - offs[r] > maxlen) maxlen = offs[r + 1] - offs[r];
    uint32_t* scratch = (uint32_t*)malloc(sizeof(uint32_t) * (maxlen + 1) * ix->nk + 4);
    uint32_t hcnt[64], ccnt;
    uint32_t* ctid = (uint32_t*)malloc(sizeof(uint32_t) * (ix->ntx + 1));
    uint32_t* csc = (uint32_t*)malloc(sizeof(uint32_t) * (ix->ntx + 1));
    uint8_t st;
    for (uint64_t r = 0; r < n; ++r) {
        map_one(ix, reads + offs[r], offs[r + 1] - offs[r], threshold, fraction, &st, hcnt, NULL,
                0, &ccnt, ctid, csc, ix->ntx + 1, scratch);
        total += ccnt;
    }
    free(scratch);
    free(ctid);
    free(csc);
    return total;
}

/* ---- EM + assignment (src/isoform_assignment.cpp:9-97) ------------------------------------ */
int orc_em(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
           const uint32_t* cand_score, uint32_t ntx, int max_iterations, double convergence,
           double* pi) {
    double* post = (double*)malloc(sizeof(double) * (ntx ? ntx : 1));
    int it;
    for (uint32_t t = 0; t < ntx; ++t) pi[t] = 1.0 / ntx;                      /* :17-20 */
    for (it = 0; it < max_iterations; ++it) {                                    /* :23 */
        double total_change = 0.0;
        for (uint32_t t = 0; t < ntx; ++t) post[t] = 0.0;
        for (uint64_t r = 0; r < nreads; ++r) {                                  /* :30-50 */
            double denominator = 0.0;
            for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c)
                denominator += pi[cand_tid[c]] * (double)cand_score[c];
            if (denominator > 1e-10) {
                double inv = 1.0 / denominator;
                for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c)
                    post[cand_tid[c]] += pi[cand_tid[c]] * (double)cand_score[c] * inv;
            }
        }
        {
            float pseudocount = 0.01f;                                           /* :53-62 */
            for (uint32_t t = 0; t < ntx; ++t) {
                double new_pi = post[t] + pseudocount / (float)nreads + pseudocount;
                total_change += fabs(new_pi - pi[t]);
                pi[t] = new_pi;
            }
        }
        if (total_change < convergence) {
            ++it;
            break;
        }
    }
    free(post);
    return it;
}

void orc_assign(uint64_t nreads, const uint64_t* cand_offs, const uint32_t* cand_tid,
                const uint32_t* cand_score, uint32_t ntx, const double* pi, double* counts,
                uint8_t* assigned) {
    for (uint32_t t = 0; t < ntx; ++t) {
        counts[t] = 0.0;
        assigned[t] = 0;
    }
    for (uint64_t r = 0; r < nreads; ++r) {                                      /* :73-94 */
        double total = 0.0;
        for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c)
            total += pi[cand_tid[c]] * cand_score[c];
        for (uint64_t c = cand_offs[r]; c < cand_offs[r + 1]; ++c) {
            if (total > 0.0) {
                counts[cand_tid[c]] += (pi[cand_tid[c]] * cand_score[c]) / total;
                assigned[cand_tid[c]] = 1;
            }
        }
    }
}

/* ---- the quant hot path from FASTQ bytes (src/main.cpp:107-151 + :181-185) ---------------
 * For bench.py's cpu_baseline and its parity sample. Phase 1 (sequential, as the reference):
 * the record machine of process_fastq_single_pass (:116-130) over the bytes: a line starting
 * with '@' opens a record whose next three lines are sequence, '+' and quality; any other line
 * is skipped. Phase 2 (nthreads over contiguous record ranges): is_valid_sequence, the length
 * filter, every k's sketch and sparse_chain per record (map_one). Phase 3 (sequential): the
 * id map — read_sketches[id] = ... (:147) keeps the LAST valid record of an id — and the
 * per-transcript totals (candidate reads, summed scores) over the kept records. */
#include <pthread.h>

typedef struct {
    const orc_index* ix;
    const char* fq;
    const uint64_t* rec;   /* per record: id start, id len, seq start, seq len */
    uint64_t r0, r1;
    uint32_t threshold;
    double fraction;
    uint8_t* status;
    uint32_t *hash_cnt, *hashes, hcap, *cand_cnt, *cand_tid, *cand_score, ccap;
    uint32_t* cnt_scratch; /* per record candidate count when no outputs are kept */
    uint64_t* tx_acc;      /* per thread: (reads << 40 | score) per transcript, NULL = none */
    int rc;
} fq_job;

static void* fq_worker(void* arg) {
    fq_job* j = (fq_job*)arg;
    const orc_index* ix = j->ix;
    uint64_t maxlen = 1;
    for (uint64_t r = j->r0; r < j->r1; ++r)
        if (j->rec[4 * r + 3] > maxlen) maxlen = j->rec[4 * r + 3];
    uint32_t* scratch = (uint32_t*)malloc(sizeof(uint32_t) * (maxlen + 1) * ix->nk + 4);
    uint32_t hc[64];
    uint32_t* ct = j->cand_tid ? NULL : (uint32_t*)malloc(sizeof(uint32_t) * (ix->ntx + 1));
    uint32_t* cs = j->cand_tid ? NULL : (uint32_t*)malloc(sizeof(uint32_t) * (ix->ntx + 1));
    for (uint64_t r = j->r0; r < j->r1 && j->rc == 0; ++r) {
        uint8_t st;
        uint32_t nc;
        const uint8_t* s = (const uint8_t*)j->fq + j->rec[4 * r + 2];
        const size_t len = j->rec[4 * r + 3];
        if (j->cand_tid)
            j->rc = map_one(ix, s, len, j->threshold, j->fraction, &st, j->hash_cnt + r * ix->nk,
                            j->hashes + r * ix->nk * j->hcap, j->hcap, &nc, j->cand_tid + r * j->ccap,
                            j->cand_score + r * j->ccap, j->ccap, scratch);
        else
            j->rc = map_one(ix, s, len, j->threshold, j->fraction, &st, hc, NULL, 0, &nc, ct, cs, ix->ntx + 1,
                            scratch);
        j->status[r] = st;
        j->cnt_scratch[r] = nc;
        if (j->tx_acc && !j->cand_tid) /* totals straight from this record's candidates */
            for (uint32_t c = 0; c < nc; ++c) j->tx_acc[ct[c]] += (1ull << 40) | cs[c];
    }
    free(scratch);
    free(ct);
    free(cs);
    return NULL;
}

static uint64_t fnv1a(const char* s, uint64_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint64_t q = 0; q < n; ++q) h = (h ^ (uint8_t)s[q]) * 1099511628211ull;
    return h;
}

int orc_fastq_map(const orc_index* ix, const char* fq, uint64_t len, uint32_t threshold, double fraction,
                  int nthreads, uint64_t max_records, uint64_t* n_records, uint8_t* status, uint32_t* hash_cnt,
                  uint32_t* hashes, uint32_t hcap, uint32_t* cand_cnt, uint32_t* cand_tid, uint32_t* cand_score,
                  uint32_t ccap, uint8_t* kept, uint64_t* tx_reads, uint64_t* tx_score) {
    /* phase 1: the record machine */
    uint64_t cap = 1024, n = 0, pos = 0;
    uint64_t* rec = (uint64_t*)malloc(sizeof(uint64_t) * 4 * cap);
    uint64_t lines[4];
    while (pos < len && n < max_records) {
        const char* nl = (const char*)memchr(fq + pos, '\n', len - pos);
        const uint64_t end = nl ? (uint64_t)(nl - fq) : len;
        if (end == pos || fq[pos] != '@') { pos = end + 1; continue; } /* :118-120 */
        /* header = [pos, end); then getline x3 (a missing line reads as empty) */
        uint64_t p = end + 1;
        for (int q = 0; q < 3; ++q) {
            if (p >= len) { lines[q] = len; continue; }
            const char* e = (const char*)memchr(fq + p, '\n', len - p);
            lines[q] = p;
            p = e ? (uint64_t)(e - fq) + 1 : len;
        }
        if (n == cap) { cap *= 2; rec = (uint64_t*)realloc(rec, sizeof(uint64_t) * 4 * cap); }
        rec[4 * n] = pos + 1;
        rec[4 * n + 1] = end - pos - 1;
        const uint64_t ss = lines[0];
        uint64_t se = ss;
        while (se < len && fq[se] != '\n') ++se;
        rec[4 * n + 2] = ss;
        rec[4 * n + 3] = se - ss;
        ++n;
        pos = p;
    }
    *n_records = n;
    /* phase 2: records in parallel */
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    uint8_t* st = status ? status : (uint8_t*)malloc(n + 1);
    uint32_t* cc = cand_cnt ? cand_cnt : (uint32_t*)malloc(sizeof(uint32_t) * (n + 1));
    fq_job jobs[256];
    pthread_t th[256];
    const int direct_totals = !cand_tid && tx_reads; /* per-thread totals, no per-record lists */
    for (int t = 0; t < nthreads; ++t) {
        fq_job* j = &jobs[t];
        memset(j, 0, sizeof(*j));
        j->ix = ix; j->fq = fq; j->rec = rec;
        j->r0 = n * t / nthreads; j->r1 = n * (t + 1) / nthreads;
        j->threshold = threshold; j->fraction = fraction;
        j->status = st; j->hash_cnt = hash_cnt; j->hashes = hashes; j->hcap = hcap;
        j->cand_cnt = cc; j->cand_tid = cand_tid; j->cand_score = cand_score; j->ccap = ccap;
        j->cnt_scratch = cc;
        j->tx_acc = direct_totals ? (uint64_t*)calloc(ix->ntx + 1, sizeof(uint64_t)) : NULL;
        pthread_create(&th[t], NULL, fq_worker, j);
    }
    int rc = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
    }
    /* phase 3: last valid record per id wins (:147), totals over the kept records */
    uint64_t tcap = 16;
    while (tcap < 2 * n + 2) tcap *= 2;
    int64_t* tab = (int64_t*)malloc(sizeof(int64_t) * tcap);
    for (uint64_t q = 0; q < tcap; ++q) tab[q] = -1;
    uint8_t* kp = kept ? kept : (uint8_t*)malloc(n + 1);
    memset(kp, 0, n + 1);
    uint64_t dups = 0;
    for (uint64_t r = 0; r < n; ++r) {
        if (st[r] != ORC_OK) continue;
        const char* id = fq + rec[4 * r];
        const uint64_t il = rec[4 * r + 1];
        uint64_t q = fnv1a(id, il) & (tcap - 1);
        while (tab[q] >= 0) {
            const uint64_t o = (uint64_t)tab[q];
            if (rec[4 * o + 1] == il && !memcmp(fq + rec[4 * o], id, il)) break;
            q = (q + 1) & (tcap - 1);
        }
        if (tab[q] >= 0) { kp[tab[q]] = 0; ++dups; }
        tab[q] = (int64_t)r;
        kp[r] = 1;
    }
    if (tx_reads) {
        memset(tx_reads, 0, sizeof(uint64_t) * ix->ntx);
        memset(tx_score, 0, sizeof(uint64_t) * ix->ntx);
        if (direct_totals && !dups) {
            for (int t = 0; t < nthreads; ++t)
                for (uint32_t x = 0; x < ix->ntx; ++x) {
                    tx_reads[x] += jobs[t].tx_acc[x] >> 40;
                    tx_score[x] += jobs[t].tx_acc[x] & ((1ull << 40) - 1);
                }
        } else if (cand_tid) {
            for (uint64_t r = 0; r < n; ++r)
                if (kp[r])
                    for (uint32_t c = 0; c < cc[r]; ++c) {
                        tx_reads[cand_tid[r * ccap + c]] += 1;
                        tx_score[cand_tid[r * ccap + c]] += cand_score[r * ccap + c];
                    }
        } else {
            rc = rc ? rc : -2; /* duplicates without per-record lists: totals unavailable */
        }
    }
    for (int t = 0; t < nthreads; ++t) free(jobs[t].tx_acc);
    free(tab);
    if (!kept) free(kp);
    if (!status) free(st);
    if (!cand_cnt) free(cc);
    free(rec);
    return rc;
}

/* ---- per-read digests (tests: per-read parity at full batch sizes) ------------------------ */
static uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}
static uint64_t dg_item(uint64_t tag, uint64_t j, uint64_t v) { return mix64((tag << 56) ^ (j << 32) ^ v); }

typedef struct {
    const orc_index* ix;
    const uint8_t* bases;
    uint32_t L, threshold;
    double fraction;
    uint64_t r0, r1;
    uint64_t* digest;
    uint64_t* tx_acc; /* (reads << 40 | score) per transcript, this thread's reads */
    int rc;
} dg_job;

static void* dg_worker(void* arg) {
    dg_job* j = (dg_job*)arg;
    const orc_index* ix = j->ix;
    uint32_t* scratch = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)j->L + 1) * ix->nk + 4);
    uint32_t* hs = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)j->L + 1) * ix->nk + 4);
    uint32_t* ct = (uint32_t*)malloc(sizeof(uint32_t) * (ix->ntx + 1));
    uint32_t* cs = (uint32_t*)malloc(sizeof(uint32_t) * (ix->ntx + 1));
    uint32_t hc[64];
    for (uint64_t r = j->r0; r < j->r1 && j->rc == 0; ++r) {
        uint8_t st;
        uint32_t nc;
        j->rc = map_one(ix, j->bases + r * j->L, j->L, j->threshold, j->fraction, &st, hc, hs, j->L + 1, &nc, ct, cs,
                        ix->ntx + 1, scratch);
        uint64_t d = dg_item(0xA5, 0, st);
        for (unsigned i = 0; i < ix->nk; ++i)
            for (uint32_t q = 0; q < hc[i]; ++q) d += dg_item(i + 1, q, hs[(size_t)i * (j->L + 1) + q]);
        for (uint32_t q = 0; q < nc; ++q) {
            d += dg_item(0xC0, q, ct[q]) + dg_item(0xD0, q, cs[q]);
            if (j->tx_acc) j->tx_acc[ct[q]] += (1ull << 40) | cs[q];
        }
        j->digest[r] = d;
    }
    free(scratch);
    free(hs);
    free(ct);
    free(cs);
    return NULL;
}

int orc_map_digest(const orc_index* ix, const uint8_t* bases, uint32_t L, uint64_t n, uint32_t threshold,
                   double fraction, int nthreads, uint64_t* digest, uint64_t* tx_reads, uint64_t* tx_score) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    dg_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        dg_job* j = &jobs[t];
        memset(j, 0, sizeof(*j));
        j->ix = ix; j->bases = bases; j->L = L; j->threshold = threshold; j->fraction = fraction;
        j->r0 = n * t / nthreads; j->r1 = n * (t + 1) / nthreads;
        j->digest = digest;
        j->tx_acc = tx_reads ? (uint64_t*)calloc(ix->ntx + 1, sizeof(uint64_t)) : NULL;
        pthread_create(&th[t], NULL, dg_worker, j);
    }
    int rc = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = -1;
    }
    if (tx_reads) {
        memset(tx_reads, 0, sizeof(uint64_t) * ix->ntx);
        memset(tx_score, 0, sizeof(uint64_t) * ix->ntx);
        for (int t = 0; t < nthreads; ++t) {
            for (uint32_t x = 0; x < ix->ntx; ++x) {
                tx_reads[x] += jobs[t].tx_acc[x] >> 40;
                tx_score[x] += jobs[t].tx_acc[x] & ((1ull << 40) - 1);
            }
            free(jobs[t].tx_acc);
        }
    }
    return rc;
}
