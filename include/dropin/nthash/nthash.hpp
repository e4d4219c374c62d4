// Drop-in for <nthash/nthash.hpp> (bcgsc ntHash >= 2.3; the reference includes it at src/main.cpp:13,
// src/sketch.cpp:7 and src/kmer.cpp, links -lnthash at build.sh:34). skq replaces libnthash on the
// quant path (the sketch runs in the HIP kernels), so a reference build that links libskq instead
// of libnthash needs this header and nothing else.
//
// Header-only, forward strand only: the subset the reference calls — NtHash(seq, num_hashes, k,
// pos), roll(), get_forward_hash(), get_pos() (src/sketch.cpp:31-33, src/kmer.cpp:26-30). The 64-bit
// forward hash is ntHash's: fwd(s_0..s_{k-1}) = XOR_i srol^{k-1-i}(SEED[s_i]) with the split rotate
// (high 31 bits and low 33 bits rotating apart); a window holding a byte outside ACGTUacgtu is
// skipped (init() jumps past the window's last such byte; roll() with such an incoming byte jumps
// pos += k and re-inits). Pinned against the SEED/DIMER/TETRAMER/X31L/X33R tables embedded in the
// reference's build/test and the SURVEY.md §8c known answers (tests/test_dropin_ref.py).
// Reverse-strand and multi-hash accessors are not provided (no caller on the reference's path).
#ifndef SKQ_DROPIN_NTHASH_HPP
#define SKQ_DROPIN_NTHASH_HPP

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <iostream>
#include <string>

namespace nthash {

namespace detail {

inline uint64_t seed(unsigned char c) {
    switch (c) {
    case 'A': case 'a': return 0x3c8bfbb395c60474ULL;
    case 'C': case 'c': return 0x3193c18562a02b4cULL;
    case 'G': case 'g': return 0x20323ed082572324ULL;
    case 'T': case 't': case 'U': case 'u': return 0x295549f54be24456ULL;
    default: return 0;  // SEED_N: the window is skipped
    }
}

// split rotate left by d: bits 33..63 rotate among themselves, bits 0..32 among themselves
inline uint64_t srol(uint64_t x, unsigned d) {
    const uint64_t hi = x >> 33, lo = x & ((1ULL << 33) - 1);
    const unsigned dh = d % 31, dl = d % 33;
    const uint64_t h2 = dh ? (((hi << dh) | (hi >> (31 - dh))) & ((1ULL << 31) - 1)) : hi;
    const uint64_t l2 = dl ? (((lo << dl) | (lo >> (33 - dl))) & ((1ULL << 33) - 1)) : lo;
    return (h2 << 33) | l2;
}

[[noreturn]] inline void fail(const std::string& msg) {
    std::cerr << "[ntHash::NtHash] ERROR: " << msg << std::endl;
    std::exit(EXIT_FAILURE);
}

}  // namespace detail

class NtHash {
  public:
    NtHash(const char* seq, size_t seq_len, uint8_t num_hashes, uint16_t k, size_t pos = 0)
        : seq_(seq), len_(seq_len), k_(k), pos_(pos) {
        if (k == 0) detail::fail("k must be greater than 0");
        if (num_hashes == 0) detail::fail("num_hashes must be greater than 0");
        if (seq_len < k)
            detail::fail("sequence length (" + std::to_string(seq_len) + ") is smaller than k (" +
                         std::to_string(k) + ")");
        if (pos >= seq_len) detail::fail("passed position (" + std::to_string(pos) + ") exceeds sequence length");
        for (int b = 0; b < 4; ++b) rolk_[b] = detail::srol(detail::seed("ACGT"[b]), k);
    }
    NtHash(const std::string& seq, uint8_t num_hashes, uint16_t k, size_t pos = 0)
        : NtHash(seq.data(), seq.size(), num_hashes, k, pos) {}

    // Next valid window: the first call hashes the first one; false when none is left.
    bool roll() {
        if (!init_) return init();
        if (pos_ >= len_ - k_) return false;
        const unsigned char in = (unsigned char)seq_[pos_ + k_];
        if (detail::seed(in) == 0) {
            pos_ += k_;
            return init();
        }
        const uint64_t out = detail::seed((unsigned char)seq_[pos_]);
        uint64_t rk = 0;
        for (int b = 0; b < 4; ++b)
            if (out == detail::seed("ACGT"[b])) rk = rolk_[b];
        fwd_ = detail::srol(fwd_, 1) ^ detail::seed(in) ^ rk;
        ++pos_;
        return true;
    }

    uint64_t get_forward_hash() const { return fwd_; }
    size_t get_pos() const { return pos_; }

  private:
    bool init() {
        while (pos_ + k_ <= len_) {
            long bad = -1;
            for (long i = (long)k_ - 1; i >= 0; --i)
                if (detail::seed((unsigned char)seq_[pos_ + (size_t)i]) == 0) {
                    bad = i;
                    break;
                }
            if (bad < 0) break;
            pos_ += (size_t)bad + 1;
        }
        if (pos_ + k_ > len_) return false;
        fwd_ = 0;
        for (unsigned i = 0; i < k_; ++i) fwd_ = detail::srol(fwd_, 1) ^ detail::seed((unsigned char)seq_[pos_ + i]);
        init_ = true;
        return true;
    }

    const char* seq_;
    size_t len_;
    unsigned k_;
    size_t pos_;
    bool init_ = false;
    uint64_t fwd_ = 0;
    uint64_t rolk_[4] = {};
};

}  // namespace nthash

#endif  // SKQ_DROPIN_NTHASH_HPP
