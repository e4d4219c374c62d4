// skq_internal.h — structures shared by the HIP kernels (skq_kernels.hip) and the C-ABI host
// side (skq_capi.hip). Not part of the public ABI.
#pragma once
#include <cstdint>

#include "skq.h"

namespace skq {

constexpr int WG = 256;            // threads per workgroup for both kernels (4 waves)
constexpr int LFAST = 256;         // reads longer than this take the slow path
constexpr int DCAP = 16;           // distinct transcripts per read on the fast chain path
constexpr int CCAP = DCAP;         // candidate slots per read (fast path can't exceed DCAP)
constexpr int HFAST = 16;          // hashes per (read, k) the fast chain path accepts
constexpr int NK_FAST = 4;         // k slots the fast chain path packs (8-bit counts)
constexpr uint64_t EMPTY_SLOT = ~0ull;
constexpr uint32_t HASH_MUL = 0x9E3779B1u;

// status flags above SKQ_STATUS_MASK (internal)
constexpr uint8_t ST_SLOW1 = 0x10;  // sketch handled by the slow path

// control block (u32 words): the sketch half (words 0-7) is zeroed before every sketch, the
// chain half (words 8-15) before every chain.
enum Ctrl : int {
    C_OVF1 = 0,     // sketch overflow list length
    C_ERR1 = 1,     // sketch error bits
    C_BUMP_H = 2,   // u64 (words 2-3): hash_ext words used
    C_OVF2 = 8,     // chain overflow list length
    C_ERR2 = 9,     // chain error bits
    C_BUMP_S = 10,  // u64 (words 10-11): chain scratch u64 words used
    C_BUMP_C = 12,  // u64 (words 12-13): cand_ext pairs used
    C_WORDS = 16
};
enum Err : uint32_t {
    E_OVF1_FULL = 1, E_OVF2_FULL = 2, E_HASH_EXT = 4, E_SCRATCH = 8, E_CAND_EXT = 16
};

struct DevTable {
    uint64_t slot_base;  // first slot of this k's table in the slot array
    uint32_t log2cap;
    uint32_t present;    // 0: the index has no table for this k (skipped, src/sparse_chaining.cpp:51-53)
};

struct SketchParams {
    const uint8_t* reads;
    const uint64_t* offs;  // null => fixed_len
    uint64_t fixed_len;
    uint64_t n;
    uint32_t nk;
    uint32_t maxk;
    uint32_t ks[SKQ_MAX_K];
    uint32_t threshold;
    uint32_t tile_chunks;  // 16-byte chunks staged per workgroup
    uint32_t hcap;
    uint32_t ovf_cap;
    const uint64_t* rolltab;  // [nk][32] 33-bit entries: seed(in) ^ rot^k(seed(out)), out=4 => none
    uint8_t* status;
    uint32_t* hash_cnt;
    uint32_t* hashes;
    uint32_t* hash_ext;
    uint64_t hash_ext_cap;
    uint32_t* ctrl;
    uint32_t* ovf1;
};

struct ChainParams {
    uint64_t n;
    uint32_t nk;
    uint32_t hcap;
    double fraction;
    int accumulate;
    uint32_t ovf_cap;
    const uint8_t* status;     // null => every read sketched (chain_sketches)
    const uint32_t* hash_cnt;
    const uint32_t* hashes;    // padded (session) or flat (explicit offsets)
    const uint32_t* hash_ext;
    const uint64_t* hash_offs; // null => padded layout
    const uint8_t* present;    // null => all k present
    const uint64_t* slots;
    const uint32_t* post;
    DevTable tabs[SKQ_MAX_K];
    uint32_t* cand_cnt;
    uint32_t* cand_tid;
    uint32_t* cand_score;
    uint32_t* cand_ext;
    uint64_t cand_ext_cap;     // pairs
    uint64_t* scratch;
    uint64_t scratch_cap;      // u64 words
    uint64_t* tx_reads;
    uint64_t* tx_score;
    uint32_t* ctrl;
    uint32_t* ovf2;
};

// records the message returned by skq_last_error(); returns code (skq_capi.hip)
int set_error(int code, const char* msg);

// launchers (skq_kernels.hip)
int launch_sketch(const SketchParams& p, void* stream);
int launch_sketch_slow(const SketchParams& p, void* stream);
int launch_chain(const ChainParams& p, void* stream);
int launch_chain_slow(const ChainParams& p, void* stream);
size_t sketch_lds_bytes(uint32_t nk, uint32_t tile_chunks, uint32_t hcap);

// 33-bit ntHash lane (bits 0..32 of ntHash's split rotate evolve on their own)
constexpr uint64_t M33 = (1ull << 33) - 1;
inline uint64_t rot33(uint64_t x, unsigned d) {
    d %= 33;
    return d ? (((x << d) | (x >> (33 - d))) & M33) : x;
}
// seed33 by 2-bit code: ((ascii >> 1) & 3): A=0, C=1, T=2, G=3
constexpr uint64_t SEED33[4] = {0x195c60474ull, 0x162a02b4cull, 0x14be24456ull, 0x082572324ull};

}  // namespace skq
