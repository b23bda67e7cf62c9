// Fast path of libkwmatch (gfx950): lean scan + register-resident resolve.
//
// Anchors.  Every use of a name is found through a short "anchor" substring
// (4..8 bytes, or the whole name when it is only 2-3 bytes) chosen at the
// rarest 4-byte offset of the span it stands for, using q-gram statistics of a
// background sample of the corpus.  A use verifies its whole span around the
// anchor hit:
//   U      whole uppercase name + the two \b conditions  (match_keywords.py:167)
//   FULL   whole fuzzy name, byte-exact  (an exact substring = score 100)
//   PIECE  one pigeonhole piece of a fuzzy name (seeds the LCS verification)
//   RXW    whole name as a '.'-wildcard regex (positions of re.finditer)
// Any anchor choice is correct; only the speed depends on the statistics.
//
// Filter.  4-byte keys in a 2^18-bit LDS table: word = hash(b0,b1,b2),
// bit = mix(b3); 3-byte anchors fill their whole word.  2-byte anchors are
// found through a cheap byte-class gate + an exact 64K-bit bigram table.
#pragma once
#include "kwmatch_device.hpp"

namespace kw {

constexpr int FK_WAVES = 16;                    // waves per workgroup (1024 threads)
constexpr int FK_BLOCK = FK_WAVES * WAVE;
constexpr int FK_FILT_WORDS = 8192;             // 32 KB
constexpr int FK_B2_WORDS = 2048;               // 8 KB (64K bits)
constexpr int FK_CAND = 256;                    // candidates per compaction round
constexpr int FK_ITEMS = 64;                    // items per field on the fast path
constexpr int FK_CP_CAP = 16384;                // bytes of a non-ASCII field the fast path decodes
constexpr uint32_t FK_MUL1 = 0x9E3779u;         // 24-bit multipliers (v_mul_u32_u24)
constexpr uint32_t FK_MUL2 = 0xC2B2AEu;

enum FastUseKind : uint32_t { FU_UPPER = 0, FU_FULL = 1, FU_PIECE = 2, FU_RXW = 3 };

// pattern regex kind (bits [25:24] of fpat_info... kept in a separate array)
enum RxKind : uint32_t { RXK_LITERAL = 0, RXK_WILD = 1, RXK_GENERIC = 2 };

struct FastTables {
    const uint32_t *filt;       // FK_FILT_WORDS
    const uint32_t *b2;         // FK_B2_WORDS
    uint32_t gate_lo[4], gate_hi[4];   // byte ranges gating the 2-byte path
    int n_gate;                 // 0 = no 2-byte anchors, -1 = test every position
    const uint64_t *ht_key;     // (len << 32) | key bytes; ~0 = empty
    const uint32_t *ht_begin;
    const uint32_t *ht_cnt;
    uint32_t ht_mask;
    const uint32_t *kl;         // anchor ids
    const uint64_t *as_head;    // anchor bytes (<= 8), little endian
    const uint32_t *as_len;
    const uint32_t *as_use_begin;
    const uint32_t *as_use_cnt;
    const uint32_t *use_pat;
    const uint32_t *use_info0;  // kind | aoff << 8 | sboff << 16
    const uint32_t *use_info1;  // sblen | pcp << 16 | pcl << 24
    const uint32_t *pat_info;   // as DevTables (PI_*, m, blen)
    const uint32_t *pat_rxk;    // RxKind
    const uint32_t *pat_boff;   // byte offset of the name in pat_bytes
    const uint8_t *pat_bytes;
    const uint32_t *pat_cp_off;
    const uint32_t *pat_cps;
    const uint64_t *pat_sig;    // char-set signature (bit c & 63)
    const int32_t *f_count_ge;
    const uint64_t *sub_key;
    const uint32_t *sub_begin;
    const uint32_t *sub_cnt;
    const uint32_t *sub_pat;
    uint32_t sub_mask;
    const uint32_t *word_bits;
    int f_first;
    int empty_pat;
};

struct FastScratch {
    kw_hit *out;                // per wave: out_cap records
    uint32_t *out_cnt;          // per wave
    uint32_t out_cap;
    uint32_t *cps;              // per wave: CP_CAP decoded code points (non-ASCII fields)
    uint32_t *cpbase;           // per wave: CP_CAP/4 cumulative lead counts per 16-byte chunk
    uint32_t *defer_list;       // docs sent to the generic kernel
    uint32_t *defer_cnt;
    uint32_t defer_cap;
    uint32_t *status;
    unsigned long long *stats;  // [0] candidates [1] anchor hits [2] verify items [3] LCS windows [4] deferred
};

}  // namespace kw
