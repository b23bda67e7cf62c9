// Device-side data structures and helpers of libkwmatch (gfx950 only).
//
// The compiled knowledge base lives in HBM as flat arrays (struct DevTables);
// the 32 KB first-level filter is staged into LDS by every workgroup.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kwmatch.h"

namespace kw {

constexpr int WAVE = 64;
constexpr int WAVES_PER_BLOCK = 4;
constexpr int BLOCK = WAVE * WAVES_PER_BLOCK;
constexpr int FILT_BITS = 18;                       // 2^18-bit filter = 32 KB of LDS
constexpr int FILT_WORDS = 1 << (FILT_BITS - 5);
constexpr int SCAN_TILE = 1024;                     // bytes per wave per scan step (16 B / lane)
constexpr int CAND_CAP = SCAN_TILE;                 // candidates per tile (<= positions)
constexpr int ITEM_CAP = 16384;                     // anchor uses per field per doc, initial (grows)
constexpr int CP_CAP = 65536;                       // decoded code points per non-ASCII field, initial (grows)
constexpr int MAXM = 64;                            // longest fuzzy name (rapidfuzz short-needle path)
constexpr int SHORT_EXACT_MAX = 10;                 // fields this short can only match exactly
constexpr int RX_MAX_QUANT = 16;                    // quantified atoms per regex program
constexpr uint32_t HASH_MUL = 0x9E3779B1u;
constexpr uint64_t SUB_B = 0x100000001B3ull;        // substring polynomial hash base

// item = one occurrence of an anchor use inside a field, packed for sorting by
// (pattern, byte position, kind, use):
//   [63:44] pattern  [43:21] field-relative byte pos  [20:19] kind  [18:0] use
constexpr int IT_PAT_SHIFT = 44;
constexpr int IT_POS_SHIFT = 21;
constexpr int IT_KIND_SHIFT = 19;
constexpr uint64_t IT_POS_MASK = (1ull << 23) - 1;
constexpr uint32_t IT_USE_MASK = (1u << 19) - 1;
constexpr int64_t MAX_FIELD_BYTES = (int64_t)IT_POS_MASK;

enum UseKind : uint32_t { USE_UPPER = 0, USE_FULL = 1, USE_PIECE = 2 };

// pat_info bits
constexpr uint32_t PI_FUZZY = 1u;        // class F (else U)
constexpr uint32_t PI_LITERAL = 2u;      // F: re.finditer(name) == literal search
constexpr uint32_t PI_WORD_FIRST = 4u;   // U: first code point is a \b word char
constexpr uint32_t PI_WORD_LAST = 8u;    // U: last code point is a \b word char
constexpr uint32_t PI_ASCII = 16u;       // every code point < 128 (bytes = code points)
constexpr uint32_t PI_TXUNSAFE = 32u;    // F: the transcoded view cannot decide it (a code point without a
                                         // marker, or quantified regex atoms over non-ASCII code points)
// m (code points) in bits [15:8], byte length in bits [31:16]
__host__ __device__ inline uint32_t pi_m(uint32_t pi) { return (pi >> 8) & 0xFF; }
__host__ __device__ inline uint32_t pi_blen(uint32_t pi) { return pi >> 16; }

// use_info: kind [1:0], piece cp offset [15:8], piece cp length [23:16]
struct DevTables {
    const uint32_t *filt;
    const uint32_t *ht_key;
    const uint32_t *ht_begin;
    const uint32_t *ht_cnt;
    uint32_t ht_mask;
    int ht_shift;
    const uint32_t *kl_anchor;
    const uint64_t *as_head;
    const uint32_t *as_off;
    const uint32_t *as_len;
    const uint32_t *as_use_begin;
    const uint32_t *as_use_cnt;
    const uint8_t *as_bytes;
    const uint32_t *use_pat;
    const uint32_t *use_info;
    const uint32_t *pat_info;
    const uint32_t *pat_cp_off;
    const uint32_t *pat_cps;
    const uint64_t *pm_ascii;      // [n_pat][128]
    const uint32_t *pm_ext_off;    // [n_pat+1]
    const uint32_t *pm_ext_cp;
    const uint64_t *pm_ext_mask;
    const uint32_t *rx_off;        // [n_pat+1], index into rx_atoms
    const int4 *rx_atoms;
    const uint32_t *word_bits;     // 0x110000 bits
    const int32_t *f_count_ge;     // [MAXM+2]
    // exact-substring table for short fields (<= SHORT_EXACT_MAX code points)
    const uint64_t *sub_key;
    const uint32_t *sub_begin;
    const uint32_t *sub_cnt;
    const uint32_t *sub_pat;
    uint32_t sub_mask;
    int n_pat;
    int f_first;
    int empty_pat;                 // pattern id of the empty fuzzy name, or -1
};

struct DevScratch {
    uint64_t *items;               // per wave: 2 * item_cap
    uint32_t *cps;                 // per wave: cp_cap
    uint32_t *blkcnt;              // per wave: cp_cap/16 + 2 (cumulative lead bytes per 64 B)
    uint32_t item_cap;             // anchor uses per field (grown by the host when a document needs more)
    uint32_t cp_cap;               // decoded code points per non-ASCII field (likewise)
    uint32_t *gmax;                // [2] largest item count / code point count a deferred field needed
    kw_hit *out;                   // per wave: out_cap
    uint32_t *out_cnt;             // per wave
    uint32_t *status;              // [0] error bits, [1] max item count seen
    unsigned long long *stats;     // [0] candidates [1] anchor hits [2] windows
    uint32_t out_cap;
};

constexpr uint32_t ST_ITEM_OVERFLOW = 1u;
constexpr uint32_t ST_OUT_OVERFLOW = 2u;
constexpr uint32_t ST_CP_OVERFLOW = 4u;
constexpr uint32_t ST_FIELD_TOO_LONG = 8u;
constexpr uint32_t ST_RX_OVERFLOW = 16u;     // a resolve wave queued more regex searches than rx_cap
constexpr uint32_t ST_TASK_OVERFLOW = 32u;   // a scan wave made more tasks than a task region holds
constexpr uint32_t ST_DSET_FULL = 64u;       // the decided-name set is full
static_assert(KW_RESCAN_GENERIC_ITEMS == 1 && KW_RESCAN_RESULTS == 2 && KW_RESCAN_GENERIC_CPS == 4 &&
              KW_RESCAN_REGEX_QUEUE == 16 && KW_RESCAN_TASK_QUEUES == 32 && KW_RESCAN_DECIDED_SET == 64 &&
              KW_RESCAN_REGIONS == 128, "the public rescan bits are the ST_* overflow bits");
constexpr uint32_t ST_CAND_OVERFLOW = 128u;  // a filter region held more candidates, or a probe region more items, than fit

}  // namespace kw
