// Fast path of libkwmatch (gfx950): a lean byte scan (kwmatch_split.hpp: filter, probe, epilogue) that
// turns every anchor occurrence into an item, and a resolve kernel
// (kw_resolve_kernel) that decides the names of each field from its items.
//
// Anchors.  Every use of a name is found through a short "anchor" substring
// (4..8 bytes, or the whole name when it is only 2-3 bytes) chosen at the
// rarest 4-byte offset of the span it stands for, using q-gram statistics of a
// background sample of the corpus.  A use verifies its whole span around the
// anchor hit:
//   U      whole uppercase name + the two \b conditions  (match_keywords.py:167)
//   FULL   whole fuzzy name, byte-exact  (an exact substring = score 100)
//   PIECE  one pigeonhole piece of a fuzzy name with m >= 21 (seeds the LCS
//          verification; shorter names only allow exact interior windows)
// Fuzzy names with 11 <= m <= 20 can also pass on an edge window: the first or
// last m-1 code points of the field equal the name with one code point
// deleted.  Those are found per field through the "edge" hash table of all
// one-deletion variants and enter the item list as EDGE items.  A decided
// name whose re.finditer needs the regex engine is searched wave-parallel
// over its field after the decision (rx_positions).
// Any anchor choice is correct; only the speed depends on the statistics.
//
// Filters (all in LDS).  Stage 1 looks at every byte position j: the 4-gram
// starting there is hashed (two 24-bit products: bytes j..j+2 and j+1..j+3,
// fk_s1_hash) into a 2^19-bit table of the anchors' first four bytes; anchors
// of 2-3 bytes: their first two bytes in an exact 64K-bit pair table.  Only the
// survivors (~1 % of the positions) run stage 2, each in its own lane: an
// independent hash of the 4-byte key (2^18 bits), of the 3-byte key (2^16 bits)
// or of the 2-byte key (2^16 bits) must hit before the global anchor hash
// table is probed.  Field edges: the first / last four bytes of a field are
// tested against the prefix / suffix keys of the one-deletion variants
// (2 x 2^15 bits); only flagged fields run the edge check.
#pragma once
#include "kwmatch_device.hpp"

namespace kw {

constexpr int FK_S1_BITS = 19;                  // stage 1: 2^19 bits = 64 KB
constexpr int FK_P2_WORDS = 2048;               // stage 1, 2-3 byte anchors: exact pair table, 8 KB
// Stage-2 table sizes (filter LDS 132 KiB with them; 17 / 14 / 14 before: config 4's 52k-name KB filled the
// 4-byte table, stage-2 survivors 24.6M -> 18.8M, probe 2.04 -> 1.77 ms, config 4 9.21 -> 8.91 ms, config 2
// unchanged; r05_stage2_tables_ab.txt)
#ifndef FK_L2_BITS_CFG
#define FK_L2_BITS_CFG 18
#endif
#ifndef FK_T3_BITS_CFG
#define FK_T3_BITS_CFG 16
#endif
#ifndef FK_B2_BITS_CFG
#define FK_B2_BITS_CFG 16
#endif
constexpr int FK_L2_BITS = FK_L2_BITS_CFG;      // stage 2, 4-byte keys: 32 KB
constexpr int FK_T3_BITS = FK_T3_BITS_CFG;      // stage 2, 3-byte keys: 8 KB
constexpr int FK_B2_BITS = FK_B2_BITS_CFG;      // stage 2, 2-byte keys: 8 KB (<= 16: fk_b2h_index)
static_assert(FK_B2_BITS <= 16, "fk_b2h_index takes the high bits of a 16-bit index");
constexpr int FK_EDGE_BITS = 20;                // edge prefix / suffix 8-byte keys: 2 x 128 KB (global, L2)
constexpr int FK_ITEMS0 = 512;                  // items of field 0 (text) on the fast path (power of 2: LDS sort)
constexpr int FK_ITEMS1 = 64;                   // items of field 1 (title)
constexpr int FK_ITEMS_MAX = FK_ITEMS0;         // one field's item buffer in the resolve kernel
constexpr int FK_BIG0 = 4096;                   // items of the text / title of a big document (epilogue:
constexpr int FK_BIG1 = 512;                    //   the workgroup's 36 KiB of LDS; resolve: FK_BIG0 per field)
constexpr int FK_CP_CAP = 16384;                // bytes of a non-ASCII field the fast path decodes
constexpr int RK_WAVES = 4;                     // waves per resolve workgroup
constexpr int RK_BLOCK = RK_WAVES * WAVE;
constexpr uint32_t FK_MUL1 = 0x9E3779u;         // 24-bit multiplier (v_mul_u32_u24)
constexpr uint32_t FK_MUL2 = 0x85EBCA6Bu;
constexpr uint32_t FK_MUL3 = 0xC2B2AE35u;
constexpr uint32_t FK_MUL4 = 0x27D4EB2Fu;

constexpr int FK_S1_WORDS = 1 << (FK_S1_BITS - 5);
constexpr uint32_t FK_S1_M1 = 0xD2511Fu;        // stage-1 hash multipliers (24 bits: v_mul_u32_u24 / v_mad_u32_u24)
constexpr uint32_t FK_S1_M2 = 0x9E3779u;
constexpr uint32_t FK_S1_EXT_MAX = 16384;       // stage-1 4-grams of the fuzzy 3-byte anchors (256 each)
constexpr int FK_L2_WORDS = 1 << (FK_L2_BITS - 5);
constexpr int FK_T3_WORDS = 1 << (FK_T3_BITS - 5);
constexpr int FK_B2_WORDS = 1 << (FK_B2_BITS - 5);
constexpr int FK_EDGE_WORDS = 1 << (FK_EDGE_BITS - 5);

// item kinds (2 bits).  3 is FU_RXM in the probe's items (a match of a quantifier-free regex name's program,
// '.' wildcards; ASCII fields) and FU_EDGE in the resolve kernel's lists, where an edge item's use is
// IT_USE_MASK (an RXM item's is a real use).
enum FastUseKind : uint32_t { FU_UPPER = 0, FU_FULL = 1, FU_PIECE = 2, FU_EDGE = 3, FU_RXM = 3 };

// how re.finditer(name) finds positions: literal search or the regex engine
enum RxKind : uint32_t { RXK_LITERAL = 0, RXK_REGEX = 1 };
constexpr uint32_t EDGE_MIN_M = 11, EDGE_MAX_M = 20;   // names with edge-only fuzzy windows

// per-document header written by the scan kernel (uint2):
//   x = index of the document's first item in FastScratch::items
//   y = n0 [7:0] | n1 [15:8] | flags
// document header .y: n0 (bits 0..9) | n1 << DH_N1_SHIFT (bits 10..16) | flags
constexpr uint32_t DH_N1_SHIFT = 10;
constexpr uint32_t DH_NEED = 1u << 17;          // the resolve kernel has work on this document
constexpr uint32_t DH_EDGE0 = 1u << 18;         // field 0: edge prefilter hit (prefix or suffix)
constexpr uint32_t DH_EDGE1 = 1u << 19;
constexpr uint32_t DH_NA0 = 1u << 20;           // field 0 has non-ASCII bytes
constexpr uint32_t DH_NA1 = 1u << 21;
constexpr uint32_t DH_DEFER = 1u << 22;         // sent to the generic kernel by the scan
constexpr uint32_t DH_TX = 1u << 23;            // finished by the epilogue on its transcoded view (hdr)
constexpr uint32_t DH_RESOLVE = 1u << 24;       // non-ASCII document left to the resolve kernel (dflags)
static_assert(FK_ITEMS0 < 1024 && FK_ITEMS1 < 128, "item counts must fit the document header");

struct FastTables {
    const uint32_t *s1;         // FK_S1_WORDS: the anchors' first four bytes (fk_s1_hash)
    const uint32_t *p2;         // FK_P2_WORDS: first two bytes of the 2-3 byte anchors (exact)
    const uint32_t *l2;         // FK_L2_WORDS
    const uint32_t *t3;         // FK_T3_WORDS
    const uint32_t *b2;         // FK_B2_WORDS
    const uint32_t *edge_pre;   // FK_EDGE_WORDS
    const uint32_t *edge_suf;   // FK_EDGE_WORDS
    int has_short;              // any 2- or 3-byte anchor in the stage-1 pair box
    uint32_t gate[6];           // the pair box: first byte {A, B, N}, second byte {A, B, N} (fk_in_box)
    int has_t3;                 // any 3-byte anchor
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
    const uint64_t *pat_bsig;   // bigram-set signature of the one-byte code points, 128 bits (fk_bg_bit)
    const int32_t *f_count_ge;
    const uint64_t *sub_key;
    const uint32_t *sub_begin;
    const uint32_t *sub_cnt;
    const uint32_t *sub_pat;
    uint32_t sub_mask;
    const uint64_t *edge_key;   // (hash of L code points + L * golden) | 1; 0 = empty
    const uint32_t *edge_begin;
    const uint32_t *edge_cnt;
    const uint32_t *edge_ent;   // pattern << 5 | deleted code-point index
    uint32_t edge_mask;
    const uint32_t *word_bits;
    int f_first;
    int empty_pat;
    const uint4 *ht4;           // probe records: {key lo, key hi, first arec, count} per slot
    const uint4 *arec;          // {head lo, head hi, first use, uses << 8 | len} (grouped by key)
    const uint4 *urec;          // {use_info0, use_info1, pattern, byte offset of the span in pat_bytes}
    const uint4 *urec2;         // {first 8 bytes of the span, last 8 bytes} (little endian, <= 8 when shorter)
    // quantifier-free regex names (literals and '.', <= 64 atoms): shift-and tables
    const int32_t *rxf_idx;     // per pattern: row r, or -1 (quantified: the backtracking engine)
    const uint64_t *rxf_pm;     // [r][128] ASCII masks ('.' bits except for '\n')
    const uint64_t *rxf_any;    // [r] '.' bits (masks of non-ASCII code points)
    const uint32_t *rxf_len;    // [r] atoms = match length in code points
    const uint32_t *rxf_ext_off;   // [r + 1] non-ASCII literal atoms
    const uint32_t *rxf_ext_cp;
    const uint64_t *rxf_ext_mask;
    // transcoded view of non-ASCII documents (one byte per code point: ASCII as is, the other code points of
    // the fuzzy names as markers 0x81..0xFF, every other code point 0x80)
    const uint32_t *pat_tcps;   // per pattern (pat_cp_off): code points with the non-ASCII ones as markers
    const uint8_t *pat_tbytes;  // the same, one byte each (names on lanes: short fields, verify)
    const uint32_t *tx_key;     // [256] non-ASCII code point -> tx_val (open addressing, ~0 = empty)
    const uint32_t *tx_val;
    const uint32_t *tx_inv;     // [128] marker - 0x80 -> code point (~0 for 0x80: no name holds it)
    int tx_unsafe_short;        // a name the view cannot decide (PI_TXUNSAFE) may decide a short field
    const uint32_t *txu_pat;    // those names (n_txu)
    uint32_t n_txu;
    int tx_unsafe_edge;         // ... or an edge window
    const uint64_t *use_wild;   // per use: wildcard positions of an RXM program string
    const uint32_t *pat_rxl;    // per pattern: its RXM program length (0: no RXM use; positions by the rx tasks)
};

struct FastScratch {
    uint64_t *items;            // per filter region: item_cap items (the probe's), indexed by 32-bit hdr.x
    uint32_t item_cap;          // regions x item_cap < 2^32 (launch_scan clamps it)
    uint32_t bigq;              // big documents an epilogue workgroup queues for itself (<= EK_BIGQ; more: resolve)
    uint32_t item_grow;         // 1: a region whose items overflow asks the host for larger regions (rescan);
                                // 0 (item_cap clamped): its batches' documents only defer to the generic kernel
    uint2 *hdr;                 // per document
    kw_hit *out;                // per resolve wave: out_cap records
    uint32_t *out_cnt;          // per resolve wave
    uint32_t out_cap;
    uint32_t *cps;              // per resolve wave: FK_CP_CAP decoded code points (non-ASCII fields)
    uint32_t *cpbase;           // per resolve wave: cumulative lead counts per 64-byte block
    uint32_t *defer_list;       // docs sent to the generic kernel
    uint32_t *defer_cnt;
    uint32_t defer_cap;
    uint32_t *big_list;         // non-ASCII docs with more items than the resolve kernel holds (defer_cap; filled
    uint32_t *big_cnt;          //   from the tail end, count in big_cnt[1])
    uint32_t *status;
    unsigned long long *stats;  // see kw_stats
    uint4 *rx_tasks;            // per resolve wave: rx_cap regex-position tasks (doc, field|ascii, pattern, n)
    uint32_t rx_cap;
    // flat resolve of all-ASCII documents (scan epilogue -> task kernel)
    kw_hit *kout;               // per scan wave: out_cap records (hits the scan epilogue emits)
    uint32_t *kout_cnt;
    kw_hit *tout;               // per task wave: out_cap records
    uint32_t *tout_cnt;
    uint4 *vq, *eq, *sq, *xq;   // per scan wave: verify / edge / short / regex task regions
    uint32_t vcap, ecap, scap, xcap;
    uint32_t *vcnt, *ecnt, *scnt, *xcnt;   // per scan wave
    uint32_t *xmark;            // per scan wave: the regex tasks the epilogue queued (xcnt after it; KW_RX_SPLIT)
    uint32_t *tmax;             // [4] largest task count a wave needed (rescan sizing)
    unsigned long long *dset;   // decided (doc, field, pattern) set: open addressing, 0 = empty
    unsigned long long dmask;
    // split scan (kwmatch_split.hpp): filter regions -> candidates -> items
    uint32_t *cand;                // per filter region: cand_cap records (group headers, candidates: kwmatch_split.hpp)
    uint32_t cand_cap;
    uint32_t *ccnt;             // per filter region: candidates written
    uint2 *ncnt;                // per document: items of field 0 / field 1 (the probe adds them up)
    uint32_t *dflags;           // per document: DH_NA0 / DH_NA1 (the filter ORs them in) and DH_DEFER (probe)
    uint32_t *cmax;             // [2] largest candidate / item count a region needed (rescan sizing)
    // the epilogue's transcoded view of non-ASCII documents
    uint8_t *tarena;            // tx_cap bytes, bump-allocated per document (tx_used)
    unsigned long long tx_cap;
    unsigned long long *tx_used;
    uint4 *vrec;                // per document: {text start lo, hi | transcoded << 31, text / title code points}
    uint32_t *res_list;         // documents the epilogue left to the resolve kernel (DH_RESOLVE; defer_cap)
    uint32_t *res_cnt;
    // dynamic work distribution: [0] the filter's next work unit (chunk of groups), [1] the probe's next region
    // (zeroed per scan);
    // dyn = 0: grid-stride groups (KW_STATIC_GROUPS=1)
    uint32_t *gnext;
    int dyn;
    int64_t chunk_groups;       // groups per filter work unit = candidate region (kwmatch_split.hpp)
};

// the next group a wave takes: grid-stride (g += n_waves) or, with S.dyn, the next one of a per-kernel counter
// (groups of uneven cost then end together; a wave's groups still ascend)
__device__ __forceinline__ int64_t fk_next_group(uint32_t *ctr, bool dyn, int64_t g, int64_t n_waves)
{
    if (!dyn) return g + n_waves;
    uint32_t v = 0;
    if (lane_id() == 0) v = atomicAdd(ctr, 1u);
    return (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// host + device hashes of the LDS tables
// stage 1: the 4-gram b0..b3 at a position as k4 = b0 | b1 << 8 | b2 << 16 | b3 << 24; h = (b0..b2) * M1 +
// (b1..b3) * M2 (a v_mul_u32_u24 and a v_mad_u32_u24; the one-multiply form h = (k4 mod 2^24) * M1 + k4 was
// measured in round 5 and dropped: its bit index sees only b0's low 5 bits).  Word h >> 18 of the table, bit h & 31.
__host__ __device__ __forceinline__ uint32_t fk_s1_hash(uint32_t k4)
{
    return (k4 & 0xFFFFFFu) * FK_S1_M1 + ((k4 >> 8) & 0xFFFFFFu) * FK_S1_M2;
}
__host__ __device__ __forceinline__ uint32_t fk_s1_word(uint32_t h) { return h >> (32 - FK_S1_BITS + 5); }
__device__ __forceinline__ uint32_t lds_word_at(const uint32_t *t, uint32_t byte_off)
{
    return *(const uint32_t *)((const uint8_t *)t + byte_off);
}
__host__ __device__ __forceinline__ uint32_t fk_l2_index(uint32_t key4) { return (key4 * FK_MUL2) >> (32 - FK_L2_BITS); }
__host__ __device__ __forceinline__ uint32_t fk_t3_index(uint32_t key4)
{
    return ((key4 & 0xFFFFFFu) * FK_MUL3) >> (32 - FK_T3_BITS);
}
__host__ __device__ __forceinline__ uint32_t fk_edge_index(uint64_t key8)
{
    return (uint32_t)((key8 * 0x9E3779B97F4A7C15ull) >> (64 - FK_EDGE_BITS));
}
// bigram signature bit (0..127) of two one-byte code points (the short kernel's second filter)
__host__ __device__ __forceinline__ uint32_t fk_bg_bit(uint32_t a, uint32_t b)
{
    return ((((a & 0xFFu) << 8) | (b & 0xFFu)) * 40503u >> 9) & 127u;
}
__host__ __device__ __forceinline__ uint32_t fk_b2_index(uint32_t key2)
{
    return ((key2 & 0xFFFFu) * 40503u) & 0xFFFFu;     // bijection on 16 bits (odd multiplier): the exact pair table
}
__host__ __device__ __forceinline__ uint32_t fk_b2h_index(uint32_t key2) { return fk_b2_index(key2) >> (16 - FK_B2_BITS); }
__host__ __device__ __forceinline__ uint32_t fk_ht_slot(uint64_t k, uint32_t mask)
{
    uint64_t x = k * 0x9E3779B97F4A7C15ull;
    return (uint32_t)(x >> 40) & mask;
}

}  // namespace kw
