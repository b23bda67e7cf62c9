// libkwmatch: CDX link-row normalise + keep-first dedup (include/kwdedup.h).
//
// Reference: yahoo_links_selenium.py:63-79 (per part) and :160-174 (merge);
// restated in oracle/dedup_oracle.py.
//
//   dd_transform_kernel  lane = row over the wave's 64 rows, staged in LDS by
//                        LDS-DMA; groups of 64 rows claimed 8 at a time, so
//                        rows enter the table in about row order.  Finds the
//                        cut (first "html" after a code point that is not
//                        '\n'; a staged row scanned 8 bytes a step with 32-bit
//                        offsets), plans the rewrite of the prefix (':80'
//                        removed, 'http:' -> 'https:', ".html" appended),
//                        flags 'news/%' / "news/'", and hashes the normalised
//                        words (one 64-bit hash: tag and slot).  Nothing of
//                        the normalised URL is stored: a row keeps a 16-byte
//                        descriptor (raw start, length, cut, 's' insertion,
//                        the one ':80' gap) from which later kernels
//                        regenerate its words from the raw bytes (NormRow,
//                        RowGen).  Rows with other extra ':' run the
//                        byte-serial rewrite (dd_slow_kernel) into a small
//                        slow-row arena.  Each kept row is inserted at once
//                        (table_insert): slots {24-bit tag, 8-bit run epoch,
//                        row}, the first inserter claims a slot by CAS, an
//                        earlier row displaces the holder by atomicMin
//                        (keep='first'); a row that finds an earlier holder
//                        lists the pair (row, holder), a displacing row lists
//                        (holder, row), in its claim's own segment.
//   dd_pairs_kernel      a pair's later row is a duplicate iff its normalised
//                        bytes equal the earlier row's (4 lanes a pair, the
//                        descriptors handed out by shuffles).  A differing
//                        pair's later row is compared with its tag's first row
//                        from the table (dd_recheck_kernel); rows that share a
//                        tag with a different URL are listed and resolved
//                        exactly on the host.
//   dd_count / dd_tile_sums / dd_scan_tiles / dd_place / dd_copy_staged
//                        dense offsets (a two-level tile scan), source rows
//                        and bytes of the kept rows (32 kept rows a wave, their
//                        raw span staged by LDS-DMA, words regenerated from
//                        LDS into an output stage, aligned 16-byte stores).
//
// All byte/integer work: the roofline is HBM bandwidth; the table's random
// atomics bound the insert.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/kwmatch.h"
#include "../../include/kwdedup.h"
#include "kwenv.hpp"

namespace dd {

constexpr int BLOCK = 256;
constexpr int SCAN_ROWS = 4;                       // rows per thread in the scan kernels
constexpr int SCAN_TILE = BLOCK * SCAN_ROWS;
constexpr int SCAN_CHUNKS = 512;                   // chunks of tiles in the two-level tile scan
constexpr uint32_t HTML4 = 0x6C6D7468u;            // "html"
constexpr uint32_t NEWS4 = 0x7377656Eu;            // "news"
constexpr uint64_t DOTHTML = 0x6C6D74682Eull;      // ".html"
constexpr uint8_t CODE_COLLIDE = 4;                // internal: tag shared with a different URL
constexpr uint32_t COLLIDE_CAP = 1u << 16;         // CODE_COLLIDE rows listed by the recheck kernel

constexpr uint32_t NO_HINT = 0xFFFFFFFFu;         // a kept row that took its tag's slot
constexpr uint32_t SLOW_ROW = 0xFFFFFFFFu;        // plan.x of a byte-serial row (plan.y: its slow-arena word)
constexpr uint32_t NO_GAP = 0x7FFFFFFFu;          // plan.y bits 0..30 without a ':80' gap
constexpr uint32_t LEN_BIG = 0xFFFFFFu;           // rowd's 24-bit length field of a longer row (len3 holds it)
// a table slot: the hash's high 24 bits (tag) | the run's epoch (8 bits; another epoch: empty) | the row + 1

__device__ __forceinline__ uint32_t ld32(const uint8_t *__restrict__ a, int64_t p)
{
    const int64_t a0 = p & ~(int64_t)3;
    const uint32_t x0 = *(const uint32_t *)(a + a0);
    const uint32_t x1 = *(const uint32_t *)(a + a0 + 4);
    return __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)(p & 3));
}

__device__ __forceinline__ uint64_t ld64(const uint8_t *__restrict__ a, int64_t p)
{
    const int64_t a0 = p & ~(int64_t)3;
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t x0 = *(const uint32_t *)(a + a0);
    const uint32_t x1 = *(const uint32_t *)(a + a0 + 4);
    const uint32_t x2 = *(const uint32_t *)(a + a0 + 8);
    return (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s) << 32);
}

__device__ __forceinline__ uint32_t eq_bytes(uint32_t v, uint32_t pat)   // 0x80 in exactly the bytes equal to pat's
{
    const uint32_t d = v ^ pat;
    return ~(((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
}

__host__ __device__ __forceinline__ uint64_t mix1(uint64_t h, uint64_t w)
{
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 32);
}
__host__ __device__ __forceinline__ uint64_t fmix(uint64_t h)
{
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    return h ^ (h >> 33);
}

struct Scratch {
    uint4 *rowd;             // per kept row, what RowGen needs in one 16-byte load: x, y[7:0] = the raw start
                             //   (40 bits), y[31:8] = the normalised length (LEN_BIG: see len3); z, w = the plan:
                             //   z = the cut j (raw: the length; SLOW_ROW), w = 's' insertion << 31 | the ':80'
                             //   gap's raw position (NO_GAP) (a slow row: its slow-arena word)
    uint32_t *len3;          // per row: normalised length
    unsigned long long *table;
    uint2 *pairs;            // (row, an earlier row with its tag) of every kept row that found one, listed per
                             //   claim of TCLAIM groups: claim c's pairs at [c * 64 * TCLAIM, + pcount[c])
    uint32_t *pcount;        // pairs per claim
    uint32_t *recheck;       // rows compared with their tag's first row from the table (cnt[5] listed)
    uint32_t *collide;       // the CODE_COLLIDE rows (cnt[9] listed; a list longer than COLLIDE_CAP: the host
                             //   finds them by a scan of the codes)
    uint64_t mask;
    uint32_t epoch;          // this run's table epoch (1..255): a slot of another epoch is empty, so the table is
                             //   cleared only when it moves, grows or the epoch wraps (the memset cost 1.4 ms a run)
    unsigned long long *cnt;   // [0], [2], [3], [4]: rows per code but KEPT; [5] differing pairs;
                               // [7] the transform's next group of 64 rows; [9] CODE_COLLIDE rows listed
    unsigned long long *gnext;   // &cnt[7]
    int weak;                // tests: hash h1 down to 4 bits (forces the collision path)
    int stats;               // KW_DEDUP_STATS: print the differing pairs (rows looked up in the table)
    int normalize;           // KW_DEDUP_NORMALIZE: apply :63-76; else keep-first over the raw strings
    uint2 *slow;             // rows (index, cut) for the byte-serial rewrite (capacity: every row)
    unsigned long long *nslow;   // [0] slow rows listed, [1] slow-arena words they may need, [2] words handed out
    uint64_t *sarena;        // the slow rows' normalised words (sized after the transform from nslow[1])
};

// byte-serial writer of the normalised URL: 8-byte words to the sparse arena + hashes + filter window
struct Emit {
    uint64_t w, win, h1;
    int64_t pos, len;
    int nb;
    bool bad;
    uint8_t *out;
    __device__ __forceinline__ void put(uint32_t c)
    {
        w |= (uint64_t)c << (8 * nb);
        ++nb;
        ++len;
        win = (win << 8) | c;
        const uint64_t w6 = win & 0xFFFFFFFFFFFFull;
        // 'news/%' and "news/'" (newest byte lowest)
        bad |= w6 == 0x6E6577732F25ull || w6 == 0x6E6577732F27ull;
        if (nb == 8) {
            *(uint64_t *)(out + pos) = w;
            h1 = mix1(h1, w);
            pos += 8;
            w = 0;
            nb = 0;
        }
    }
    __device__ __forceinline__ void finish()
    {
        if (nb) {
            *(uint64_t *)(out + pos) = w;
            h1 = mix1(h1, w);
        }
    }
};

// the reference's rewrite of the cut prefix u[0, j): ':80' removed (left to right), then 'http:' -> 'https:'
struct Rewrite {
    uint32_t P;
    int np;           // pending bytes of the ':80' window
    uint64_t Q;
    int nq;           // pending bytes of the 'http:' window
    __device__ __forceinline__ void h_push(Emit &E, uint32_t c)
    {
        Q |= (uint64_t)c << (8 * nq);
        if (++nq == 5) {
            if (Q == 0x3A70747468ull) {    // "http:"
                E.put('h'); E.put('t'); E.put('t'); E.put('p'); E.put('s'); E.put(':');
                Q = 0;
                nq = 0;
            } else {
                E.put((uint32_t)(Q & 0xFF));
                Q >>= 8;
                nq = 4;
            }
        }
    }
    __device__ __forceinline__ void r_push(Emit &E, uint32_t c)
    {
        P |= c << (8 * np);
        if (++np == 3) {
            if (P == 0x30383Au) {          // ":80"
                P = 0;
                np = 0;
            } else {
                h_push(E, P & 0xFF);
                P >>= 8;
                np = 2;
            }
        }
    }
    __device__ __forceinline__ void flush(Emit &E)
    {
        while (np) { h_push(E, P & 0xFF); P >>= 8; --np; }
        while (nq) { E.put((uint32_t)(Q & 0xFF)); Q >>= 8; --nq; }
    }
};

// row bytes from the arena in global memory, or from the wave's LDS copy of its rows
struct GlobalSrc {
    const uint8_t *a;
    __device__ __forceinline__ uint32_t ld32(int64_t p) const { return dd::ld32(a, p); }
    __device__ __forceinline__ uint64_t ld64(int64_t p) const { return dd::ld64(a, p); }
};
struct LdsSrc {
    const uint32_t *w;   // staged words; byte p of the arena is byte p - base of the stage
    int64_t base;
    __device__ __forceinline__ uint32_t ld32(int64_t p) const
    {
        const int64_t q = p - base;
        const int k = (int)(q >> 2);
        return __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)(q & 3));
    }
    __device__ __forceinline__ uint64_t ld64(int64_t p) const
    {
        const int64_t q = p - base;
        const int k = (int)(q >> 2);
        const uint32_t s = (uint32_t)(q & 3), x0 = w[k], x1 = w[k + 1], x2 = w[k + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s) << 32);
    }
};

// Open-addressing table of 64-bit slots {tag, epoch, row}: the first inserter of a tag claims a slot by CAS, an earlier
// row (smaller index) displaces the holder by atomicMin, so the slot ends with the tag's first row
// (keep='first').  Every kept row returns at most one pair (later row, earlier row) of its tag to compare: (row,
// the earlier holder it found), or (the holder, row) when it displaced the holder (each row leaves its slot at
// most once, so every row that took a slot and is not its tag's first row gets exactly one such pair);
// (row, NO_HINT) when it took an empty slot.
// The plain load is only a hint of the slot (a slot's tag never changes once claimed; its row only decreases);
// it also spares a duplicate whose holder is already visible any atomic (CAS first on every probe: transform
// 34.3 -> 42.2 ms at 500M rows — the table's atomics, not its loads, bound the insert).
// Nothing another row wrote in this kernel is read (no cross-XCD visibility is assumed): the pair and recheck
// kernels read the pairs, bits and plans after the kernel boundary.
__device__ __forceinline__ uint2 table_insert(const Scratch &S, uint64_t h, int64_t i)
{
    // slot = the hash's high 24 bits (tag) | the epoch (8 bits) | the row + 1
    const unsigned long long key = ((h >> 40) << 40) | ((uint64_t)S.epoch << 32) | (uint64_t)((uint32_t)i + 1u);
    uint64_t slot = (h ^ (h >> 29)) & S.mask;
    unsigned long long cur = S.table[slot];
    uint2 pr = make_uint2((uint32_t)i, NO_HINT);
    for (;;) {
        if (((cur >> 32) & 0xFFu) != S.epoch) {   // empty (another run's or never written)
            const unsigned long long got = atomicCAS(&S.table[slot], cur, key);
            if (got == cur) break;
            cur = got;
            continue;   // claimed meanwhile: look at the claimer
        }
        if ((cur >> 32) == (key >> 32)) {
            if (cur > key) {
                cur = atomicMin(&S.table[slot], key);
                if (cur > key) {   // displaced the holder
                    pr = make_uint2((uint32_t)cur - 1u, (uint32_t)i);
                    break;
                }
            }
            pr.y = (uint32_t)cur - 1u;
            break;
        }
        slot = (slot + 1) & S.mask;
        cur = S.table[slot];
    }
    return pr;
}

// finish a row: hash, length, code; a kept row goes into the table (returns its pair)
__device__ __forceinline__ uint2 finish_row(uint64_t h1, int64_t len3, bool bad, int64_t i,
                                               uint8_t *__restrict__ code, const Scratch &S, int64_t b, uint2 pl)
{
    h1 = fmix(h1 ^ (uint64_t)len3);
    if (S.weak) h1 &= 0xFull;
    S.len3[i] = (uint32_t)len3;
    const uint32_t l24 = len3 < (int64_t)LEN_BIG ? (uint32_t)len3 : LEN_BIG;
    S.rowd[i] = make_uint4((uint32_t)b, (uint32_t)((uint64_t)b >> 32) | (l24 << 8), pl.x, pl.y);
    code[i] = bad ? (uint8_t)KW_URL_FILTERED : (uint8_t)KW_URL_KEPT;
    return bad ? make_uint2((uint32_t)i, NO_HINT) : table_insert(S, h1, i);
}

// slow-arena words a byte-serial row of cut j may need (one extra 's' per 5 bytes, ".html", a partial word)
__host__ __device__ __forceinline__ uint64_t slow_words(int64_t j) { return (uint64_t)((j + j / 5 + 5 + 7) / 8 + 1); }

// the general rewrite of the cut prefix u[0, j), byte by byte (rows with ':80' or a second 'http:'), into the
// slow arena
__device__ uint2 slow_row(const uint8_t *__restrict__ arena, int64_t b, int64_t j, int64_t i,
                             uint8_t *__restrict__ code, const Scratch &S)
{
    const unsigned long long w0 = atomicAdd(&S.nslow[2], (unsigned long long)slow_words(j));
    Emit Em;
    Em.w = 0; Em.win = 0; Em.h1 = 0x243F6A8885A308D3ull;
    Em.pos = 0; Em.len = 0; Em.nb = 0; Em.bad = false; Em.out = (uint8_t *)(S.sarena + w0);
    Rewrite R;
    R.P = 0; R.np = 0; R.Q = 0; R.nq = 0;
    for (int64_t t = 0; t < j; t += 4) {
        const uint32_t x = ld32(arena, b + t);
        const int m = (int)(j - t < 4 ? j - t : 4);
        for (int k = 0; k < m; ++k) R.r_push(Em, (x >> (8 * k)) & 0xFFu);
    }
    R.flush(Em);
    Em.put('.'); Em.put('h'); Em.put('t'); Em.put('m'); Em.put('l');
    Em.finish();
    const uint2 pr = finish_row(Em.h1, Em.len, Em.bad, i, code, S, b, make_uint2(SLOW_ROW, (uint32_t)w0));
    if (Em.bad) atomicAdd(&S.cnt[KW_URL_FILTERED], 1ull);   // (rare rows: one atomic each)
    return pr;
}

// The normalised words of a row of the fast path, from its raw bytes and its plan: the prefix u[0, j) with
// "https" for a leading "http:" (ins), minus at most one ':80' (the gap G, in normalised coordinates), then
// ".html" at E.  Used by the transform (to hash) and by decide / the copy / the host's exact pass (to compare
// and write): one definition of the normalised bytes.
template <class Src>
struct FastWords {
    const Src &src;
    int64_t b, G, E;
    int ins;
    __device__ __forceinline__ uint64_t body(int64_t x) const   // bytes [x, x + 8) of the prefix, x < E, x % 8 == 0
    {
        uint64_t w = (ins && x == 0) ? 0x7370747468ull | (src.ld64(b + 4) << 40)   // "https" + u[4..7)
                                     : src.ld64(b + x - ins + (x >= G ? 3 : 0));
        if (x < G && G < x + 8) {
            const int k = (int)(G - x) * 8;
            w = (w & ((1ull << k) - 1)) | (src.ld64(b + G - ins + 3) << k);
        }
        return w;
    }
    __device__ __forceinline__ uint64_t splice(uint64_t w, int64_t x) const   // ".html" at E, zeros after it
    {
        if (E < x + 8) {
            if (E >= x) {
                const int sh = (int)(E - x) * 8;
                w = (sh ? (w & ((1ull << sh) - 1)) : 0ull) | (DOTHTML << sh);
            } else {
                const int64_t d = x - E;
                w = d < 8 ? DOTHTML >> (8 * d) : 0ull;
            }
        }
        return w;
    }
    __device__ __forceinline__ uint64_t word(int64_t x) const { return splice(x < E ? body(x) : 0ull, x); }
};

// Any kept row's normalised words, regenerated (RowGen::word: 8-aligned x; zeros past the length)
struct RowGen {
    const uint8_t *a;
    const uint64_t *sw;   // a slow row's words
    int64_t b, G, E;
    uint32_t len;
    int ins, raw;
    __device__ __forceinline__ void init(const Scratch &S, const uint8_t *arena, uint4 r, int64_t i)
    {
        uint32_t l = r.y >> 8;
        if (l == LEN_BIG) l = S.len3[i];
        init_len(S, arena, r, l);
    }
    // from the descriptor and the resolved length (descriptors handed between lanes)
    __device__ __forceinline__ void init_len(const Scratch &S, const uint8_t *arena, uint4 r, uint32_t l)
    {
        const uint2 pl = make_uint2(r.z, r.w);
        a = arena;
        b = (int64_t)(((uint64_t)(r.y & 0xFFu) << 32) | r.x);
        len = l;
        raw = !S.normalize;
        sw = (!raw && pl.x == SLOW_ROW) ? S.sarena + pl.y : nullptr;
        ins = (int)(pl.y >> 31);
        const uint32_t ec = pl.y & NO_GAP;
        const bool gap = ec != NO_GAP;
        G = gap ? (int64_t)ec + ins : INT64_MAX / 2;
        E = (int64_t)pl.x + ins - (gap ? 3 : 0);
    }
    __device__ __forceinline__ uint64_t word(int64_t x) const
    {
        if (x >= (int64_t)len) return 0ull;
        if (sw) return sw[x >> 3];
        if (raw) {
            const uint64_t w = ld64(a, b + x);
            return len - x >= 8 ? w : w & ((1ull << (8 * (len - x))) - 1);
        }
        const GlobalSrc src{a};
        const FastWords<GlobalSrc> F{src, b, G, E, ins};
        return F.word(x);
    }
    __device__ __forceinline__ uint32_t byte(int64_t y) const { return (uint32_t)(word(y & ~(int64_t)7) >> (8 * (y & 7))) & 0xFFu; }
};

// one row: returns -1 when done, or the cut j of a row that needs slow_row; `pair` gets finish_row's
template <class Src>
__device__ __forceinline__ int64_t transform_row(const Src &src, int64_t b, int64_t L, int64_t i,
                                                 uint8_t *__restrict__ code, const Scratch &S, uint2 &pair)
{
    if (!S.normalize) {
        // raw keep-first (the merge step :174 over already normalised rows): the key is the string itself
        uint64_t h1 = 0x243F6A8885A308D3ull;
        for (int64_t x0 = 0; x0 < L; x0 += 8) {
            uint64_t w = src.ld64(b + x0);
            if (L - x0 < 8) w &= (1ull << (8 * (L - x0))) - 1;
            h1 = mix1(h1, w);
        }
        pair = finish_row(h1, L, false, i, code, S, b, make_uint2((uint32_t)L, NO_GAP));
        return -1;
    }
    // ---- pass 1: the cut j, the first two extra ':' and the first 'news/%' | "news/'" end, one 4-byte word a
    // step with per-byte masks and no per-event loops (every event kind happens in some lane of nearly every
    // step, so per-event loops ran in nearly every step); only the rare '%' / "'" bytes take a loop
    int64_t j = -1, ec = INT64_MAX, ec2 = INT64_MAX, kf = INT64_MAX;   // ec / ec2: first two extra ':'
    bool scheme_http = false;
    uint32_t excl = 0;   // the scheme's ':' (q == 4 of "http:", q == 5 of "https:", neither starting ':80')
    if (L >= 5 && src.ld32(b) == 0x70747468u) {
        const uint32_t w4 = src.ld32(b + 4);
        if ((w4 & 0xFFu) == 0x3Au && !(L >= 7 && (w4 & 0xFFFFFFu) == 0x30383Au)) { scheme_http = true; excl = 0x80u; }
        if (L >= 6 && (w4 & 0xFFFFu) == 0x3A73u && !(L >= 8 && (w4 >> 8) == 0x30383Au)) excl = 0x8000u;
    }
    uint32_t x = src.ld32(b), xp = 0;
    for (int64_t t = 0; t < L; t += 4) {
        const uint32_t y = src.ld32(b + t + 4);
        const int64_t r = L - t;
        const uint32_t in = r >= 4 ? 0x80808080u : 0x80808080u & ((1u << (8 * r)) - 1u);   // positions < L
        // extra colons: the first two positions (all new positions lie past the recorded ones)
        uint32_t cm = eq_bytes(x, 0x3A3A3A3Au) & in;
        if (t == 4) cm &= ~excl;
        if (cm) {   // rare once the scheme's ':' is masked out
            const uint32_t cm1 = cm & (cm - 1u);
            const int64_t c0 = t + (__builtin_ctz(cm) >> 3);
            const int64_t c1 = cm1 ? t + (__builtin_ctz(cm1) >> 3) : INT64_MAX;
            ec2 = ec == INT64_MAX ? c1 : (ec2 == INT64_MAX ? c0 : ec2);
            ec = ec == INT64_MAX ? c0 : ec;
        }
        // 'news/%' | "news/'": from the (rare) '%' / "'" byte p back to its "news/" (kf = p = q + 5)
        uint32_t pm = eq_bytes(x | 0x02020202u, 0x27272727u) & in;   // '%' (0x25) and "'" (0x27) differ in bit 1 only
        while (pm) {
            const int64_t p = t + (__builtin_ctz(pm) >> 3);
            pm &= pm - 1u;
            if (p >= 5 && p < kf && src.ld32(b + p - 5) == NEWS4 && (src.ld32(b + p - 1) & 0xFFu) == 0x2Fu) kf = p;
        }
        // "html" at q with q >= 1, q + 4 <= L and no '\n' before it
        uint32_t hm = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) hm |= __builtin_amdgcn_alignbyte(y, x, k) == HTML4 ? 0x80u << (8 * k) : 0u;
        if (hm) {   // (once a row, at its end) validate: q + 4 <= L, q >= 1, no '\n' before q
            const int64_t r3 = r - 3;
            hm &= r3 >= 4 ? 0x80808080u : (r3 <= 0 ? 0u : 0x80808080u & ((1u << (8 * r3)) - 1u));
            hm &= ~eq_bytes(__builtin_amdgcn_alignbyte(x, xp, 3), 0x0A0A0A0Au);
            if (t == 0) hm &= ~0x80u;
        }
        if (hm) {
            const int64_t q = t + (__builtin_ctz(hm) >> 3);
            // the code point before "html" starts at its lead byte
            int64_t s = q - 1;
            if ((src.ld32(b + s) & 0xFFu) >= 0x80u) {
                while (s > 0 && (src.ld32(b + s) & 0xC0u) == 0x80u && q - s < 4) --s;
            }
            j = s;
            break;
        }
        xp = x;
        x = y;
    }
    if (j < 0) {
        code[i] = KW_URL_NO_HTML;
        S.len3[i] = 0;
        return -1;
    }
    const bool gap = ec < j;
    if (gap && !(ec2 >= j && ec > 5 && ec + 3 <= j && (src.ld32(b + ec) & 0xFFFFFFu) == 0x30383Au))
        return j;   // the byte-serial rewrite runs in dd_slow_kernel, off the divergent path
    // ---- fast path: the prefix u[0, j) minus at most one ':80' after the scheme (a splice with one gap at
    // G; with no other extra ':' left neither a new ':80' nor a new 'http:' can form), 'http:' -> 'https:'
    // at the scheme, ".html" at E.  Every lane runs the same word loop; only the filter window across the
    // gap is extra work for the gap rows
    const int ins = (scheme_http && j > 4) ? 1 : 0;
    const int64_t G = gap ? ec + ins : INT64_MAX / 2, E = j + ins - (gap ? 3 : 0);
    const int64_t len3 = E + 5;
    const FastWords<Src> F{src, b, G, E, ins};
    bool jn = false;
    if (gap) {
        // 'news/%' | "news/'" across the gap: windows starting at G - 5 .. G - 1 (G >= 6)
        auto seg1 = [&](int64_t x) -> uint64_t {   // bytes [x, x + 8) of u[0, ec) after the 's' insertion
            if (!ins) return src.ld64(b + x);
            if (x >= 5) return src.ld64(b + x - 1);
            const uint64_t h0 = 0x7370747468ull | (src.ld64(b + 4) << 40);
            return x ? (h0 >> (8 * x)) | (src.ld64(b + 7) << (64 - 8 * x)) : h0;
        };
        auto nword = [&](int64_t x) -> uint64_t {
            uint64_t w = 0;
            if (x < E) {
                if (x + 8 <= G) w = seg1(x);
                else if (x >= G) w = src.ld64(b + x - ins + 3);
                else {
                    const int k = (int)(G - x) * 8;
                    w = (seg1(x) & ((1ull << k) - 1)) | (src.ld64(b + G - ins + 3) << k);
                }
            }
            return F.splice(w, x);
        };
        const uint64_t lo = nword(G - 5), hi = nword(G + 3);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint64_t win = ((lo >> (8 * k)) | (k ? hi << (64 - 8 * k) : 0ull)) & 0xFFFFFFFFFFFFull;
            jn |= win == 0x252F7377656Eull || win == 0x272F7377656Eull;
        }
    }
    const bool bad = kf < j || jn;
    uint64_t h1 = 0x243F6A8885A308D3ull;
    for (int64_t x0 = 0; x0 < len3; x0 += 8) h1 = mix1(h1, F.word(x0));
    pair = finish_row(h1, len3, bad, i, code, S, b,
                      make_uint2((uint32_t)j, ((uint32_t)ins << 31) | (gap ? (uint32_t)ec : NO_GAP)));
    return -1;
}

constexpr int STAGE_BYTES = 8192;   // per-wave LDS copy of the wave's 64 rows
#ifndef DD_STEP8
#define DD_STEP8 1                  // transform_row_lds's scan: 8 bytes a step (0: 4)
#endif

// A wave's 16-byte chunks [0, nch) of src into its LDS stage by LDS-DMA (global_load_lds_dwordx4: 64 chunks
// an instruction, every instruction issued before the one wait; no VGPRs).  A loop of load-then-store waited
// for each of its ~6 loads in turn, and staging through registers all at once spilled.  Lanes past nch re-read
// the last chunk (their LDS bytes lie inside the stage, past what is read).
typedef __attribute__((address_space(1))) const void gmem_void;
typedef __attribute__((address_space(3))) void lds_void;
__device__ __forceinline__ void stage_dma(uint4 *stage, const uint8_t *__restrict__ src, int nch)
{
    const int lane = threadIdx.x & 63;
    for (int u = 0; 64 * u < nch; ++u) {
        const int c = 64 * u + lane;
        const int cc = c < nch ? c : nch - 1;
        __builtin_amdgcn_global_load_lds((gmem_void *)(src + 16 * (int64_t)cc), (lds_void *)(stage + 64 * u), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A row in the wave's LDS stage, addressed from its start with 32-bit offsets: the row starts at byte s of stage
// dword k0 (dw(k) = the row's k-th aligned dword)
struct LdsRow {
    const uint32_t *w;
    int k0;
    uint32_t s;
    __device__ __forceinline__ uint32_t dw(int k) const { return w[k0 + k]; }
    __device__ __forceinline__ uint32_t ld32(int p) const
    {
        const int q = p + (int)s, k = k0 + (q >> 2);
        return __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)(q & 3));
    }
    __device__ __forceinline__ uint64_t ld64(int p) const
    {
        const int q = p + (int)s, k = k0 + (q >> 2);
        const uint32_t sh = (uint32_t)(q & 3), x0 = w[k], x1 = w[k + 1], x2 = w[k + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sh) << 32);
    }
};

// transform_row for a staged row (normalising runs; the common case), with 32-bit offsets: the same plan, hash
// and codes.  Pass 1 reads one aligned dword a step (the rolling pair of dwords gives the unaligned window) and
// masks nothing by the row's end but the "html" candidates: an extra ':' or a 'news/%' end found at or past the
// end lies past any cut (j < L), where it changes nothing (gap needs ec < j, the filter kf < j; ec2 only matters
// as ec2 >= j).  The hash reads each normalised word with one 3-dword LDS window.
__device__ __forceinline__ int64_t transform_row_lds(const LdsRow &R, int L, int64_t i, int64_t b,
                                                     uint8_t *__restrict__ code, const Scratch &S, uint2 &pair)
{
    constexpr int NONE = 0x7FFFFFFF;
    int j = -1, ec = NONE, ec2 = NONE, kf = NONE;
    bool scheme_http = false;
    uint32_t excl = 0;   // the scheme's ':' (as transform_row)
    if (L >= 5 && R.ld32(0) == 0x70747468u) {
        const uint32_t w4 = R.ld32(4);
        if ((w4 & 0xFFu) == 0x3Au && !(L >= 7 && (w4 & 0xFFFFFFu) == 0x30383Au)) { scheme_http = true; excl = 0x80u; }
        if (L >= 6 && (w4 & 0xFFFFu) == 0x3A73u && !(L >= 8 && (w4 >> 8) == 0x30383Au)) excl = 0x8000u;
    }
#if DD_STEP8
    // 8 bytes a step (x = bytes [t, t + 4), x2 = [t + 4, t + 8), y = [t + 8, t + 12)): the loop's control, its
    // branches' tests and the dword reads (two a step, read a step ahead) are paid once per 8 bytes.  The scan
    // stops at any "html" at q in [t, t + 8); the candidates are validated out of the loop (q >= 1, q + 4 <= L,
    // no '\n' before q), first those in [t, t + 4), and a step without a valid one resumes the scan
    uint32_t d1 = R.dw(1), d2 = R.dw(2);   // the aligned dwords under x2 (and y) at a step's start
    uint32_t x = __builtin_amdgcn_alignbyte(d1, R.dw(0), R.s), xp = 0, x2 = 0, y = 0;
    int t = 0, k = 3;
    auto colons = [&](uint32_t cm, int tt) {
        const uint32_t cm1 = cm & (cm - 1u);
        const int c0 = tt + (__builtin_ctz(cm) >> 3);
        const int c1 = cm1 ? tt + (__builtin_ctz(cm1) >> 3) : NONE;
        ec2 = ec == NONE ? c1 : (ec2 == NONE ? c0 : ec2);
        ec = ec == NONE ? c0 : ec;
    };
    auto filt = [&](uint32_t pm, int tt) {
        while (pm) {
            const int p = tt + (__builtin_ctz(pm) >> 3);
            pm &= pm - 1u;
            if (p >= 5 && p < kf && R.ld32(p - 5) == NEWS4 && (R.ld32(p - 1) & 0xFFu) == 0x2Fu) kf = p;
        }
    };
    auto any_html = [&](uint32_t lo, uint32_t hi) -> bool {
        return (lo == HTML4) | (__builtin_amdgcn_alignbyte(hi, lo, 1) == HTML4) |
               (__builtin_amdgcn_alignbyte(hi, lo, 2) == HTML4) | (__builtin_amdgcn_alignbyte(hi, lo, 3) == HTML4);
    };
    // valid candidates among q = tt + 0..3 (lo = bytes [tt, tt + 4), hi the next 4, prev the 4 before)
    auto valid_html = [&](uint32_t lo, uint32_t hi, uint32_t prev, int tt) -> uint32_t {
        uint32_t hm = (lo == HTML4 ? 0x80u : 0u) | (__builtin_amdgcn_alignbyte(hi, lo, 1) == HTML4 ? 0x8000u : 0u) |
                      (__builtin_amdgcn_alignbyte(hi, lo, 2) == HTML4 ? 0x800000u : 0u) |
                      (__builtin_amdgcn_alignbyte(hi, lo, 3) == HTML4 ? 0x80000000u : 0u);
        const int r3 = L - tt - 3;   // q + 4 <= L
        hm &= r3 >= 4 ? 0x80808080u : (r3 <= 0 ? 0u : 0x80808080u & ((1u << (8 * r3)) - 1u));
        hm &= ~eq_bytes(__builtin_amdgcn_alignbyte(lo, prev, 3), 0x0A0A0A0Au);
        if (tt == 0) hm &= ~0x80u;
        return hm;
    };
    for (;;) {
        for (; t < L; t += 8, k += 2) {
            const uint32_t d3 = R.dw(k), d4 = R.dw(k + 1);
            x2 = __builtin_amdgcn_alignbyte(d2, d1, R.s);
            y = __builtin_amdgcn_alignbyte(d3, d2, R.s);
            d1 = d3;
            d2 = d4;
            const uint32_t cmA = eq_bytes(x, 0x3A3A3A3Au);
            const uint32_t cmB = eq_bytes(x2, 0x3A3A3A3Au) & (t == 0 ? ~excl : ~0u);
            if (cmA | cmB) {
                if (cmA) colons(cmA, t);
                if (cmB) colons(cmB, t + 4);
            }
            const uint32_t pmA = eq_bytes(x | 0x02020202u, 0x27272727u), pmB = eq_bytes(x2 | 0x02020202u, 0x27272727u);
            if (pmA | pmB) {
                filt(pmA, t);
                filt(pmB, t + 4);
            }
            if ((int)any_html(x, x2) | (int)any_html(x2, y)) break;   // (no short circuit: one test)
            xp = x2;
            x = y;
        }
        if (t >= L) break;   // no cut
        uint32_t hm = valid_html(x, x2, xp, t);
        int tq = t;
        if (!hm) {
            hm = valid_html(x2, y, x, t + 4);
            tq = t + 4;
        }
        if (hm) {
            const int q = tq + (__builtin_ctz(hm) >> 3);
            int sp = q - 1;
            if ((R.ld32(sp) & 0xFFu) >= 0x80u) {
                while (sp > 0 && (R.ld32(sp) & 0xC0u) == 0x80u && q - sp < 4) --sp;
            }
            j = sp;
            break;
        }
        xp = x2;   // no valid candidate in this step: on with the next
        x = y;
        t += 8;
        k += 2;
    }
#else
    // the scan stops at any "html" at q in [t, t + 4); the candidates are validated out of the loop (q >= 1,
    // q + 4 <= L, no '\n' before q), and a step without a valid one resumes the scan
    // (d1, d2: the aligned dwords k - 1, k under y; dword k + 1 is read a step ahead)
    uint32_t d1 = R.dw(1), d2 = R.dw(2);
    uint32_t x = __builtin_amdgcn_alignbyte(d1, R.dw(0), R.s), xp = 0, y = 0;
    int t = 0, k = 2;
    for (;;) {
        for (; t < L; t += 4, ++k) {
            const uint32_t dn = R.dw(k + 1);
            y = __builtin_amdgcn_alignbyte(d2, d1, R.s);
            d1 = d2;
            d2 = dn;
            uint32_t cm = eq_bytes(x, 0x3A3A3A3Au);
            if (t == 4) cm &= ~excl;
            if (cm) {
                const uint32_t cm1 = cm & (cm - 1u);
                const int c0 = t + (__builtin_ctz(cm) >> 3);
                const int c1 = cm1 ? t + (__builtin_ctz(cm1) >> 3) : NONE;
                ec2 = ec == NONE ? c1 : (ec2 == NONE ? c0 : ec2);
                ec = ec == NONE ? c0 : ec;
            }
            uint32_t pm = eq_bytes(x | 0x02020202u, 0x27272727u);
            while (pm) {
                const int p = t + (__builtin_ctz(pm) >> 3);
                pm &= pm - 1u;
                if (p >= 5 && p < kf && R.ld32(p - 5) == NEWS4 && (R.ld32(p - 1) & 0xFFu) == 0x2Fu) kf = p;
            }
            if ((x == HTML4) | (__builtin_amdgcn_alignbyte(y, x, 1) == HTML4) |
                (__builtin_amdgcn_alignbyte(y, x, 2) == HTML4) | (__builtin_amdgcn_alignbyte(y, x, 3) == HTML4))
                break;
            xp = x;
            x = y;
        }
        if (t >= L) break;   // no cut
        uint32_t hm = (x == HTML4 ? 0x80u : 0u) | (__builtin_amdgcn_alignbyte(y, x, 1) == HTML4 ? 0x8000u : 0u) |
                      (__builtin_amdgcn_alignbyte(y, x, 2) == HTML4 ? 0x800000u : 0u) |
                      (__builtin_amdgcn_alignbyte(y, x, 3) == HTML4 ? 0x80000000u : 0u);
        const int r3 = L - t - 3;   // candidates q = t + k with q + 4 <= L
        hm &= r3 >= 4 ? 0x80808080u : (r3 <= 0 ? 0u : 0x80808080u & ((1u << (8 * r3)) - 1u));
        hm &= ~eq_bytes(__builtin_amdgcn_alignbyte(x, xp, 3), 0x0A0A0A0Au);
        if (t == 0) hm &= ~0x80u;
        if (hm) {
            const int q = t + (__builtin_ctz(hm) >> 3);
            int sp = q - 1;
            if ((R.ld32(sp) & 0xFFu) >= 0x80u) {
                while (sp > 0 && (R.ld32(sp) & 0xC0u) == 0x80u && q - sp < 4) --sp;
            }
            j = sp;
            break;
        }
        xp = x;   // no valid candidate in this step: on with the next
        x = y;
        t += 4;
        ++k;
    }
#endif
    if (j < 0) {
        code[i] = KW_URL_NO_HTML;
        S.len3[i] = 0;
        return -1;
    }
    const bool gap = ec < j;
    if (gap && !(ec2 >= j && ec > 5 && ec + 3 <= j && (R.ld32(ec) & 0xFFFFFFu) == 0x30383Au))
        return j;   // the byte-serial rewrite (dd_slow_kernel)
    const int ins = (scheme_http && j > 4) ? 1 : 0;
    const int G = gap ? ec + ins : NONE, E = j + ins - (gap ? 3 : 0);
    const int len3 = E + 5;
    // the normalised word at x (x % 8 == 0, x < len3): as FastWords, with 32-bit offsets
    auto splice = [&](uint64_t w, int x) -> uint64_t {
        if (E < x + 8) {
            if (E >= x) {
                const int sh = (E - x) * 8;
                w = (sh ? (w & ((1ull << sh) - 1)) : 0ull) | (DOTHTML << sh);
            } else {
                const int d = x - E;
                w = d < 8 ? DOTHTML >> (8 * d) : 0ull;
            }
        }
        return w;
    };
    auto body = [&](int x) -> uint64_t {
        uint64_t w = (ins && x == 0) ? 0x7370747468ull | (R.ld64(4) << 40) : R.ld64(x - ins + (x >= G ? 3 : 0));
        if (x < G && G < x + 8) {
            const int k = (G - x) * 8;
            w = (w & ((1ull << k) - 1)) | (R.ld64(G - ins + 3) << k);
        }
        return w;
    };
    bool jn = false;
    if (gap) {
        // 'news/%' | "news/'" across the gap: windows starting at G - 5 .. G - 1 (as transform_row)
        auto seg1 = [&](int x) -> uint64_t {
            if (!ins) return R.ld64(x);
            if (x >= 5) return R.ld64(x - 1);
            const uint64_t h0 = 0x7370747468ull | (R.ld64(4) << 40);
            return x ? (h0 >> (8 * x)) | (R.ld64(7) << (64 - 8 * x)) : h0;
        };
        auto nword = [&](int x) -> uint64_t {
            uint64_t w = 0;
            if (x < E) {
                if (x + 8 <= G) w = seg1(x);
                else if (x >= G) w = R.ld64(x - ins + 3);
                else {
                    const int k = (G - x) * 8;
                    w = (seg1(x) & ((1ull << k) - 1)) | (R.ld64(G - ins + 3) << k);
                }
            }
            return splice(w, x);
        };
        const uint64_t lo = nword(G - 5), hi = nword(G + 3);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint64_t win = ((lo >> (8 * k)) | (k ? hi << (64 - 8 * k) : 0ull)) & 0xFFFFFFFFFFFFull;
            jn |= win == 0x252F7377656Eull || win == 0x272F7377656Eull;
        }
    }
    const bool bad = kf < j || jn;
    // the hash over the words: word 0 (the 's' insertion) and the last words (".html" at E) in general form, the
    // words between as plain windows (the ':80' gap's straddling word merged)
    uint64_t h1 = 0x243F6A8885A308D3ull;
    const int nfull = E >> 3;   // words x with x + 8 <= E: no splice
    if (nfull > 0) h1 = mix1(h1, body(0));
    for (int x = 8; x < 8 * nfull; x += 8) {
        uint64_t w = R.ld64(x - ins + (x >= G ? 3 : 0));
        if (x < G && G < x + 8) {
            const int k = (G - x) * 8;
            w = (w & ((1ull << k) - 1)) | (R.ld64(G - ins + 3) << k);
        }
        h1 = mix1(h1, w);
    }
    for (int x = 8 * nfull; x < len3; x += 8) h1 = mix1(h1, splice(x < E ? body(x) : 0ull, x));
    pair = finish_row(h1, len3, bad, i, code, S, b,
                      make_uint2((uint32_t)j, ((uint32_t)ins << 31) | (gap ? (uint32_t)ec : NO_GAP)));
    return -1;
}
constexpr int TCLAIM = 8;           // groups of 64 rows a transform wave claims at once

// lane = row; the wave's 64 rows are staged into LDS with coalesced 16-byte loads when they fit
__global__ __launch_bounds__(BLOCK) void dd_transform_kernel(const uint8_t *__restrict__ arena,
                                                             const int64_t *__restrict__ off, int64_t n,
                                                             uint8_t *__restrict__ code, Scratch S)
{
    __shared__ uint4 stage_all[(BLOCK / 64) * (STAGE_BYTES / 16)];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    uint4 *stage = stage_all + wib * (STAGE_BYTES / 16);
    const int64_t n_groups = (n + 63) / 64;
    // groups of 64 rows claimed from a counter in row order: rows enter the table in about row order, so few
    // earlier duplicates displace a later row already there (grid-stride let waves drift apart: 16-26 % of the
    // duplicates were displaced rows, which decide looks up in the table again)
    // (TCLAIM groups per claim: one counter address for every group serialised the transform, 98 vs 68 ms; so
    // a claim's pairs go to its own segment, counted by the wave)
    auto claim = [&]() -> int64_t {
        uint64_t g = 0;
        if (lane == 0) g = atomicAdd(S.gnext, (unsigned long long)TCLAIM);
        return (int64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g) |
               ((int64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g >> 32)) << 32);
    };
    uint32_t n_nohtml = 0, n_filtered = 0;   // this lane's rows per code (one atomic per wave at the end)
    for (int64_t gc = claim(); gc < n_groups; gc = claim()) {
      const int64_t gce = gc + TCLAIM < n_groups ? gc + TCLAIM : n_groups;
      uint2 *const seg = S.pairs + gc * 64;   // this claim's pairs (a wave-uniform count: no shared counter)
      uint32_t pc = 0;
      for (int64_t g = gc; g < gce; ++g) {
        const int64_t i0 = g * 64, i1 = i0 + 64 < n ? i0 + 64 : n;
        const int64_t A0 = off[i0], A1 = off[i1];
        const int64_t base = A0 & ~(int64_t)15;
        const int64_t nch = (A1 + 16 - base + 15) >> 4;   // chunks to cover [A0, A1 + 16)
        const int64_t i = i0 + lane;
        int64_t b = 0, L = 0;
        if (i < n) { b = off[i]; L = off[i + 1] - b; }
        int64_t jslow = -1;
        uint2 pair = make_uint2(0u, NO_HINT);
        if (nch * 16 + 16 <= STAGE_BYTES) {
            __builtin_amdgcn_wave_barrier();
            stage_dma(stage, arena + base, (int)nch);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (i < n) {
                if (S.normalize) {
                    const int o = (int)(b - base);
                    const LdsRow R{(const uint32_t *)stage, o >> 2, (uint32_t)(o & 3)};
                    jslow = transform_row_lds(R, (int)L, i, b, code, S, pair);
                } else {
                    LdsSrc src{(const uint32_t *)stage, base};
                    jslow = transform_row(src, b, L, i, code, S, pair);
                }
            }
        } else {
            GlobalSrc src{arena};
            if (i < n) jslow = transform_row(src, b, L, i, code, S, pair);
        }
        if (i < n && jslow < 0) {
            const uint8_t k = code[i];   // (this lane's own store)
            n_nohtml += k == KW_URL_NO_HTML;
            n_filtered += k == KW_URL_FILTERED;
        }
        // pairs to compare -> the claim's segment (at most one per row: the segment holds the claim's rows)
        const uint64_t pm = __ballot(pair.y != NO_HINT);
        if (pair.y != NO_HINT) {
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
            seg[pc + r] = pair;
        }
        pc += (uint32_t)__popcll(pm);
        // rows for the byte-serial rewrite -> the global slow list (rare rows: one atomic per wave that has any)
        const uint64_t sm = __ballot(jslow >= 0);
        if (sm) {
            unsigned long long base_k = 0;
            if (lane == 0) base_k = atomicAdd(&S.nslow[0], (unsigned long long)__popcll(sm));
            base_k = (unsigned long long)__builtin_amdgcn_readfirstlane((int)(uint32_t)base_k) |
                     ((unsigned long long)__builtin_amdgcn_readfirstlane((int)(uint32_t)(base_k >> 32)) << 32);
            if (jslow >= 0) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                S.slow[base_k + r] = make_uint2((uint32_t)i, (uint32_t)jslow);
                atomicAdd(&S.nslow[1], (unsigned long long)slow_words(jslow));
            }
        }
      }
      if (lane == 0) S.pcount[gc / TCLAIM] = pc;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        n_nohtml += __shfl_xor(n_nohtml, d, 64);
        n_filtered += __shfl_xor(n_filtered, d, 64);
    }
    if (lane == 0) {
        if (n_nohtml) atomicAdd(&S.cnt[KW_URL_NO_HTML], (unsigned long long)n_nohtml);
        if (n_filtered) atomicAdd(&S.cnt[KW_URL_FILTERED], (unsigned long long)n_filtered);
    }
}

__global__ __launch_bounds__(BLOCK) void dd_slow_kernel(const uint8_t *__restrict__ arena,
                                                        const int64_t *__restrict__ off, uint8_t *__restrict__ code,
                                                        Scratch S, uint64_t ns)
{
    for (uint64_t k = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; k < ns; k += (uint64_t)gridDim.x * BLOCK) {
        const uint2 e = S.slow[k];
        // the entry becomes the row's pair (or (row, NO_HINT)), compared with the claims' pairs
        S.slow[k] = slow_row(arena, off[e.x], (int64_t)e.y, (int64_t)e.x, code, S);
    }
}

// a row's regenerator (its descriptor: one 16-byte load)
__device__ __forceinline__ RowGen row_gen(const Scratch &S, const uint8_t *arena, int64_t i)
{
    RowGen g;
    g.init(S, arena, S.rowd[i], i);
    return g;
}

// the normalised bytes of rows a and b are equal (same length len, both regenerated): SAME_U word pairs in flight
// per round
constexpr int SAME_U = 8;
__device__ __forceinline__ bool same_url(const RowGen &x, const RowGen &y)
{
    if (x.len != y.len) return false;
    const int64_t nw = ((int64_t)x.len + 7) / 8;
    for (int64_t w = 0; w < nw; w += SAME_U) {
        uint64_t d = 0;
#pragma unroll
        for (int q = 0; q < SAME_U; ++q)
            if (w + q < nw) d |= x.word(8 * (w + q)) ^ y.word(8 * (w + q));
        if (d) return false;
    }
    return true;
}

// a row's hash again from its regenerated words (as the transform made it)
__device__ __forceinline__ uint64_t row_hash(const Scratch &S, const RowGen &g)
{
    uint64_t h = 0x243F6A8885A308D3ull;
    const int64_t nw = ((int64_t)g.len + 7) / 8;
    for (int64_t w = 0; w < nw; ++w) h = mix1(h, g.word(8 * w));
    h = fmix(h ^ (uint64_t)g.len);
    return S.weak ? h & 0xFull : h;
}

// A pair's later row is a duplicate iff its bytes equal the earlier row's; a kept row in no pair is its tag's
// first row.  A pair that differs has its later row compared with its tag's first row from the table (a tag shared by different URLs: rare): equal -> duplicate, else
// CODE_COLLIDE, which the host resolves exactly among those rows (every row of a URL other than the first
// row's gets it, so their keep-first is complete).
//
// dd_pairs_kernel: 8 lanes a pair, lane s comparing words s, s + 8, ... of the two regenerated rows, so each load
// instruction touches a few lines of 8 rows (lane = row made every load touch 64 rows' lines: 37.8 ms at 500M
// rows, 123M pairs)
#ifndef DD_PAIR_LANES
#define DD_PAIR_LANES 4
#endif
#ifndef DD_PAIR_UNROLL
#define DD_PAIR_UNROLL 4
#endif
constexpr int PAIR_LANES = DD_PAIR_LANES;    // lanes a pair
constexpr int PAIR_UNROLL = DD_PAIR_UNROLL;  // words a lane has in flight per row

// a row's descriptor and resolved length, loaded by one lane (handed to the lanes that use it by shuffles)
struct Desc {
    uint4 r;
    uint32_t len;
};
__device__ __forceinline__ Desc load_desc(const Scratch &S, int64_t i)
{
    Desc d;
    d.r = S.rowd[i];
    d.len = d.r.y >> 8;
    if (d.len == LEN_BIG) d.len = S.len3[i];
    return d;
}
__device__ __forceinline__ Desc shfl_desc(const Desc &d, int src)
{
    Desc o;
    o.r.x = (uint32_t)__shfl((int)d.r.x, src, 64);
    o.r.y = (uint32_t)__shfl((int)d.r.y, src, 64);
    o.r.z = (uint32_t)__shfl((int)d.r.z, src, 64);
    o.r.w = (uint32_t)__shfl((int)d.r.w, src, 64);
    o.len = (uint32_t)__shfl((int)d.len, src, 64);
    return o;
}

// A row's normalised words with 32-bit offsets from its raw start (RowGen's cases; rows shorter than 2^31
// bytes): one raw window a word, the 's' insertion taken from the same window (u[4..7) is its bytes 4..6).
// Src::ld64(p) = the 8 raw bytes at p: GRow from global memory (the pair compare), LRow from the wave's LDS
// stage (the copy).
struct GRow {
    const uint8_t *a;   // the row's raw start
    __device__ __forceinline__ uint64_t ld64(int p) const { return dd::ld64(a, p); }
};
struct LRow {
    const uint32_t *w;  // the stage's words; the row starts at stage byte o
    int o;
    __device__ __forceinline__ uint64_t ld64(int p) const
    {
        const int q = o + p, k = q >> 2;
        const uint32_t sh = (uint32_t)(q & 3), x0 = w[k], x1 = w[k + 1], x2 = w[k + 2];
        return (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sh) << 32);
    }
};
template <class Src>
struct NormRow {
    Src src;
    const uint64_t *sw;     // a slow row's words
    int G, E, len, ins;
    __device__ __forceinline__ void plan(const Scratch &S, uint4 r, uint32_t l)
    {
        len = (int)l;
        sw = (S.normalize && r.z == SLOW_ROW) ? S.sarena + r.w : nullptr;
        ins = (int)(r.w >> 31);
        const uint32_t ec = r.w & NO_GAP;
        const bool gap = ec != NO_GAP;
        G = gap ? (int)ec + ins : 0x7FFFFFFF;
        E = (int)r.z + ins - (gap ? 3 : 0);
    }
    __device__ __forceinline__ uint64_t word(int x, bool normalize) const   // x < len, x % 8 == 0
    {
        if (!normalize) {
            const uint64_t w = src.ld64(x);
            return len - x >= 8 ? w : w & ((1ull << (8 * (len - x))) - 1);
        }
        if (sw) return sw[x >> 3];
        int p = x - ins + (x >= G ? 3 : 0);
        p = p < 0 ? 0 : p;
        uint64_t v = src.ld64(p);
        if (ins & (x == 0)) v = 0x7370747468ull | ((v >> 32) << 40);
        if (x < G && G < x + 8) {
            const int k = (G - x) * 8;
            v = (v & ((1ull << k) - 1)) | (src.ld64(G - ins + 3) << k);
        }
        v = x < E ? v : 0ull;
        if (E < x + 8) {
            if (E >= x) {
                const int sh = (E - x) * 8;
                v = (sh ? (v & ((1ull << sh) - 1)) : 0ull) | (DOTHTML << sh);
            } else {
                const int d = x - E;
                v = d < 8 ? DOTHTML >> (8 * d) : 0ull;
            }
        }
        return v;
    }
};
__device__ __forceinline__ int64_t desc_start(uint4 r) { return (int64_t)(((uint64_t)(r.y & 0xFFu) << 32) | r.x); }

// pairs e[0, m) (m <= 64, wave-uniform): lane t loads pair t's two descriptors, then 8 rounds of 8 pairs, lane s
// of a pair's group comparing words s, s + 8, ... of the two regenerated rows (each load instruction touches a
// few lines of 8 rows; the descriptors' dependent loads are paid once per 64 pairs)
__device__ __forceinline__ void compare_pairs(const uint8_t *__restrict__ arena, uint8_t *__restrict__ code,
                                              const Scratch &S, const uint2 *__restrict__ e, uint32_t m,
                                              uint32_t &n_dup)
{
    const int lane = threadIdx.x & 63, grp = lane / PAIR_LANES, s = lane & (PAIR_LANES - 1);
    uint2 pr = make_uint2(0u, NO_HINT);
    if ((uint32_t)lane < m) pr = e[lane];
    const bool live = pr.y != NO_HINT;   // (the slow list's entries without a pair)
    Desc dx{}, dy{};
    if (live) {
        dx = load_desc(S, pr.x);
        dy = load_desc(S, pr.y);
    }
    const uint64_t lm = __ballot(live);
    for (uint32_t r0 = 0; r0 < m; r0 += 64 / PAIR_LANES) {
        const int src = (int)r0 + grp;
        const Desc x = shfl_desc(dx, src), y = shfl_desc(dy, src);
        const uint32_t row = (uint32_t)__shfl((int)pr.x, src, 64);
        const bool act = (uint32_t)src < m && ((lm >> src) & 1ull);
        uint64_t d = 0;
        if (act) {
            // (rows of 2 GiB and more count as differing: the recheck compares them with 64-bit offsets)
            d = x.len != y.len || x.len >= 0x80000000u;
            if (!d) {
                NormRow<GRow> gx, gy;
                gx.src = GRow{arena + desc_start(x.r)};
                gx.plan(S, x.r, x.len);
                gy.src = GRow{arena + desc_start(y.r)};
                gy.plan(S, y.r, y.len);
                const int nw = (gx.len + 7) >> 3;
                const bool nz = S.normalize != 0;
                for (int w0 = s; w0 < nw; w0 += PAIR_LANES * PAIR_UNROLL) {
                    uint64_t xa[PAIR_UNROLL], ya[PAIR_UNROLL];
#pragma unroll
                    for (int u = 0; u < PAIR_UNROLL; ++u) {
                        const int w = w0 + u * PAIR_LANES;
                        xa[u] = w < nw ? gx.word(8 * w, nz) : 0ull;
                        ya[u] = w < nw ? gy.word(8 * w, nz) : 0ull;
                    }
#pragma unroll
                    for (int u = 0; u < PAIR_UNROLL; ++u) d |= xa[u] ^ ya[u];
                }
            }
        }
        const uint64_t bm = __ballot(d != 0);
        const bool eq = ((bm >> (lane & ~(PAIR_LANES - 1))) & ((1ull << PAIR_LANES) - 1)) == 0;
        if (act && s == 0) {
            if (eq) {
                code[row] = (uint8_t)KW_URL_DUPLICATE;
                ++n_dup;
            } else {
                S.recheck[atomicAdd(&S.cnt[5], 1ull)] = row;   // (rare)
            }
        }
    }
}

// a wave per claim: its pairs 64 at a time; then the slow rows' entries, 64 at a time
#ifndef DD_PAIRS_MINB
#define DD_PAIRS_MINB 1   // (A/B: blocks per CU the compiler must fit)
#endif
__global__ __launch_bounds__(BLOCK, DD_PAIRS_MINB) void dd_pairs_kernel(const uint8_t *__restrict__ arena, uint8_t *__restrict__ code,
                                                         Scratch S, int64_t n_claims, uint64_t ns)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * BLOCK) >> 6;
    uint32_t n_dup = 0;
    for (int64_t c = wave; c < n_claims; c += n_waves) {
        const uint32_t pc = S.pcount[c];
        const uint2 *seg = S.pairs + c * 64 * TCLAIM;
        for (uint32_t k = 0; k < pc; k += 64) compare_pairs(arena, code, S, seg + k, pc - k < 64 ? pc - k : 64, n_dup);
    }
    for (uint64_t k = (uint64_t)wave * 64; k < ns; k += (uint64_t)n_waves * 64)
        compare_pairs(arena, code, S, S.slow + k, (uint32_t)(ns - k < 64 ? ns - k : 64), n_dup);
    for (int d = 32; d >= 1; d >>= 1) n_dup += __shfl_xor(n_dup, d, 64);
    if (lane == 0 && n_dup) atomicAdd(&S.cnt[KW_URL_DUPLICATE], (unsigned long long)n_dup);
}

// a row against its tag's first row from the table (lane = row; rare rows): duplicate or CODE_COLLIDE
__device__ __forceinline__ void recheck_row(const uint8_t *__restrict__ arena, uint8_t *__restrict__ code,
                                            const Scratch &S, uint32_t i)
{
    const RowGen gi = row_gen(S, arena, i);
    const uint64_t h = row_hash(S, gi);
    uint64_t slot = (h ^ (h >> 29)) & S.mask;
    unsigned long long cur;
    const uint32_t want = (uint32_t)((h >> 40) << 8) | S.epoch;   // its tag and this run's epoch
    for (;;) {   // (the row's own insert left its tag on this probe path)
        cur = S.table[slot];
        if ((uint32_t)(cur >> 32) == want) break;
        slot = (slot + 1) & S.mask;
    }
    const uint32_t r0 = (uint32_t)cur - 1u;
    const bool eq = r0 != i && same_url(gi, row_gen(S, arena, r0));
    code[i] = eq ? (uint8_t)KW_URL_DUPLICATE : CODE_COLLIDE;
    atomicAdd(&S.cnt[eq ? KW_URL_DUPLICATE : CODE_COLLIDE], 1ull);
    if (!eq) {
        const unsigned long long k = atomicAdd(&S.cnt[9], 1ull);
        if (k < COLLIDE_CAP) S.collide[k] = i;
    }
}

// the later rows of the pairs that differed (the list)
__global__ __launch_bounds__(BLOCK) void dd_recheck_kernel(const uint8_t *__restrict__ arena,
                                                           uint8_t *__restrict__ code, Scratch S)
{
    const unsigned long long nr = S.cnt[5];
    for (unsigned long long k = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x; k < nr;
         k += (unsigned long long)gridDim.x * BLOCK)
        recheck_row(arena, code, S, S.recheck[k]);
}

// the CODE_COLLIDE rows (rare: a 32-bit tag shared by two URLs in one probe run), listed for the host's exact pass
__global__ __launch_bounds__(BLOCK) void dd_collect_kernel(const uint8_t *__restrict__ code, int64_t n,
                                                           unsigned long long *__restrict__ count,
                                                           uint32_t *__restrict__ list, uint32_t cap)
{
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK) {
        if (code[i] != CODE_COLLIDE) continue;
        const unsigned long long p = atomicAdd(count, 1ull);
        if (p < cap) list[p] = (uint32_t)i;
    }
}

// ---- dense kept rows: per-tile counts, one-block scan of the tiles, placement, byte copy
__device__ __forceinline__ void block_excl_scan2(uint64_t &a, uint64_t &b, uint64_t *sh, uint64_t &ta, uint64_t &tb)
{
    // exclusive scan of (a, b) over the block; ta/tb = block totals
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t xa = a, xb = b;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t ya = __shfl_up(xa, d, 64), yb = __shfl_up(xb, d, 64);
        if (lane >= d) { xa += ya; xb += yb; }
    }
    if (lane == 63) { sh[2 * wv] = xa; sh[2 * wv + 1] = xb; }
    __syncthreads();
    uint64_t pa = 0, pb = 0;
    ta = 0;
    tb = 0;
    for (int w = 0; w < BLOCK / 64; ++w) {
        if (w < wv) { pa += sh[2 * w]; pb += sh[2 * w + 1]; }
        ta += sh[2 * w];
        tb += sh[2 * w + 1];
    }
    __syncthreads();
    a = pa + xa - a;
    b = pb + xb - b;
}

__global__ __launch_bounds__(BLOCK) void dd_count_kernel(const uint8_t *__restrict__ code, int64_t n, Scratch S,
                                                         unsigned long long *__restrict__ tile_cnt,
                                                         unsigned long long *__restrict__ tile_bytes)
{
    __shared__ uint64_t sh[2 * BLOCK / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ROWS;
    uint64_t c = 0, by = 0;
    for (int r = 0; r < SCAN_ROWS; ++r) {
        const int64_t i = base + r;
        if (i < n && code[i] == KW_URL_KEPT) { ++c; by += S.len3[i]; }
    }
    uint64_t ta, tb;
    block_excl_scan2(c, by, sh, ta, tb);
    if (threadIdx.x == 0) { tile_cnt[blockIdx.x] = ta; tile_bytes[blockIdx.x] = tb; }
}

// the (count, bytes) sums of the tile chunks [c * per_blk, (c + 1) * per_blk)
__global__ __launch_bounds__(BLOCK) void dd_tile_sums_kernel(const unsigned long long *__restrict__ tile_cnt,
                                                             const unsigned long long *__restrict__ tile_bytes,
                                                             int64_t nt, int64_t per_blk,
                                                             unsigned long long *__restrict__ sum_cnt,
                                                             unsigned long long *__restrict__ sum_bytes)
{
    __shared__ unsigned long long sc_[BLOCK / 64], sb_[BLOCK / 64];
    const int64_t b0 = (int64_t)blockIdx.x * per_blk, b1 = b0 + per_blk < nt ? b0 + per_blk : nt;
    unsigned long long c = 0, b = 0;
    for (int64_t k = b0 + threadIdx.x; k < b1; k += BLOCK) { c += tile_cnt[k]; b += tile_bytes[k]; }
    for (int d = 32; d >= 1; d >>= 1) { c += __shfl_xor(c, d, 64); b += __shfl_xor(b, d, 64); }
    if ((threadIdx.x & 63) == 0) { sc_[threadIdx.x >> 6] = c; sb_[threadIdx.x >> 6] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long tc = 0, tb = 0;
        for (int w = 0; w < BLOCK / 64; ++w) { tc += sc_[w]; tb += sb_[w]; }
        sum_cnt[blockIdx.x] = tc;
        sum_bytes[blockIdx.x] = tb;
    }
}

// exclusive scan of the per-tile (count, bytes) pairs, block c over tiles [c * per_blk, (c + 1) * per_blk) from
// its prefix pre[c] (none: 0): each thread sums a contiguous segment (loads unrolled by 8, in flight together),
// the 1024 segment sums are scanned by wave shuffles and LDS (16 wave totals), then each thread rewrites its
// segment; totals (if given) = the block's sums.  The tiles are scanned in two levels (dd_tile_sums_kernel
// per chunk, this kernel on the chunk sums, then on each chunk): one block over all 0.5M tiles took 1.15 ms.
__global__ __launch_bounds__(1024) void dd_scan_tiles_kernel(unsigned long long *__restrict__ tile_cnt,
                                                             unsigned long long *__restrict__ tile_bytes, int64_t nt,
                                                             unsigned long long *__restrict__ totals,
                                                             int64_t per_blk, const unsigned long long *__restrict__ pre_cnt,
                                                             const unsigned long long *__restrict__ pre_bytes)
{
    __shared__ unsigned long long wc[16], wb[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t b0 = (int64_t)blockIdx.x * per_blk;
    const int64_t bn = (b0 + per_blk < nt ? b0 + per_blk : nt) - b0;
    tile_cnt += b0;
    tile_bytes += b0;
    nt = bn > 0 ? bn : 0;
    const int64_t per = (nt + 1023) / 1024;
    const int64_t k0 = t * per < nt ? t * per : nt, k1 = (t + 1) * per < nt ? (t + 1) * per : nt;
    unsigned long long sc = 0, sb = 0;
    int64_t k = k0;
    for (; k + 8 <= k1; k += 8) {
        unsigned long long c[8], b[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) { c[i] = tile_cnt[k + i]; b[i] = tile_bytes[k + i]; }
#pragma unroll
        for (int i = 0; i < 8; ++i) { sc += c[i]; sb += b[i]; }
    }
    for (; k < k1; ++k) { sc += tile_cnt[k]; sb += tile_bytes[k]; }
    // inclusive scan of (sc, sb) over the wave, then over the 16 waves
    unsigned long long xc = sc, xb = sb;
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long yc = __shfl_up(xc, d, 64), yb = __shfl_up(xb, d, 64);
        if (lane >= d) { xc += yc; xb += yb; }
    }
    if (lane == 63) { wc[wv] = xc; wb[wv] = xb; }
    __syncthreads();
    unsigned long long pc = 0, pb = 0, tc = 0, tb = 0;
    for (int w = 0; w < 16; ++w) {
        if (w < wv) { pc += wc[w]; pb += wb[w]; }
        tc += wc[w];
        tb += wb[w];
    }
    if (t == 0 && totals) { totals[0] = tc; totals[1] = tb; }
    unsigned long long ac = pc + xc - sc, ab = pb + xb - sb;   // exclusive prefix of this thread's segment
    if (pre_cnt) {
        ac += pre_cnt[blockIdx.x];
        ab += pre_bytes[blockIdx.x];
    }
    for (k = k0; k + 8 <= k1; k += 8) {
        unsigned long long c[8], b[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) { c[i] = tile_cnt[k + i]; b[i] = tile_bytes[k + i]; }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            tile_cnt[k + i] = ac;
            tile_bytes[k + i] = ab;
            ac += c[i];
            ab += b[i];
        }
    }
    for (; k < k1; ++k) {
        const unsigned long long vc = tile_cnt[k], vb = tile_bytes[k];
        tile_cnt[k] = ac;
        tile_bytes[k] = ab;
        ac += vc;
        ab += vb;
    }
}

__global__ __launch_bounds__(BLOCK) void dd_place_kernel(const uint8_t *__restrict__ code, int64_t n, Scratch S,
                                                         const unsigned long long *__restrict__ tile_cnt,
                                                         const unsigned long long *__restrict__ tile_bytes,
                                                         int64_t *__restrict__ kept_off, int64_t *__restrict__ kept_row)
{
    // the tile's kept entries assembled in LDS, then written as two contiguous runs (each thread writing its
    // own rows' entries in place wrote every line in 3-entry pieces: 12 GB of writes for 5.6 GB of entries)
    __shared__ uint64_t sh[2 * BLOCK / 64];
    __shared__ int64_t soff[SCAN_TILE], srow[SCAN_TILE];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ROWS;
    uint8_t k[SCAN_ROWS];
    uint32_t l[SCAN_ROWS];
    uint64_t c = 0, by = 0;
#pragma unroll
    for (int r = 0; r < SCAN_ROWS; ++r) {
        const int64_t i = base + r;
        k[r] = i < n ? code[i] : (uint8_t)0xFF;
        l[r] = k[r] == KW_URL_KEPT ? S.len3[i] : 0u;
        c += k[r] == KW_URL_KEPT;
        by += l[r];
    }
    uint64_t ta, tb;
    block_excl_scan2(c, by, sh, ta, tb);   // (c, by): this thread's first entry within the tile, its offset
    const uint64_t c0 = tile_cnt[blockIdx.x], b0 = tile_bytes[blockIdx.x];
    uint32_t q = (uint32_t)c;
#pragma unroll
    for (int r = 0; r < SCAN_ROWS; ++r) {
        if (k[r] == KW_URL_KEPT) {
            soff[q] = (int64_t)(b0 + by);
            srow[q] = base + r;
            ++q;
            by += l[r];
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < (uint32_t)ta; e += BLOCK) {
        kept_off[c0 + e] = soff[e];
        kept_row[c0 + e] = srow[e];
    }
}

// (groups whose dense range exceeds a wave's LDS stage: rows of 128 bytes on average or more) lane = row: the
// row's regenerated words written byte by byte at its dense offset (every byte has one writer)
__device__ __attribute__((noinline)) void copy_group_rows(int64_t k0, int64_t n_kept, const int64_t *__restrict__ kept_off,
                                                         const int64_t *__restrict__ kept_row,
                                                         const uint8_t *__restrict__ arena, const Scratch &S,
                                                         uint8_t *__restrict__ dst, int nrows = 64)
{
    const int lane = threadIdx.x & 63;
    const int64_t kk = k0 + lane;
    if (lane >= nrows || kk >= n_kept) return;
    const int64_t d0 = kept_off[kk], len = kept_off[kk + 1] - d0;
    const RowGen g = row_gen(S, arena, kept_row[kk]);
#pragma unroll 1
    for (int64_t x = 0; x < len; x += 8) {
        const uint64_t w = g.word(x);
        const int m = len - x < 8 ? (int)(len - x) : 8;
#pragma unroll 1
        for (int k = 0; k < m; ++k) dst[d0 + x + k] = (uint8_t)(w >> (8 * k));
    }
}


// dense kept rows: a wave owns kept rows [k0, k0 + 64) whose dense bytes are one contiguous range [D0, D1).
// The range is staged in the wave's LDS (zeroed, then every lane ORs its row's dwords in at the row's dense
// offset: the partial dwords two rows share merge by ds_or_b32) and written out with aligned 16-byte stores,
// the two partial 16-byte chunks it may share with the neighbouring groups byte by byte.  A group whose range
// exceeds the stage takes copy_group_rows.
constexpr int CP_STAGE = 8192;   // bytes of LDS per wave
__global__ __launch_bounds__(BLOCK) void dd_copy_kernel(int64_t n_kept, const int64_t *__restrict__ kept_off,
                                                        const int64_t *__restrict__ kept_row,
                                                        const uint8_t *__restrict__ arena, Scratch S,
                                                        uint8_t *__restrict__ dst)
{
    __shared__ uint4 stage_all[(BLOCK / 64) * (CP_STAGE / 16)];
    const int lane = threadIdx.x & 63;
    const int wib = threadIdx.x >> 6;
    uint4 *st16 = stage_all + wib * (CP_STAGE / 16);
    uint32_t *st32 = (uint32_t *)st16;
    const uint8_t *st8 = (const uint8_t *)st16;
    const int64_t wave = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * BLOCK) >> 6;
    for (int64_t k0 = wave * 64; k0 < n_kept; k0 += n_waves * 64) {
        const int64_t kk = k0 + lane;
        const int64_t kend = k0 + 64 < n_kept ? k0 + 64 : n_kept;
        const int64_t D0 = kept_off[k0], D1 = kept_off[kend];
        const int64_t A = D0 & ~(int64_t)15;
        if (D1 - A > CP_STAGE) {   // (wave-uniform)
            copy_group_rows(k0, n_kept, kept_off, kept_row, arena, S, dst);
            continue;
        }
        int64_t d0 = 0, len = 0;
        uint32_t row = 0;
        if (kk < n_kept) {
            row = (uint32_t)kept_row[kk];
            d0 = kept_off[kk];
            len = kept_off[kk + 1] - d0;
        }
        const int nz = (int)((D1 - A + 15) >> 4);
        __builtin_amdgcn_wave_barrier();
        for (int c = lane; c < nz; c += 64) st16[c] = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (len > 0) {
            // the row's regenerated words are zero past its end: 16 source dwords per round from 8 words in
            // flight, each destination dword the shifted pair of source dwords; the first and last destination
            // dwords may hold a neighbour's bytes (ds_or), the rest are this row's alone (plain stores into the
            // zeroed stage)
            const int64_t o = d0 - A;
            const uint32_t sh = (uint32_t)(o & 3) * 8u;
            uint32_t *dw = st32 + (o >> 2);
            RowGen g;
            g.init_len(S, arena, S.rowd[row], (uint32_t)len);   // (the length: the dense range's)
            const int nw8 = (int)((len + 7) >> 3);
            const int K = (int)(((o & 3) + len + 3) >> 2);
            uint32_t prev = 0;
            for (int k0 = 0; k0 < K; k0 += 16) {
                uint2 v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint64_t wq = (k0 >> 1) + q < nw8 ? g.word(8 * (int64_t)((k0 >> 1) + q)) : 0ull;
                    v[q] = make_uint2((uint32_t)wq, (uint32_t)(wq >> 32));
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t cur = (j & 1) ? v[j >> 1].y : v[j >> 1].x;
                    const uint32_t out = sh ? (cur << sh) | (prev >> (32u - sh)) : cur;
                    prev = cur;
                    const int k = k0 + j;
                    if (k < K) {
                        if (k == 0 || k == K - 1) atomicOr(&dw[k], out);
                        else dw[k] = out;
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int64_t a0 = (D0 + 15) & ~(int64_t)15, a1 = D1 & ~(int64_t)15;
        if (a0 >= a1) {
            for (int64_t x = D0 + lane; x < D1; x += 64) dst[x] = st8[x - A];
        } else {
            if (D0 + lane < a0) dst[D0 + lane] = st8[D0 + lane - A];
            if (a1 + lane < D1) dst[a1 + lane] = st8[a1 + lane - A];
            for (int64_t q = a0 + 16 * (int64_t)lane; q < a1; q += 16 * 64)
                *(uint4 *)(dst + q) = st16[(q - A) >> 4];
        }
    }
}

// The dense copy with staged input: a wave owns 32 kept rows (two lanes a row: the first and second half of its
// words), stages the raw bytes they are made from with coalesced 16-byte loads (the rows are consecutive in the
// arena but for the dropped rows between them), regenerates the words from LDS into the zeroed output stage,
// and writes the dense range out as dd_copy_kernel does.  The lane-per-row copy regenerated each word from
// global memory: a load instruction touched a line of each of 64 rows, and with 20 waves' rows per CU the L1
// held none of them between a row's words (every word a new trip to L2).  A task whose raw span or dense range
// exceeds its stage takes copy_group_rows.
constexpr int CPS_ROWS = 32;
constexpr int CPS_IN = 6144, CPS_OUT = 4096;   // LDS bytes per wave (one wave a block)
__global__ __launch_bounds__(64) void dd_copy_staged_kernel(int64_t n_kept, const int64_t *__restrict__ kept_off,
                                                            const int64_t *__restrict__ kept_row,
                                                            const uint8_t *__restrict__ arena, Scratch S,
                                                            uint8_t *__restrict__ dst)
{
    __shared__ uint4 in16[CPS_IN / 16];
    __shared__ uint4 out16[CPS_OUT / 16];
    uint32_t *out32 = (uint32_t *)out16;
    const uint8_t *out8 = (const uint8_t *)out16;
    const int lane = threadIdx.x & 63, r = lane & (CPS_ROWS - 1), half = lane / CPS_ROWS;
    const int64_t n_tasks = (n_kept + CPS_ROWS - 1) / CPS_ROWS;
    for (int64_t tk = blockIdx.x; tk < n_tasks; tk += gridDim.x) {
        const int64_t k0 = tk * CPS_ROWS, kk = k0 + r;
        const int nr = (int)(n_kept - k0 < CPS_ROWS ? n_kept - k0 : CPS_ROWS);
        int64_t d0 = 0, len = 0, row = 0, need = 0;
        uint4 rd = make_uint4(0u, 0u, 0u, 0u);
        if (r < nr) {
            row = kept_row[kk];
            d0 = kept_off[kk];
            len = kept_off[kk + 1] - d0;
            rd = S.rowd[row];
        }
        const int64_t b = (int64_t)(((uint64_t)(rd.y & 0xFFu) << 32) | rd.x);
        // the raw bytes a row's words read: below its cut + 16 (the 8-byte windows past a ':80' gap), its whole
        // length when not normalising, none for a slow row; the last row's end bounds every row's
        need = b + 16 + (!S.normalize ? len : (rd.z == SLOW_ROW ? 0 : (int64_t)rd.z));
        const int64_t D0 = __shfl(d0, 0, 64), D1 = __shfl(d0 + len, nr - 1, 64);
        const int64_t B0 = __shfl(b, 0, 64) & ~(int64_t)15, B1 = __shfl(need, nr - 1, 64);
        const int64_t OA = D0 & ~(int64_t)15;
        if (B1 - B0 > CPS_IN || D1 - OA > CPS_OUT) {   // (wave-uniform)
            copy_group_rows(k0, n_kept, kept_off, kept_row, arena, S, dst, nr);
            continue;
        }
        const int nin = (int)((B1 - B0 + 15) >> 4), nz = (int)((D1 - OA + 15) >> 4);
        __builtin_amdgcn_wave_barrier();
        stage_dma(in16, arena + B0, nin);
        for (int c = lane; c < nz; c += 64) out16[c] = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (r < nr && len > 0) {
            NormRow<LRow> g;
            g.src = LRow{(const uint32_t *)in16, (int)(b - B0)};
            g.plan(S, rd, (uint32_t)len);
            const bool nz = S.normalize != 0;
            const int nw = (int)((len + 7) >> 3), nwh = (nw + 1) >> 1;
            const int w0 = half ? nwh : 0, nwl = half ? nw - nwh : nwh;   // this lane's words [w0, w0 + nwl)
            if (nwl > 0) {
                const int64_t o = d0 - OA + 8 * (int64_t)w0;
                // (the first half's words end inside the row, or at its end when it holds them all)
                const int64_t rest = len - 8 * (int64_t)w0;
                const int64_t bytes = half || rest < 8 * (int64_t)nwl ? rest : 8 * (int64_t)nwl;
                const uint32_t sh = (uint32_t)(o & 3) * 8u;
                uint32_t *dw = out32 + (o >> 2);
                const int K = (int)(((o & 3) + bytes + 3) >> 2);
                uint32_t prev = 0;
                for (int k0w = 0; k0w < K; k0w += 8) {
                    uint2 v[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int wi = (k0w >> 1) + q;
                        const uint64_t wq = wi < nwl ? g.word(8 * (w0 + wi), nz) : 0ull;
                        v[q] = make_uint2((uint32_t)wq, (uint32_t)(wq >> 32));
                    }
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const uint32_t cur = (jj & 1) ? v[jj >> 1].y : v[jj >> 1].x;
                        const uint32_t out = sh ? (cur << sh) | (prev >> (32u - sh)) : cur;
                        prev = cur;
                        const int k = k0w + jj;
                        if (k < K) {
                            if (k == 0 || k == K - 1) atomicOr(&dw[k], out);
                            else dw[k] = out;
                        }
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int64_t a0 = (D0 + 15) & ~(int64_t)15, a1 = D1 & ~(int64_t)15;
        if (a0 >= a1) {
            for (int64_t x = D0 + lane; x < D1; x += 64) dst[x] = out8[x - OA];
        } else {
            if (D0 + lane < a0) dst[D0 + lane] = out8[D0 + lane - OA];
            if (a1 + lane < D1) dst[a1 + lane] = out8[a1 + lane - OA];
            for (int64_t q = a0 + 16 * (int64_t)lane; q < a1; q += 16 * 64)
                *(uint4 *)(dst + q) = out16[(q - OA) >> 4];
        }
    }
}

// the lengths of listed rows, then their normalised bytes (8-aligned slots at boff[k]): the host's exact pass
__global__ __launch_bounds__(BLOCK) void dd_gather_len_kernel(const uint32_t *__restrict__ rows, uint32_t m, Scratch S,
                                                              uint32_t *__restrict__ out)
{
    for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < m; k += gridDim.x * BLOCK) out[k] = S.len3[rows[k]];
}

__global__ __launch_bounds__(BLOCK) void dd_materialize_kernel(const uint8_t *__restrict__ arena,
                                                               const int64_t *__restrict__ off, Scratch S,
                                                               const uint32_t *__restrict__ rows, uint32_t m,
                                                               const uint64_t *__restrict__ boff, uint8_t *__restrict__ buf)
{
    for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < m; k += gridDim.x * BLOCK) {
        const uint32_t r = rows[k];
        const RowGen g = row_gen(S, arena, r);
        for (int64_t x = 0; x < (int64_t)g.len; x += 8) *(uint64_t *)(buf + boff[k] + x) = g.word(x);
    }
}

}  // namespace dd

using namespace dd;

struct kw_dedup {
    int device = 0;
    int cus = 256;
    int copy_bpc = 4, pairs_bpc = 4, copys_bpc = 16;   // resident blocks per CU of the statically divided kernels (one round of
                                       // blocks: a second partial round left CUs idle at the end)
    std::string err;
    void *d_buf = nullptr;
    size_t buf_bytes = 0;
    Scratch S{};
    unsigned long long *tile_cnt = nullptr, *tile_bytes = nullptr, *totals = nullptr;
    unsigned long long *chunk_cnt = nullptr, *chunk_bytes = nullptr;   // the tile scan's chunk sums
    int64_t *kept_off = nullptr, *kept_row = nullptr;
    uint8_t *kept_bytes = nullptr;
    size_t kept_bytes_cap = 0;
    void *d_kept = nullptr;
    void *d_collide = nullptr;   // count + list of the CODE_COLLIDE rows
    void *d_sarena = nullptr;    // the slow rows' normalised words
    size_t sarena_bytes = 0;
    int64_t n = 0, n_kept = 0, n_kept_bytes = 0;
    void *table_at = nullptr;   // where the table was last cleared, its slots, the epoch of the last run
    uint64_t table_slots = 0;
    uint32_t epoch = 0;
    int64_t counts[4] = {0, 0, 0, 0};
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    bool have_run = false;
};

#define DDCHK(h, x)                                                                    \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            (h)->err = std::string("HIP error ") + hipGetErrorString(e_) + " at " #x; \
            return KW_EHIP;                                                            \
        }                                                                              \
    } while (0)

extern "C" int kw_dedup_create(int32_t device, kw_dedup **out)
{
    if (!out) return KW_EINVAL;
    kw_dedup *h = new kw_dedup();
    *out = h;
    h->device = device;
    DDCHK(h, hipSetDevice(device));
    hipDeviceProp_t prop;
    DDCHK(h, hipGetDeviceProperties(&prop, device));
    h->cus = prop.multiProcessorCount;
    DDCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&h->copy_bpc, dd_copy_kernel, BLOCK, 0));
    DDCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&h->pairs_bpc, dd_pairs_kernel, BLOCK, 0));
    DDCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&h->copys_bpc, dd_copy_staged_kernel, 64, 0));
    h->copy_bpc = std::max(1, h->copy_bpc);
    h->copys_bpc = std::max(1, h->copys_bpc);
    h->pairs_bpc = std::max(1, h->pairs_bpc);
    for (auto &e : h->ev) DDCHK(h, hipEventCreate(&e));
    return KW_OK;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// exact keep-first over the rows that share a hash tag with a different URL (in row order): their normalised
// bytes regenerated on the device, compared on the host
static int resolve_collisions(kw_dedup *h, const uint8_t *d_arena, const int64_t *d_off, int64_t n, uint8_t *d_code,
                              hipStream_t st, unsigned long long listed)
{
    constexpr uint32_t CAP = COLLIDE_CAP;
    std::vector<uint32_t> rows;
    unsigned long long *d_cnt = (unsigned long long *)h->d_collide;
    unsigned long long m = listed;   // the recheck kernel's list (its rows: the CODE_COLLIDE rows)
    if (m > CAP) {   // (a longer list: the codes scanned again, by the kernel up to CAP, then on the host)
        DDCHK(h, hipMemsetAsync(d_cnt, 0, 8, st));
        const int grid = (int)std::min<int64_t>((n + BLOCK - 1) / BLOCK, (int64_t)h->cus * 16);
        hipLaunchKernelGGL(dd_collect_kernel, dim3(grid), dim3(BLOCK), 0, st, (const uint8_t *)d_code, n, d_cnt,
                           (uint32_t *)(d_cnt + 1), CAP);
        DDCHK(h, hipGetLastError());
        DDCHK(h, hipMemcpyAsync(&m, d_cnt, 8, hipMemcpyDeviceToHost, st));
        DDCHK(h, hipStreamSynchronize(st));
    }
    if (m <= CAP) {
        rows.resize(m);
        if (m) DDCHK(h, hipMemcpy(rows.data(), d_cnt + 1, 4 * m, hipMemcpyDeviceToHost));
        std::sort(rows.begin(), rows.end());
    } else {
        std::vector<uint8_t> code(n);
        DDCHK(h, hipMemcpy(code.data(), d_code, n, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < n; ++i)
            if (code[i] == CODE_COLLIDE) rows.push_back((uint32_t)i);
    }
    const uint32_t k = (uint32_t)rows.size();
    if (k == 0) return KW_OK;
    uint32_t *d_rows = nullptr, *d_len = nullptr;
    uint64_t *d_boff = nullptr;
    uint8_t *d_buf = nullptr;
    std::vector<uint32_t> len(k);
    std::vector<uint64_t> boff(k + 1, 0);
    int rc = KW_OK;
    auto fail = [&](hipError_t e, const char *what) {
        h->err = std::string("HIP error ") + hipGetErrorString(e) + " at " + what;
        rc = KW_EHIP;
    };
    hipError_t e;
    if ((e = hipMalloc(&d_rows, 4 * (size_t)k)) != hipSuccess) fail(e, "collide rows");
    if (!rc && (e = hipMalloc(&d_len, 4 * (size_t)k)) != hipSuccess) fail(e, "collide lengths");
    if (!rc && (e = hipMemcpy(d_rows, rows.data(), 4 * (size_t)k, hipMemcpyHostToDevice)) != hipSuccess) fail(e, "rows");
    const int g2 = (int)std::min<uint32_t>((k + BLOCK - 1) / BLOCK, 1024u);
    if (!rc) {
        hipLaunchKernelGGL(dd_gather_len_kernel, dim3(g2), dim3(BLOCK), 0, st, (const uint32_t *)d_rows, k, h->S, d_len);
        if ((e = hipMemcpyAsync(len.data(), d_len, 4 * (size_t)k, hipMemcpyDeviceToHost, st)) != hipSuccess) fail(e, "lengths");
        if (!rc && (e = hipStreamSynchronize(st)) != hipSuccess) fail(e, "sync");
    }
    for (uint32_t q = 0; q < k; ++q) boff[q + 1] = boff[q] + ((len[q] + 7) & ~7u);
    if (!rc && (e = hipMalloc(&d_boff, 8 * ((size_t)k + 1))) != hipSuccess) fail(e, "offsets");
    if (!rc && (e = hipMalloc(&d_buf, boff[k] + 8)) != hipSuccess) fail(e, "bytes");
    std::vector<uint8_t> buf(boff[k] + 8);
    if (!rc && (e = hipMemcpy(d_boff, boff.data(), 8 * ((size_t)k + 1), hipMemcpyHostToDevice)) != hipSuccess) fail(e, "boff");
    if (!rc) {
        hipLaunchKernelGGL(dd_materialize_kernel, dim3(g2), dim3(BLOCK), 0, st, d_arena, d_off, h->S,
                           (const uint32_t *)d_rows, k, (const uint64_t *)d_boff, d_buf);
        if ((e = hipMemcpyAsync(buf.data(), d_buf, boff[k], hipMemcpyDeviceToHost, st)) != hipSuccess) fail(e, "bytes back");
        if (!rc && (e = hipStreamSynchronize(st)) != hipSuccess) fail(e, "sync");
    }
    std::vector<uint8_t> codes(k);
    if (!rc) {
        std::unordered_set<std::string> seen;
        for (uint32_t q = 0; q < k; ++q) {
            const std::string s((const char *)buf.data() + boff[q], len[q]);
            codes[q] = seen.insert(s).second ? (uint8_t)KW_URL_KEPT : (uint8_t)KW_URL_DUPLICATE;
            ++h->counts[codes[q]];
        }
        for (uint32_t q = 0; q < k && !rc; ++q)
            if ((e = hipMemcpy(d_code + rows[q], &codes[q], 1, hipMemcpyHostToDevice)) != hipSuccess) fail(e, "code");
    }
    if (d_rows) (void)hipFree(d_rows);
    if (d_len) (void)hipFree(d_len);
    if (d_boff) (void)hipFree(d_boff);
    if (d_buf) (void)hipFree(d_buf);
    return rc;
}

extern "C" int kw_dedup_run(kw_dedup *h, const uint8_t *d_arena, const int64_t *d_off, int64_t n, int32_t flags,
                            uint8_t *d_code, void *stream)
{
    if (!h) return KW_EINVAL;
    if (n < 0 || (n > 0 && (!d_arena || !d_off || !d_code))) { h->err = "kw_dedup_run: bad arguments"; return KW_EINVAL; }
    if (((uintptr_t)d_arena & 15) != 0) { h->err = "kw_dedup_run: arena must be 16-byte aligned"; return KW_EINVAL; }
    if (n >= ((int64_t)1 << 32)) { h->err = "kw_dedup_run: more than 2^32 - 1 rows"; return KW_EUNSUPPORTED; }
    DDCHK(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    h->n = n;
    h->have_run = true;
    for (int k = 0; k < 4; ++k) h->counts[k] = 0;
    h->n_kept = h->n_kept_bytes = 0;
    if (n == 0) return KW_OK;
    // ---- scratch (grown on demand)
    uint64_t tsize = 1024;
    while (tsize < 2 * (uint64_t)n) tsize <<= 1;
    const int64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    const int64_t n_claims = ((n + 63) / 64 + TCLAIM - 1) / TCLAIM;
    int tbpc = 8;   // transform blocks per CU (KW_DEDUP_TBLOCKS_PER_CU; 4, 5, 8, 16: 130.7-130.8 ms alike in round 4)
    if (const char *e = kw_env("KW_DEDUP_TBLOCKS_PER_CU")) tbpc = std::max(1, atoi(e));
    const int tgrid = (int)std::min<int64_t>((n + BLOCK - 1) / BLOCK, (int64_t)h->cus * tbpc);
    const size_t need = align256(16 * (size_t)n) + align256(4 * (size_t)n) + align256(8 * tsize) +
                        align256(8 * ((size_t)n_claims * 64 * TCLAIM)) + align256(4 * (size_t)n_claims) +
                        align256(4 * (size_t)n) +
                        align256(8 * 16) +
                        align256(8 * 4) + align256(8 * (size_t)n) + 2 * align256(8 * (size_t)ntiles) +
                        align256(16) + 2 * align256(8 * SCAN_CHUNKS) + 2 * align256(8 * ((size_t)n + 1));
    if (need > h->buf_bytes) {
        if (h->d_buf) (void)hipFree(h->d_buf);
        h->d_buf = nullptr;
        h->buf_bytes = 0;
        DDCHK(h, hipMalloc(&h->d_buf, need));
        h->buf_bytes = need;
    }
    uint8_t *p = (uint8_t *)h->d_buf;
    auto carve = [&](size_t bytes) { uint8_t *r = p; p += align256(bytes); return r; };
    Scratch &S = h->S;
    S.rowd = (uint4 *)carve(16 * (size_t)n);
    S.len3 = (uint32_t *)carve(4 * (size_t)n);
    S.table = (unsigned long long *)carve(8 * tsize);
    S.pairs = (uint2 *)carve(8 * ((size_t)n_claims * 64 * TCLAIM));
    S.pcount = (uint32_t *)carve(4 * (size_t)n_claims);
    S.recheck = (uint32_t *)carve(4 * (size_t)n);
    S.mask = tsize - 1;
    S.cnt = (unsigned long long *)carve(8 * 16);
    S.gnext = S.cnt + 7;
    S.nslow = (unsigned long long *)carve(8 * 4);
    S.slow = (uint2 *)carve(8 * (size_t)n);
    S.sarena = (uint64_t *)h->d_sarena;
    if (!h->d_collide) DDCHK(h, hipMalloc(&h->d_collide, 8 + 4 * (size_t)COLLIDE_CAP));
    S.collide = (uint32_t *)((unsigned long long *)h->d_collide + 1);
    S.weak = kw_env("KW_TEST_DEDUP_WEAK_HASH") ? 1 : 0;
    S.stats = kw_env("KW_DEDUP_STATS") ? 1 : 0;
    S.normalize = (flags & KW_DEDUP_NORMALIZE) ? 1 : 0;
    h->tile_cnt = (unsigned long long *)carve(8 * (size_t)ntiles);
    h->tile_bytes = (unsigned long long *)carve(8 * (size_t)ntiles);
    h->totals = (unsigned long long *)carve(16);
    h->chunk_cnt = (unsigned long long *)carve(8 * SCAN_CHUNKS);
    h->chunk_bytes = (unsigned long long *)carve(8 * SCAN_CHUNKS);
    h->kept_off = (int64_t *)carve(8 * ((size_t)n + 1));
    h->kept_row = (int64_t *)carve(8 * ((size_t)n + 1));
    DDCHK(h, hipMemsetAsync(S.cnt, 0, 128, st));
    DDCHK(h, hipMemsetAsync(S.nslow, 0, 32, st));
    // the table is cleared when it moved or grew, or when the epoch wraps; else this run's epoch marks its slots
    if ((void *)S.table != h->table_at || tsize != h->table_slots || h->epoch >= 255) {
        DDCHK(h, hipMemsetAsync(S.table, 0, 8 * tsize, st));
        h->table_at = (void *)S.table;
        h->table_slots = tsize;
        h->epoch = 0;
    }
    S.epoch = ++h->epoch;
    DDCHK(h, hipEventRecord(h->ev[0], st));
    hipLaunchKernelGGL(dd_transform_kernel, dim3(tgrid), dim3(BLOCK), 0, st, d_arena, d_off, n, d_code, S);
    DDCHK(h, hipGetLastError());
    DDCHK(h, hipEventRecord(h->ev[1], st));
    // the byte-serial rows (rare): their slow-arena words are sized from the transform's count
    unsigned long long ns2[2];
    DDCHK(h, hipMemcpyAsync(ns2, S.nslow, sizeof(ns2), hipMemcpyDeviceToHost, st));
    DDCHK(h, hipStreamSynchronize(st));
    if (ns2[0]) {
        const size_t sbytes = 8 * (size_t)ns2[1] + 64;
        if (sbytes > h->sarena_bytes) {
            if (h->d_sarena) (void)hipFree(h->d_sarena);
            h->d_sarena = nullptr;
            h->sarena_bytes = 0;
            DDCHK(h, hipMalloc(&h->d_sarena, sbytes + sbytes / 4));
            h->sarena_bytes = sbytes + sbytes / 4;
        }
        S.sarena = (uint64_t *)h->d_sarena;
        const int sgrid = (int)std::min<uint64_t>((ns2[0] + BLOCK - 1) / BLOCK, (uint64_t)h->cus * 16);
        hipLaunchKernelGGL(dd_slow_kernel, dim3(sgrid), dim3(BLOCK), 0, st, d_arena, d_off, d_code, S, (uint64_t)ns2[0]);
        DDCHK(h, hipGetLastError());
    }
    DDCHK(h, hipEventRecord(h->ev[2], st));
    // decide: the pairs compared (8 lanes a pair), then the later rows of the differing ones against the table
    hipLaunchKernelGGL(dd_pairs_kernel, dim3((int)std::min<int64_t>((n_claims + 3) / 4, (int64_t)h->cus * h->pairs_bpc)),
                       dim3(BLOCK), 0, st, d_arena, d_code, S, n_claims, (uint64_t)ns2[0]);
    hipLaunchKernelGGL(dd_recheck_kernel, dim3(h->cus * 4), dim3(BLOCK), 0, st, d_arena, d_code, S);
    DDCHK(h, hipGetLastError());
    unsigned long long cnt[10];
    DDCHK(h, hipMemcpyAsync(cnt, S.cnt, sizeof(cnt), hipMemcpyDeviceToHost, st));
    DDCHK(h, hipStreamSynchronize(st));
    if (S.stats)
        fprintf(stderr, "kw_dedup: table lookups: %llu differing pairs\n", cnt[5]);
    // per code (the CODE_COLLIDE rows are added by resolve_collisions); KEPT: the rest
    h->counts[KW_URL_NO_HTML] = (int64_t)cnt[KW_URL_NO_HTML];
    h->counts[KW_URL_FILTERED] = (int64_t)cnt[KW_URL_FILTERED];
    h->counts[KW_URL_DUPLICATE] = (int64_t)cnt[KW_URL_DUPLICATE];
    h->counts[KW_URL_KEPT] = n - (int64_t)(cnt[KW_URL_NO_HTML] + cnt[KW_URL_FILTERED] + cnt[KW_URL_DUPLICATE] +
                                           cnt[CODE_COLLIDE]);
    if (cnt[CODE_COLLIDE]) {
        int rc = resolve_collisions(h, d_arena, d_off, n, d_code, st, cnt[9]);
        if (rc) return rc;
    }
    DDCHK(h, hipEventRecord(h->ev[3], st));
    hipLaunchKernelGGL(dd_count_kernel, dim3((unsigned)ntiles), dim3(BLOCK), 0, st, (const uint8_t *)d_code, n, S,
                       h->tile_cnt, h->tile_bytes);
    {   // the tiles' exclusive scan in two levels: chunk sums, their scan (one block), each chunk from its prefix
        const int64_t nchunk = std::min<int64_t>(SCAN_CHUNKS, ntiles);
        const int64_t per = (ntiles + nchunk - 1) / nchunk;
        hipLaunchKernelGGL(dd_tile_sums_kernel, dim3((unsigned)nchunk), dim3(BLOCK), 0, st,
                           (const unsigned long long *)h->tile_cnt, (const unsigned long long *)h->tile_bytes, ntiles,
                           per, h->chunk_cnt, h->chunk_bytes);
        hipLaunchKernelGGL(dd_scan_tiles_kernel, dim3(1), dim3(1024), 0, st, h->chunk_cnt, h->chunk_bytes, nchunk,
                           h->totals, nchunk, (const unsigned long long *)nullptr, (const unsigned long long *)nullptr);
        hipLaunchKernelGGL(dd_scan_tiles_kernel, dim3((unsigned)nchunk), dim3(1024), 0, st, h->tile_cnt, h->tile_bytes,
                           ntiles, (unsigned long long *)nullptr, per, (const unsigned long long *)h->chunk_cnt,
                           (const unsigned long long *)h->chunk_bytes);
    }
    hipLaunchKernelGGL(dd_place_kernel, dim3((unsigned)ntiles), dim3(BLOCK), 0, st, (const uint8_t *)d_code, n, S,
                       h->tile_cnt, h->tile_bytes, h->kept_off, h->kept_row);
    DDCHK(h, hipGetLastError());
    unsigned long long tot[2];
    DDCHK(h, hipMemcpyAsync(tot, h->totals, sizeof(tot), hipMemcpyDeviceToHost, st));
    DDCHK(h, hipStreamSynchronize(st));
    h->n_kept = (int64_t)tot[0];
    h->n_kept_bytes = (int64_t)tot[1];
    DDCHK(h, hipMemcpyAsync(h->kept_off + h->n_kept, &h->n_kept_bytes, 8, hipMemcpyHostToDevice, st));
    if ((size_t)h->n_kept_bytes + 64 > h->kept_bytes_cap) {
        if (h->d_kept) (void)hipFree(h->d_kept);
        h->d_kept = nullptr;
        h->kept_bytes_cap = 0;
        DDCHK(h, hipMalloc(&h->d_kept, (size_t)h->n_kept_bytes + 64));
        h->kept_bytes_cap = (size_t)h->n_kept_bytes + 64;
    }
    h->kept_bytes = (uint8_t *)h->d_kept;
    if (h->n_kept > 0) {
        const int cgrid = (int)std::min<int64_t>((h->n_kept + 63) / 64 * 64 / BLOCK + 1, (int64_t)h->cus * 8);
        if (kw_env("KW_DEDUP_COPY_LANE_ROW"))   // (A/B: the lane-per-row copy from global memory)
            hipLaunchKernelGGL(dd_copy_kernel, dim3(cgrid), dim3(BLOCK), 0, st, h->n_kept, (const int64_t *)h->kept_off,
                               (const int64_t *)h->kept_row, d_arena, S, h->kept_bytes);
        else
            hipLaunchKernelGGL(dd_copy_staged_kernel, dim3((int)std::min<int64_t>((h->n_kept + CPS_ROWS - 1) / CPS_ROWS,
                                                                                (int64_t)h->cus * h->copys_bpc)),
                               dim3(64), 0, st, h->n_kept, (const int64_t *)h->kept_off, (const int64_t *)h->kept_row,
                               d_arena, S, h->kept_bytes);
        DDCHK(h, hipGetLastError());
    }
    DDCHK(h, hipEventRecord(h->ev[4], st));
    DDCHK(h, hipStreamSynchronize(st));
    return KW_OK;
}

extern "C" int kw_dedup_counts(kw_dedup *h, int64_t *counts)
{
    if (!h || !counts) return KW_EINVAL;
    if (!h->have_run) { h->err = "kw_dedup_counts: no run"; return KW_ESTATE; }
    for (int k = 0; k < 4; ++k) counts[k] = h->counts[k];
    return KW_OK;
}

extern "C" int kw_dedup_kept_size(kw_dedup *h, int64_t *n_kept, int64_t *n_bytes)
{
    if (!h || !n_kept || !n_bytes) return KW_EINVAL;
    if (!h->have_run) { h->err = "kw_dedup_kept_size: no run"; return KW_ESTATE; }
    *n_kept = h->n_kept;
    *n_bytes = h->n_kept_bytes;
    return KW_OK;
}

extern "C" int kw_dedup_kept_copy(kw_dedup *h, uint8_t *d_bytes, int64_t *d_off, int64_t *d_rows, void *stream)
{
    if (!h) return KW_EINVAL;
    if (!h->have_run) { h->err = "kw_dedup_kept_copy: no run"; return KW_ESTATE; }
    DDCHK(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    if (h->n == 0 || h->n_kept == 0) {
        if (d_off) DDCHK(h, hipMemsetAsync(d_off, 0, 8, st));
        return KW_OK;
    }
    if (d_bytes && h->n_kept_bytes)
        DDCHK(h, hipMemcpyAsync(d_bytes, h->kept_bytes, (size_t)h->n_kept_bytes, hipMemcpyDeviceToDevice, st));
    if (d_off) DDCHK(h, hipMemcpyAsync(d_off, h->kept_off, 8 * ((size_t)h->n_kept + 1), hipMemcpyDeviceToDevice, st));
    if (d_rows) DDCHK(h, hipMemcpyAsync(d_rows, h->kept_row, 8 * (size_t)h->n_kept, hipMemcpyDeviceToDevice, st));
    return KW_OK;
}

extern "C" int kw_dedup_last_ms(kw_dedup *h, float *ms, int32_t k)
{
    if (!h || !ms) return KW_EINVAL;
    if (!h->have_run || h->n == 0) { for (int i = 0; i < k; ++i) ms[i] = 0.f; return KW_OK; }
    for (int i = 0; i < k && i < 4; ++i) DDCHK(h, hipEventElapsedTime(&ms[i], h->ev[i], h->ev[i + 1]));
    if (k > 4) DDCHK(h, hipEventElapsedTime(&ms[4], h->ev[0], h->ev[4]));
    return KW_OK;
}

extern "C" const char *kw_dedup_last_error(kw_dedup *h) { return h ? h->err.c_str() : "null handle"; }

extern "C" int kw_dedup_destroy(kw_dedup *h)
{
    if (!h) return KW_OK;
    (void)hipSetDevice(h->device);
    if (h->d_buf) (void)hipFree(h->d_buf);
    if (h->d_kept) (void)hipFree(h->d_kept);
    if (h->d_collide) (void)hipFree(h->d_collide);
    if (h->d_sarena) (void)hipFree(h->d_sarena);
    for (auto &e : h->ev)
        if (e) (void)hipEventDestroy(e);
    delete h;
    return KW_OK;
}

namespace {
__global__ void dd_keep_mask_kernel(const uint8_t *__restrict__ code, int64_t n, uint8_t *__restrict__ mask)
{
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLOCK)
        mask[i] = code[i] == KW_URL_KEPT ? 1 : 0;
}
}  // namespace

extern "C" int dedup_urls(const uint8_t *d_arena, const int64_t *d_off, int64_t n, uint8_t *d_keep_mask, void *stream)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return KW_EHIP;
    kw_dedup *h = nullptr;
    int rc = kw_dedup_create(dev, &h);
    if (rc == KW_OK) rc = kw_dedup_run(h, d_arena, d_off, n, KW_DEDUP_NORMALIZE, d_keep_mask, stream);
    if (rc == KW_OK && n > 0) {
        const int grid = (int)std::min<int64_t>((n + BLOCK - 1) / BLOCK, 4096);
        hipLaunchKernelGGL(dd_keep_mask_kernel, dim3(grid), dim3(BLOCK), 0, (hipStream_t)stream,
                           (const uint8_t *)d_keep_mask, n, d_keep_mask);
        if (hipGetLastError() != hipSuccess) rc = KW_EHIP;
        else if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) rc = KW_EHIP;
    }
    kw_dedup_destroy(h);
    return rc;
}
