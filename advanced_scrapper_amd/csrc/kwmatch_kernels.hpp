// HIP kernels of libkwmatch for gfx950 (MI355X).
//
// One wavefront owns one document at a time (grid-stride over documents):
//
//   scan     the document's bytes [text | title] stream through the wave in
//            1 KB tiles (16 B per lane, one global_load_dwordx4).  Every byte
//            position is tested against a 2^18-bit filter of the anchors'
//            3-byte prefixes held in LDS; survivors are compacted in position
//            order (wave prefix sum), probed in the global anchor hash table
//            and compared byte-exactly.  Uppercase-class names also check the
//            \b rule (match_keywords.py:167) on the neighbouring code points.
//            Each accepted anchor use becomes an "item" in the wave's scratch.
//   resolve  per field: items are sorted (bitonic, wave-cooperative), walked
//            per pattern, and turned into results:
//              U names  -> re.finditer positions (leftmost, non-overlapping)
//              F names  -> exact occurrence = score 100; otherwise the name's
//                          pieces (pigeonhole) seed bit-parallel LCS over the
//                          rapidfuzz partial_ratio window family (> 95 rule);
//                          decided names get re.finditer(name) positions
//                          (literal search or the regex atom program).
//            Fields no longer than 64 code points also take the "short path"
//            where the field is the needle and the names are the haystacks.
//
// All arithmetic is integer; results are bit-exact with the CPU oracle.
#pragma once
#include "kwmatch_device.hpp"

// profiling builds: 0 = filter only, 1 = + anchor probe, 2 = + resolve w/o LCS, 3 = full
#ifndef KW_STAGE
#define KW_STAGE 3
#endif

namespace kw {

// ------------------------------------------------------------------ wave utils
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (WAVE - 1)); }

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// make this wave's global-memory stores visible to its own other lanes
__device__ __forceinline__ void wave_sync_global()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t mbcnt(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int wave_excl_scan(int v, int *total)
{
    const int lane = lane_id();
    int x = v;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        int y = __shfl_up(x, d, WAVE);
        if (lane >= d) x += y;
    }
    *total = __shfl(x, WAVE - 1, WAVE);
    return x - v;
}

// the same exclusive scan with DPP row shifts and row broadcasts (no LDS traffic, no bpermute latency chain);
// total = the wave's sum
__device__ __forceinline__ int wave_excl_scan_dpp(int v, int *total)
{
    int x = v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    *total = __builtin_amdgcn_readlane(x, WAVE - 1);
    return x - v;
}

__device__ __forceinline__ int wave_sum(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, WAVE);
    return v;
}

// ------------------------------------------------------------------ text utils
__device__ __forceinline__ bool is_word_cp(const DevTables &T, uint32_t c)
{
    if (c < 128) {
        return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
    }
    if (c >= 0x110000u) return false;
    return (T.word_bits[c >> 5] >> (c & 31)) & 1u;
}

// decode the code point starting at p (p < e); returns its byte length
__device__ __forceinline__ uint32_t decode_at(const uint8_t *__restrict__ a, int64_t p, int64_t e, uint32_t *cp)
{
    uint32_t b0 = a[p];
    if (b0 < 0x80) { *cp = b0; return 1; }
    uint32_t n = (b0 >= 0xF0) ? 4 : (b0 >= 0xE0) ? 3 : 2;
    uint32_t c = b0 & (0x7F >> n);
    for (uint32_t k = 1; k < n; ++k) {
        uint32_t b = (p + k < e) ? a[p + k] : 0x80;
        c = (c << 6) | (b & 0x3F);
    }
    *cp = c;
    return n;
}

// code point that ends right before byte p (p > s)
__device__ __forceinline__ uint32_t decode_before(const uint8_t *__restrict__ a, int64_t s, int64_t p)
{
    int64_t q = p - 1;
    while (q > s && (a[q] & 0xC0) == 0x80 && p - q < 4) --q;
    uint32_t cp;
    decode_at(a, q, p, &cp);
    return cp;
}

// ------------------------------------------------------------------ per-wave context
struct FieldCtx {
    const uint8_t *arena;
    int64_t fb, fe;         // byte range
    uint32_t n;             // code points
    bool ascii;
    const uint32_t *cps;    // decoded code points (non-ASCII fields)
    const uint32_t *blkcnt; // cumulative lead-byte counts per 64 B block
    uint32_t doc, field;
    bool tx = false;        // the epilogue's transcoded view (ascii: one byte per code point, markers >= 0x80)
};

__device__ __forceinline__ uint32_t fcp(const FieldCtx &F, uint32_t i)
{
    return F.ascii ? (uint32_t)F.arena[F.fb + i] : F.cps[i];
}

// byte offset (field relative) -> code-point offset
__device__ __forceinline__ uint32_t to_cp(const FieldCtx &F, uint32_t bpos)
{
    if (F.ascii) return bpos;
    uint32_t blk = bpos >> 6;
    uint32_t c = F.blkcnt[blk];
    for (uint32_t i = blk << 6; i < bpos; ++i) c += ((F.arena[F.fb + i] & 0xC0) != 0x80);
    return c;
}

struct OutCtx {
    kw_hit *out;
    uint32_t cap;
    uint32_t n;        // wave-uniform running count
    uint32_t *shared;  // non-null: the count lives here and several waves append (atomics)
};

// every lane with `emit` appends one record (order: lane order)
__device__ __forceinline__ void emit_hits(OutCtx &O, const DevScratch &S, bool emit, uint32_t doc, uint32_t pat,
                                          uint32_t pos, uint32_t field)
{
    uint64_t m = __ballot(emit);
    if (!m) return;
    uint32_t r = mbcnt(m);
    if (O.shared) {
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(O.shared, (uint32_t)__popcll(m));
        O.n = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
    }
    uint32_t idx = O.n + r;
    if (emit) {
        if (idx < O.cap) {
            kw_hit h;
            h.doc = doc;
            h.pattern = pat;
            h.pos = pos;
            h.field = field;
            O.out[idx] = h;
        } else {
            atomicOr(&S.status[0], ST_OUT_OVERFLOW);
        }
    }
    O.n += (uint32_t)__popcll(m);
}

// ------------------------------------------------------------------ bit-parallel LCS helpers
__device__ __forceinline__ uint64_t pm_lookup(const DevTables &T, uint32_t pat, uint32_t c)
{
    if (c < 128) return T.pm_ascii[(size_t)pat * 128 + c];
    uint32_t b = T.pm_ext_off[pat], e = T.pm_ext_off[pat + 1];
    for (uint32_t k = b; k < e; ++k)
        if (T.pm_ext_cp[k] == c) return T.pm_ext_mask[k];
    return 0;
}

__device__ __forceinline__ uint64_t lcs_step(uint64_t V, uint64_t M)
{
    uint64_t U = V & M;
    return (V + U) | (V - U);
}

__device__ __forceinline__ uint64_t low_mask(uint32_t m) { return m >= 64 ? ~0ull : ((1ull << m) - 1); }

__device__ __forceinline__ bool passes(uint32_t lcs, uint32_t l1, uint32_t lw)
{
    uint32_t lensum = l1 + lw;
    return 20u * (lensum - 2u * lcs) < lensum;
}

// max indel distance of a full window: LCS >= m - kfull(m)
__device__ __forceinline__ uint32_t kfull(uint32_t m)
{
    uint32_t k = 0;
    while (20u * (k + 1) < m) ++k;   // 20*(m - L) < m with L = m - k
    return k;
}

// ------------------------------------------------------------------ regex atoms
// greedy backtracking matcher for the atom subset; returns end or -1
__device__ int rx_match(const DevTables &T, const FieldCtx &F, uint32_t pat, uint32_t s)
{
    const uint32_t ab = T.rx_off[pat], ae = T.rx_off[pat + 1];
    const uint32_t na = ae - ab;
    int st_atom[RX_MAX_QUANT], st_pos[RX_MAX_QUANT], st_cnt[RX_MAX_QUANT];
    int sp = 0;
    uint32_t a = 0;
    int pos = (int)s;
    const int n = (int)F.n;
    for (;;) {
        bool fail = false;
        if (a == na) return pos;
        int4 at = T.rx_atoms[ab + a];
        if (at.z == 1 && at.w == 1) {
            if (pos < n) {
                uint32_t c = fcp(F, (uint32_t)pos);
                bool ok = (at.x == KW_RX_LIT) ? (c == (uint32_t)at.y) : (c != '\n');
                if (ok) { ++pos; ++a; continue; }
            }
            fail = true;
        } else {
            int k = 0;
            while ((at.w < 0 || k < at.w) && pos + k < n) {
                uint32_t c = fcp(F, (uint32_t)(pos + k));
                bool ok = (at.x == KW_RX_LIT) ? (c == (uint32_t)at.y) : (c != '\n');
                if (!ok) break;
                ++k;
            }
            if (k < at.z) {
                fail = true;
            } else {
                st_atom[sp] = (int)a; st_pos[sp] = pos; st_cnt[sp] = k; ++sp;
                pos += k;
                ++a;
                continue;
            }
        }
        if (fail) {
            bool resumed = false;
            while (sp > 0) {
                int t = sp - 1;
                int4 qa = T.rx_atoms[ab + st_atom[t]];
                if (st_cnt[t] > qa.z) {
                    st_cnt[t]--;
                    pos = st_pos[t] + st_cnt[t];
                    a = (uint32_t)st_atom[t] + 1;
                    resumed = true;
                    break;
                }
                --sp;
            }
            if (!resumed) return -1;
        }
    }
}

// wave-cooperative re.finditer positions of a regex-program pattern; returns count emitted
__device__ uint32_t rx_positions(const DevTables &T, const DevScratch &S, const FieldCtx &F, OutCtx &O, uint32_t pat)
{
    const int lane = lane_id();
    uint32_t last_end = 0, emitted = 0;
    for (uint32_t s0 = 0; s0 < F.n; s0 += WAVE) {
        uint32_t s = s0 + lane;
        int e = (s < F.n) ? rx_match(T, F, pat, s) : -1;
        uint64_t m = __ballot(e >= 0);
        uint64_t keep = 0;
        while (m) {
            int l = __builtin_ctzll(m);
            m &= m - 1;
            uint32_t st = s0 + (uint32_t)l;
            int en = __shfl(e, l, WAVE);
            if (st >= last_end) {
                keep |= 1ull << l;
                last_end = (uint32_t)en > st ? (uint32_t)en : st + 1;
            }
        }
        emit_hits(O, S, (keep >> lane) & 1ull, F.doc, pat, s, F.field);
        emitted += (uint32_t)__popcll(keep);
    }
    return emitted;
}

// ------------------------------------------------------------------ sorting
// wave bitonic sort of n (power of two) u64 keys in the wave's scratch
__device__ void wave_sort_global(uint64_t *a, uint32_t n)
{
    const int lane = lane_id();
    for (uint32_t k = 2; k <= n; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
                uint32_t i = i0 + lane;
                uint32_t l = i ^ j;
                if (i < n && l > i) {
                    uint64_t x = a[i], y = a[l];
                    bool up = (i & k) == 0;
                    if ((x > y) == up) { a[i] = y; a[l] = x; }
                }
            }
            wave_sync_global();
        }
    }
}

// sort up to 64 keys held one per lane (pad with ~0)
__device__ __forceinline__ uint64_t wave_sort_reg(uint64_t x)
{
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= WAVE; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            uint64_t y = __shfl_xor(x, j, WAVE);
            bool up = (lane & k) == 0;
            bool lower = (lane & j) == 0;
            // lower lane keeps min when ascending
            bool take_min = (lower == up);
            uint64_t mn = x < y ? x : y, mx = x < y ? y : x;
            x = take_min ? mn : mx;
        }
    }
    return x;
}

// ------------------------------------------------------------------ resolve helpers
__device__ __forceinline__ uint32_t it_pat(uint64_t it) { return (uint32_t)(it >> IT_PAT_SHIFT); }
__device__ __forceinline__ uint32_t it_pos(uint64_t it) { return (uint32_t)((it >> IT_POS_SHIFT) & IT_POS_MASK); }
__device__ __forceinline__ uint32_t it_kind(uint64_t it) { return (uint32_t)((it >> IT_KIND_SHIFT) & 3u); }
__device__ __forceinline__ uint32_t it_use(uint64_t it) { return (uint32_t)(it & IT_USE_MASK); }

// greedy leftmost non-overlapping selection over the items [gs, ge) of one
// pattern whose kind == want (positions sorted ascending); blen = match bytes.
__device__ uint32_t emit_nonoverlap(const DevScratch &S, const FieldCtx &F, OutCtx &O, const uint64_t *items,
                                    uint32_t gs, uint32_t ge, uint32_t want, uint32_t blen, uint32_t pat)
{
    const int lane = lane_id();
    uint32_t last_end = 0, emitted = 0;
    bool have_last = false;
    for (uint32_t c = gs; c < ge; c += WAVE) {
        uint32_t i = c + lane;
        bool valid = false;
        uint32_t pos = 0;
        if (i < ge) {
            uint64_t it = items[i];
            valid = it_kind(it) == want;
            pos = it_pos(it);
        }
        uint64_t vm = __ballot(valid);
        uint64_t keep = 0;
        // fast path: no valid item overlaps the previous valid one
        int prev_l = -1;
        uint32_t prev_end = last_end;
        bool prev_have = have_last;
        uint64_t mm = vm;
        while (mm) {
            int l = __builtin_ctzll(mm);
            mm &= mm - 1;
            uint32_t p = (uint32_t)__shfl((int)pos, l, WAVE);
            if (!prev_have || p >= prev_end) {
                keep |= 1ull << l;
                prev_end = p + blen;
                prev_have = true;
            }
            prev_l = l;
        }
        (void)prev_l;
        last_end = prev_end;
        have_last = prev_have;
        bool k = (keep >> lane) & 1ull;
        emit_hits(O, S, k, F.doc, pat, k ? to_cp(F, pos) : 0, F.field);
        emitted += (uint32_t)__popcll(keep);
    }
    return emitted;
}

}  // namespace kw

namespace kw {

// ------------------------------------------------------------------ fuzzy verification
// One PIECE occurrence (this lane): does any window of the partial_ratio family
// that contains it pass 20*d < n1+|W|?  (needle = name, m < n)
__device__ bool verify_piece(const DevTables &T, const FieldCtx &F, uint32_t P, uint32_t m, uint32_t q, uint32_t o,
                             uint32_t plen, unsigned long long &nwin)
{
    if (KW_STAGE < 3) return false;
    const uint32_t n = F.n;
    const uint64_t mask = low_mask(m);
    const uint32_t k = kfull(m);
    if (k > 0) {   // full windows text[p:p+m], p in [q-o-k, q-o+k]
        int pmin = (int)q - (int)o - (int)k, pmax = (int)q - (int)o + (int)k;
        if (pmin < 0) pmin = 0;
        if (pmax > (int)(n - m)) pmax = (int)(n - m);
        for (int p = pmin; p <= pmax; ++p) {
            uint64_t V = ~0ull;
            for (uint32_t j = 0; j < m; ++j) V = lcs_step(V, pm_lookup(T, P, fcp(F, (uint32_t)p + j)));
            ++nwin;
            uint32_t L = (uint32_t)__popcll(~V & mask);
            if (20u * (m - L) < m) return true;
        }
    }
    if (q + plen <= m - 1) {   // prefixes text[:w], w in [1, m)
        uint64_t V = ~0ull;
        ++nwin;
        for (uint32_t w = 1; w < m; ++w) {
            V = lcs_step(V, pm_lookup(T, P, fcp(F, w - 1)));
            if (passes((uint32_t)__popcll(~V & mask), m, w)) return true;
        }
    }
    if (q + m > n) {           // suffixes text[i:], i in (n-m, n)
        uint64_t V = ~0ull;
        ++nwin;
        for (uint32_t kk = 1; kk < m; ++kk) {
            uint32_t i = n - kk;
            uint64_t M = __brevll(pm_lookup(T, P, fcp(F, i))) >> (64 - m);
            V = lcs_step(V, M);
            if (passes((uint32_t)__popcll(~V & mask), m, kk)) return true;
        }
    }
    return false;
}

// Pieces of one occurrence of a name share its alignment base = q - o, and the window family a
// piece is verified over depends only on the base and on whether prefix (q + pl + 1 <= m) or suffix
// (q + m > n) windows can contain the piece: a piece whose key equals the last verified one is
// skipped.
__device__ __forceinline__ int64_t piece_window_key(uint32_t q, uint32_t o, uint32_t pl, uint32_t m, uint32_t n)
{
    const int64_t base = (int64_t)q - (int64_t)o;
    const int64_t pre = q + pl + 1 <= m ? 1 : 0, suf = q + m > n ? 1 : 0;
    return ((base + (1ll << 40)) << 2) | (pre << 1) | suf;
}

// the fast path's wave-cooperative verification (kwmatch_fast_kernel.hpp)
__device__ bool fk_verify_piece(const FieldCtx &F, uint32_t nm, uint32_t m, uint32_t q, uint32_t o, uint32_t pl,
                                unsigned long long &nwin);

// ------------------------------------------------------------------ resolve
__device__ void process_group(const DevTables &T, const DevScratch &S, const FieldCtx &F, OutCtx &O,
                              const uint64_t *items, uint32_t gs, uint32_t ge, uint32_t P, unsigned long long &nwin)
{
    const int lane = lane_id();
    const uint32_t pi = T.pat_info[P];
    const uint32_t m = pi_m(pi), blen = pi_blen(pi);
    if (!(pi & PI_FUZZY)) {
        emit_nonoverlap(S, F, O, items, gs, ge, USE_UPPER, blen, P);
        return;
    }
    if (m >= F.n) return;   // the short path owns names at least as long as the field
    bool decided = false;
    for (uint32_t c = gs; c < ge && !decided; c += WAVE) {
        uint32_t i = c + lane;
        bool full = (i < ge) && it_kind(items[i]) == USE_FULL;
        decided = __ballot(full) != 0;
    }
    // pieces wave-serially, each by the wave-cooperative bit-parallel LCS (name code points one per
    // lane, match vectors by ballot); one verification per window key
    const uint32_t nm = (lane < (int)m) ? T.pat_cps[T.pat_cp_off[P] + lane] : 0xFFFFFFFDu;
    int64_t last_key = -1;
    for (uint32_t c = gs; c < ge && !decided; c += WAVE) {
        const uint32_t i = c + lane;
        const bool piece = i < ge && it_kind(items[i]) == USE_PIECE;
        uint32_t q = 0, info = 0;
        if (piece) {
            q = to_cp(F, it_pos(items[i]));
            info = T.use_info[it_use(items[i])];
        }
        uint64_t pm = __ballot(piece);
        while (pm && !decided) {
            const int l = __builtin_ctzll(pm);
            pm &= pm - 1;
            const uint32_t lq = (uint32_t)__builtin_amdgcn_readlane((int)q, l);
            const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)info, l);
            const uint32_t o = (li >> 8) & 0xFF, plen = (li >> 16) & 0xFF;
            const int64_t key = piece_window_key(lq, o, plen, m, F.n);
            if (key == last_key) continue;
            last_key = key;
            decided = fk_verify_piece(F, nm, m, lq, o, plen, nwin);
        }
    }
    if (!decided) return;
    uint32_t cnt = (pi & PI_LITERAL) ? emit_nonoverlap(S, F, O, items, gs, ge, USE_FULL, blen, P)
                                     : rx_positions(T, S, F, O, P);
    if (cnt == 0) emit_hits(O, S, lane == 0, F.doc, P, KW_NOPOS, F.field);
}

// positions of a decided short-path pattern held by lane `l`
__device__ void short_emit(const DevTables &T, const DevScratch &S, const FieldCtx &F, OutCtx &O, uint64_t dec,
                           uint64_t exact, uint32_t pbase)
{
    const int lane = lane_id();
    // literal names: re.finditer(name, s) finds the name only when it equals the field
    uint64_t lit = 0;
    uint64_t mm = dec;
    while (mm) {
        int l = __builtin_ctzll(mm);
        mm &= mm - 1;
        uint32_t P = pbase + (uint32_t)l;
        uint32_t pi = T.pat_info[P];
        if (pi & PI_LITERAL) {
            lit |= 1ull << l;
        } else {
            uint32_t cnt = rx_positions(T, S, F, O, P);
            if (cnt == 0) emit_hits(O, S, lane == 0, F.doc, P, KW_NOPOS, F.field);
        }
    }
    bool me = (lit >> lane) & 1ull;
    bool ex = (exact >> lane) & 1ull;
    emit_hits(O, S, me, F.doc, pbase + lane, ex ? 0u : KW_NOPOS, F.field);
}

__device__ void short_path(const DevTables &T, const DevScratch &S, const FieldCtx &F, OutCtx &O, uint64_t *lpm,
                           uint32_t *lext_cp, uint64_t *lext_mask, unsigned long long &nwin)
{
    const int lane = lane_id();
    const uint32_t n = F.n;
    if (n == 0) {
        if (T.empty_pat >= 0) emit_hits(O, S, lane == 0, F.doc, (uint32_t)T.empty_pat, 0u, F.field);
        return;
    }
    if (n <= (uint32_t)SHORT_EXACT_MAX) {
        // the field must occur verbatim inside the name: look it up in the
        // table of all name substrings of <= SHORT_EXACT_MAX code points
        uint64_t h = 0;
        for (uint32_t i = 0; i < n; ++i) h = h * SUB_B + fcp(F, i);
        uint64_t key = (h + (uint64_t)n * 0x9E3779B97F4A7C15ull) | 1ull;
        uint32_t slot = (uint32_t)(key >> 32) & T.sub_mask;
        uint32_t b = 0, cnt = 0;
        for (;;) {
            uint64_t kk = T.sub_key[slot];
            if (kk == key) { b = T.sub_begin[slot]; cnt = T.sub_cnt[slot]; break; }
            if (kk == 0) break;
            slot = (slot + 1) & T.sub_mask;
        }
        b = __builtin_amdgcn_readfirstlane(b);
        cnt = __builtin_amdgcn_readfirstlane(cnt);
        for (uint32_t c0 = 0; c0 < cnt; c0 += WAVE) {
            uint32_t idx = c0 + lane;
            bool hit = false, exact = false;
            uint32_t P = 0;
            if (idx < cnt) {
                const uint32_t e = T.sub_pat[b + idx];
                P = e & 0xFFFFFu;
                uint32_t m = pi_m(T.pat_info[P]);
                const uint32_t *nm = T.pat_cps + T.pat_cp_off[P];
                {   // the substring's recorded offset first, every offset if the hash collided
                    const uint32_t p = e >> 20;
                    bool eq = p + n <= m;
                    for (uint32_t j = 0; j < n && eq; ++j) eq = nm[p + j] == fcp(F, j);
                    hit = eq;
                }
                for (uint32_t p = 0; p + n <= m && !hit; ++p) {
                    bool eq = true;
                    for (uint32_t j = 0; j < n; ++j)
                        if (nm[p + j] != fcp(F, j)) { eq = false; break; }
                    hit = eq;
                }
                exact = hit && (m == n);
            }
            // patterns in this list are not contiguous: emit one by one
            uint64_t dm = __ballot(hit);
            uint64_t em = __ballot(exact);
            while (dm) {
                int l = __builtin_ctzll(dm);
                dm &= dm - 1;
                uint32_t PP = (uint32_t)__shfl((int)P, l, WAVE);
                uint32_t pi = T.pat_info[PP];
                if (pi & PI_LITERAL) {
                    emit_hits(O, S, lane == 0, F.doc, PP, ((em >> l) & 1ull) ? 0u : KW_NOPOS, F.field);
                } else {
                    uint32_t c = rx_positions(T, S, F, O, PP);
                    if (c == 0) emit_hits(O, S, lane == 0, F.doc, PP, KW_NOPOS, F.field);
                }
            }
        }
        return;
    }
    const uint32_t count = (uint32_t)T.f_count_ge[n];
    if (count == 0) return;
    // pattern-match vectors of the field (the needle) in LDS
    lpm[lane] = 0;
    lpm[lane + 64] = 0;
    wave_sync();
    uint32_t n_ext = 0;
    {
        uint32_t c = (lane < (int)n) ? fcp(F, (uint32_t)lane) : 0xFFFFFFFFu;
        if (c < 128) atomicOr((unsigned long long *)&lpm[c], 1ull << lane);
        uint64_t nonascii = __ballot(c != 0xFFFFFFFFu && c >= 128);
        while (nonascii) {   // uniform: build the extended list
            int l = __builtin_ctzll(nonascii);
            nonascii &= nonascii - 1;
            uint32_t cc = (uint32_t)__shfl((int)c, l, WAVE);
            uint32_t k = 0;
            while (k < n_ext && lext_cp[k] != cc) ++k;
            if (lane == 0) {
                if (k == n_ext) { lext_cp[k] = cc; lext_mask[k] = 0; }
                lext_mask[k] |= 1ull << l;
            }
            if (k == n_ext) ++n_ext;
            wave_sync();
        }
    }
    wave_sync();
    const uint64_t maskn = low_mask(n);
    auto fpm = [&](uint32_t c) -> uint64_t {
        if (c < 128) return lpm[c];
        for (uint32_t k = 0; k < n_ext; ++k)
            if (lext_cp[k] == c) return lext_mask[k];
        return 0ull;
    };
    for (uint32_t c0 = 0; c0 < count; c0 += WAVE) {
        uint32_t idx = c0 + lane;
        bool pass = false, exact = false;
        const uint32_t P = (uint32_t)T.f_first + idx;
        if (idx < count) {
            const uint32_t m = pi_m(T.pat_info[P]);
            const uint32_t *nm = T.pat_cps + T.pat_cp_off[P];
            uint64_t Vf = ~0ull;
            for (uint32_t p = 0; p + n <= m && !pass; ++p) {   // full windows of the name
                uint64_t V = ~0ull;
                for (uint32_t j = 0; j < n; ++j) V = lcs_step(V, fpm(nm[p + j]));
                ++nwin;
                if (p == 0) Vf = V;
                uint32_t L = (uint32_t)__popcll(~V & maskn);
                if (20u * (n - L) < n) pass = true;
                if (L == n && m == n) exact = true;
            }
            if (!pass) {   // prefixes name[:i]
                uint64_t V = ~0ull;
                for (uint32_t i = 1; i < n && !pass; ++i) {
                    V = lcs_step(V, fpm(nm[i - 1]));
                    if (passes((uint32_t)__popcll(~V & maskn), n, i)) pass = true;
                }
            }
            uint64_t Vr = ~0ull;
            if (!pass) {   // suffixes name[i:], i in (m-n, m)
                uint64_t V = ~0ull;
                for (uint32_t kk = 1; kk < n && !pass; ++kk) {
                    uint32_t i = m - kk;
                    V = lcs_step(V, __brevll(fpm(nm[i])) >> (64 - n));
                    if (passes((uint32_t)__popcll(~V & maskn), n, kk)) pass = true;
                }
            }
            if (!pass && m == n) {
                // the swapped run: needle = name, windows = prefixes / suffixes of the field
                Vr = ~0ull;
                for (uint32_t j = 0; j < m; ++j) Vr = lcs_step(Vr, __brevll(fpm(nm[m - 1 - j])) >> (64 - n));
                for (uint32_t i = 1; i < n && !pass; ++i) {
                    if (passes((uint32_t)__popcll(~Vf & low_mask(i)), m, i)) pass = true;
                    if (passes((uint32_t)__popcll(~Vr & low_mask(n - i)), m, n - i)) pass = true;
                }
            }
        }
        uint64_t dec = __ballot(pass);
        uint64_t ex = __ballot(exact);
        if (dec) short_emit(T, S, F, O, dec, ex, (uint32_t)T.f_first + c0);
    }
}

__device__ void resolve_field(const DevTables &T, const DevScratch &S, const FieldCtx &F, OutCtx &O, uint64_t *items,
                              uint32_t N, uint64_t *lpm, uint32_t *lext_cp, uint64_t *lext_mask,
                              unsigned long long &nwin)
{
    const int lane = lane_id();
    if (N > 0) {
        uint32_t n2 = 1;
        while (n2 < N) n2 <<= 1;
        if (n2 <= (uint32_t)WAVE) {
            uint64_t x = (lane < (int)N) ? items[lane] : ~0ull;
            x = wave_sort_reg(x);
            if (lane < (int)N) items[lane] = x;
            wave_sync_global();
        } else {
            for (uint32_t i = N + lane; i < n2; i += WAVE) items[i] = ~0ull;
            wave_sync_global();
            wave_sort_global(items, n2);
        }
        uint32_t gs = 0;
        while (gs < N) {
            const uint32_t P = __builtin_amdgcn_readfirstlane(it_pat(items[gs]));
            uint32_t ge = N;
            for (uint32_t c = gs;; c += WAVE) {
                uint32_t i = c + lane;
                bool diff = (i >= N) || it_pat(items[i]) != P;
                uint64_t m = __ballot(diff);
                if (m) { ge = c + (uint32_t)__builtin_ctzll(m); break; }
            }
            process_group(T, S, F, O, items, gs, ge, P, nwin);
            gs = ge;
        }
    }
    if (F.n <= (uint32_t)MAXM) short_path(T, S, F, O, lpm, lext_cp, lext_mask, nwin);
}

// decode a non-ASCII field into code points (+ per-64-byte cumulative counts)
__device__ uint32_t decode_field(const DevScratch &S, const uint8_t *__restrict__ arena, int64_t fb, int64_t fe,
                                 uint32_t *cps, uint32_t *blkcnt)
{
    const int lane = lane_id();
    const int64_t L = fe - fb;
    uint32_t cnt = 0;
    for (int64_t b0 = 0; b0 < L; b0 += WAVE) {
        int64_t i = b0 + lane;
        bool valid = i < L;
        uint32_t byte = valid ? arena[fb + i] : 0x80u;
        bool lead = valid && ((byte & 0xC0) != 0x80);
        uint64_t m = __ballot(lead);
        uint32_t idx = cnt + mbcnt(m);
        if (lead && idx < S.cp_cap) {
            uint32_t cp;
            decode_at(arena, fb + i, fe, &cp);
            cps[idx] = cp;
        }
        if (lane == 0 && (b0 >> 6) < (int64_t)(S.cp_cap / 16)) blkcnt[b0 >> 6] = cnt;
        cnt += (uint32_t)__popcll(m);
    }
    if ((cnt > S.cp_cap || L > (int64_t)S.cp_cap * 4) && lane == 0) {
        // the host grows the code point buffers to the largest need and runs the scan again
        atomicOr(&S.status[0], ST_CP_OVERFLOW);
        atomicMax(&S.gmax[1], (uint32_t)(L < 0xFFFFFFFFll ? L : 0xFFFFFFFFll));
    }
    wave_sync_global();
    return cnt;
}

// ------------------------------------------------------------------ scan
__device__ __forceinline__ uint64_t load8(const uint8_t *__restrict__ a, int64_t p)
{
    const int64_t a0 = p & ~(int64_t)3;
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t x0 = *(const uint32_t *)(a + a0);
    const uint32_t x1 = *(const uint32_t *)(a + a0 + 4);
    const uint32_t x2 = *(const uint32_t *)(a + a0 + 8);
    const uint32_t lo = __builtin_amdgcn_alignbyte(x1, x0, s);
    const uint32_t hi = __builtin_amdgcn_alignbyte(x2, x1, s);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ void process_candidate(const DevTables &T, const DevScratch &S, const uint8_t *__restrict__ arena,
                                  int64_t t0, int64_t t1, int64_t t2, uint32_t rel, uint64_t *items0, uint64_t *items1,
                                  uint32_t *icnt, unsigned long long &nanchor)
{
    const int64_t p = t0 + rel;
    const int f = p < t1 ? 0 : 1;
    const int64_t fb = f ? t1 : t0, fe = f ? t2 : t1;
    const uint64_t h8 = load8(arena, p);
    const uint32_t key = (uint32_t)(h8 & 0xFFFFFFu);
    uint32_t slot = (key * HASH_MUL) >> T.ht_shift;
    uint32_t kb = 0, kc = 0;
    for (;;) {
        uint32_t kk = T.ht_key[slot];
        if (kk == key) { kb = T.ht_begin[slot]; kc = T.ht_cnt[slot]; break; }
        if (kk == 0xFFFFFFFFu) break;
        slot = (slot + 1) & T.ht_mask;
    }
    uint64_t *items = f ? items1 : items0;
    for (uint32_t t = 0; t < kc; ++t) {
        const uint32_t a = T.kl_anchor[kb + t];
        const uint32_t len = T.as_len[a];
        if (p + (int64_t)len > fe) continue;
        const uint64_t m8 = len >= 8 ? ~0ull : ((1ull << (8 * len)) - 1);
        if ((h8 ^ T.as_head[a]) & m8) continue;
        if (len > 8) {
            const uint8_t *ab = T.as_bytes + T.as_off[a];
            bool eq = true;
            for (uint32_t x = 8; x < len; ++x)
                if (arena[p + x] != ab[x]) { eq = false; break; }
            if (!eq) continue;
        }
        ++nanchor;
        const uint32_t ub = T.as_use_begin[a], uc = T.as_use_cnt[a];
        for (uint32_t u = ub; u < ub + uc; ++u) {
            const uint32_t info = T.use_info[u];
            const uint32_t kind = info & 3u;
            const uint32_t pat = T.use_pat[u];
            if (kind == USE_UPPER) {
                const uint32_t pi = T.pat_info[pat];
                const bool wf = (pi & PI_WORD_FIRST) != 0, wl = (pi & PI_WORD_LAST) != 0;
                const bool wp = (p > fb) ? is_word_cp(T, decode_before(arena, fb, p)) : false;
                if (wp == wf) continue;
                bool wn = false;
                if (p + (int64_t)len < fe) {
                    uint32_t c;
                    decode_at(arena, p + len, fe, &c);
                    wn = is_word_cp(T, c);
                }
                if (wn == wl) continue;
            }
            const uint64_t item = ((uint64_t)pat << IT_PAT_SHIFT) | ((uint64_t)(p - fb) << IT_POS_SHIFT) |
                                  ((uint64_t)kind << IT_KIND_SHIFT) | (uint64_t)u;
            const uint32_t idx = atomicAdd(&icnt[f], 1u);
            if (idx < S.item_cap) items[idx] = item;
            else { atomicOr(&S.status[0], ST_ITEM_OVERFLOW); atomicMax(&S.gmax[0], idx + 1); }   // grown + rescanned
        }
    }
}

__global__ __launch_bounds__(BLOCK) void kw_scan_kernel(DevTables T, const uint8_t *__restrict__ arena,
                                                        const int64_t *__restrict__ off, int64_t n_docs, DevScratch S,
                                                        const uint32_t *__restrict__ doc_list,
                                                        const uint32_t *__restrict__ list_cnt, uint32_t list_cap)
{
    // doc_list != nullptr: process only the listed documents (the fast kernel's deferrals)
    if (doc_list) {
        uint32_t c = *list_cnt;
        n_docs = c < list_cap ? c : list_cap;
    }
    if ((int64_t)blockIdx.x * WAVES_PER_BLOCK >= n_docs) return;   // no document for any wave of this block
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    uint32_t *filt = (uint32_t *)smem_raw;
    uint64_t *pm_all = (uint64_t *)(filt + FILT_WORDS);                 // WAVES*128
    uint64_t *extm_all = pm_all + WAVES_PER_BLOCK * 128;                // WAVES*64
    uint32_t *cand_all = (uint32_t *)(extm_all + WAVES_PER_BLOCK * 64); // WAVES*CAND_CAP
    uint32_t *extc_all = cand_all + WAVES_PER_BLOCK * CAND_CAP;         // WAVES*64
    uint32_t *icnt_all = extc_all + WAVES_PER_BLOCK * 64;               // WAVES*2

    for (int i = threadIdx.x; i < FILT_WORDS; i += BLOCK) filt[i] = T.filt[i];
    __syncthreads();

    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t wave = (int64_t)blockIdx.x * WAVES_PER_BLOCK + wib;
    const int64_t n_waves = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    uint32_t *cand = cand_all + wib * CAND_CAP;
    uint64_t *lpm = pm_all + wib * 128;
    uint64_t *lext_mask = extm_all + wib * 64;
    uint32_t *lext_cp = extc_all + wib * 64;
    uint32_t *icnt = icnt_all + wib * 2;
    uint64_t *items0 = S.items + (size_t)wave * 2 * S.item_cap;
    uint64_t *items1 = items0 + S.item_cap;
    uint32_t *cps = S.cps + (size_t)wave * S.cp_cap;
    uint32_t *blkcnt = S.blkcnt + (size_t)wave * (S.cp_cap / 16 + 2);

    OutCtx O;
    O.shared = nullptr;
    O.out = S.out + (size_t)wave * S.out_cap;
    O.cap = S.out_cap;
    O.n = 0;
    unsigned long long ncand = 0, nanchor = 0, nwin = 0;

    for (int64_t di = wave; di < n_docs; di += n_waves) {
        const int64_t d = doc_list ? (int64_t)doc_list[di] : di;
        const int64_t t0 = off[2 * d], t1 = off[2 * d + 1], t2 = off[2 * d + 2];
        if (t1 - t0 > MAX_FIELD_BYTES || t2 - t1 > MAX_FIELD_BYTES) {
            if (lane == 0) atomicOr(&S.status[0], ST_FIELD_TOO_LONG);
            continue;
        }
        if (lane < 2) icnt[lane] = 0;
        wave_sync();
        uint32_t cpt = 0, cpu = 0;
        bool na0 = false, na1 = false;
        const int64_t base = t0 & ~(int64_t)15;
        for (int64_t blk = base; blk < t2; blk += SCAN_TILE) {
            const int64_t lp = blk + lane * 16;
            uint32_t W[5];
            if (lp < t2) {
                const uint4 v = *(const uint4 *)(arena + lp);
                W[0] = v.x; W[1] = v.y; W[2] = v.z; W[3] = v.w;
            } else {
                W[0] = W[1] = W[2] = W[3] = 0;
            }
            W[4] = (uint32_t)__shfl_down((int)W[0], 1, WAVE);
            if (lane == WAVE - 1) {
                const int64_t q = blk + SCAN_TILE;
                W[4] = (q < t2) ? *(const uint32_t *)(arena + q) : 0u;
            }
            uint32_t cmask = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int64_t pos = lp + j;
                const uint32_t win = __builtin_amdgcn_alignbyte(W[(j >> 2) + 1], W[j >> 2], j & 3);
                const uint32_t byte = win & 0xFFu;
                const bool in = pos >= t0 && pos < t2;
                const bool intext = pos < t1;
                const bool lead = in && ((byte & 0xC0u) != 0x80u);
                cpt += (lead && intext);
                cpu += (lead && !intext);
                if (in && byte >= 0x80u) {
                    if (intext) na0 = true;
                    else na1 = true;
                }
                const int64_t fe = intext ? t1 : t2;
                const uint32_t h = ((win & 0xFFFFFFu) * HASH_MUL) >> (32 - FILT_BITS);
                const bool hit = in && (pos + 2 <= fe) && ((filt[h >> 5] >> (h & 31)) & 1u);
                cmask |= (uint32_t)hit << j;
            }
            int total;
            int k = wave_excl_scan(__popc(cmask), &total);
            if (total == 0) continue;
            ncand += (lane == 0) ? (unsigned long long)total : 0ull;
            while (cmask) {
                const int j = __ffs(cmask) - 1;
                cmask &= cmask - 1;
                cand[k++] = (uint32_t)(lp + j - t0);
            }
            wave_sync();
            for (int i0 = 0; i0 < total; i0 += WAVE) {
                const int i = i0 + lane;
                if (KW_STAGE >= 1 && i < total) process_candidate(T, S, arena, t0, t1, t2, cand[i], items0, items1, icnt, nanchor);
            }
            wave_sync();
        }
        wave_sync_global();
        uint32_t N0 = icnt[0], N1 = icnt[1];
        if (N0 > S.item_cap) N0 = S.item_cap;
        if (N1 > S.item_cap) N1 = S.item_cap;
        N0 = __builtin_amdgcn_readfirstlane(N0);
        N1 = __builtin_amdgcn_readfirstlane(N1);
        const uint32_t ncp0 = (uint32_t)wave_sum((int)cpt), ncp1 = (uint32_t)wave_sum((int)cpu);
        const bool ascii0 = __ballot(na0) == 0, ascii1 = __ballot(na1) == 0;
        for (int f = 0; f < 2; ++f) {
            FieldCtx F;
            F.arena = arena;
            F.fb = f ? t1 : t0;
            F.fe = f ? t2 : t1;
            F.n = f ? ncp1 : ncp0;
            F.ascii = f ? ascii1 : ascii0;
            F.cps = cps;
            F.blkcnt = blkcnt;
            F.doc = (uint32_t)d;
            F.field = (uint32_t)f;
            const uint32_t N = f ? N1 : N0;
            if (N == 0 && F.n > (uint32_t)MAXM) continue;
            if (!F.ascii) decode_field(S, arena, F.fb, F.fe, cps, blkcnt);
            if (KW_STAGE >= 2) resolve_field(T, S, F, O, f ? items1 : items0, N, lpm, lext_cp, lext_mask, nwin);
        }
    }
    if (lane == 0) {
        S.out_cnt[wave] = O.n;
        atomicAdd(&S.stats[0], ncand);
    }
    // per-lane counters
    unsigned long long a = nanchor, w = nwin;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) {
        a += __shfl_xor(a, dd, WAVE);
        w += __shfl_xor(w, dd, WAVE);
    }
    if (lane == 0) {
        atomicAdd(&S.stats[1], a);
        atomicAdd(&S.stats[2], w);
    }
}

constexpr size_t kScanLds = (size_t)FILT_WORDS * 4 + (size_t)WAVES_PER_BLOCK * (128 * 8 + 64 * 8 + CAND_CAP * 4 + 64 * 4 + 2 * 4);

// exclusive scan of the per-wave record counts (one block)
__global__ void kw_offsets_kernel(const uint32_t *__restrict__ cnt, int n_waves, uint32_t cap,
                                  unsigned long long *__restrict__ offs, unsigned long long *__restrict__ total)
{
    __shared__ unsigned long long part[2][1024];
    const int t = threadIdx.x;
    const int per = (n_waves + 1023) / 1024;
    const int i0 = t * per, i1 = min((t + 1) * per, n_waves);
    unsigned long long s = 0;
    // a thread's segment 8 loads at a time, in flight together (one load per iteration waited a round trip each)
    for (int i = i0; i < i1; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i + k < i1 ? cnt[i + k] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k] < cap ? v[k] : cap;
    }
    // inclusive block scan (Hillis-Steele over the 1024 partial sums, double-buffered)
    int b = 0;
    part[0][t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const unsigned long long v = part[b][t] + (t >= d ? part[b][t - d] : 0ull);
        b ^= 1;
        part[b][t] = v;
        __syncthreads();
    }
    unsigned long long acc = part[b][t] - s;      // exclusive
    if (t == 1023) {
        offs[n_waves] = part[b][t];
        *total = part[b][t];
    }
    for (int i = i0; i < i1; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i + k < i1 ? cnt[i + k] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i + k < i1) {
                offs[i + k] = acc;
                acc += v[k] < cap ? v[k] : cap;
            }
    }
}

__global__ void kw_gather_kernel(const kw_hit *__restrict__ src, uint32_t cap, const uint32_t *__restrict__ cnt,
                                 const unsigned long long *__restrict__ offs, kw_hit *__restrict__ dst)
{
    const int w = blockIdx.x;
    const uint32_t n = cnt[w] < cap ? cnt[w] : cap;
    const kw_hit *s = src + (size_t)w * cap;
    kw_hit *d = dst + offs[w];
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

}  // namespace kw
