// Fast path kernels (see kwmatch_fast.hpp).  Included after kwmatch_kernels.hpp
// (shares its wave/text helpers).
//
//   (the byte scan -- filter, anchor probe, all-ASCII epilogue -- is kwmatch_split.hpp)
//   kw_resolve_kernel  one wave per document with work: sort the items of a
//                      field, decide fuzzy names (exact / edge / LCS-verified
//                      pieces), report re.finditer positions
//
// Rare documents (more than FK_ITEMS0 / FK_ITEMS1 items in the text / title, one name with more than
// 64 items in a field, non-ASCII fields longer
// than FK_CP_CAP bytes) are handed to the generic kernel (kw_scan_kernel).
#pragma once
#include "kwmatch_fast.hpp"
#include "kwmatch_kernels.hpp"

#ifndef EPI_SHORT_PREF   // the group epilogue's signature test of short fields before their tasks
#define EPI_SHORT_PREF 1
#endif
#ifndef SHORT_TB   // short kernel: every name on lanes (one-byte code points, 256-entry match vectors)
#define SHORT_TB 1
#endif
#ifndef SHORT_BG   // short kernel: the bigram-signature filter after the character signature
#define SHORT_BG 1
#endif
#ifndef VK_U   // verify jobs: name match-vector loads in flight
#define VK_U 8
#endif
// task kernels' minimum waves per SIMD (register budget: 4 -> 128 VGPRs, 5 -> 102, 6 -> 84, 8 -> 64)
#ifndef VK_PRETEST
#define VK_PRETEST 1   // the verify kernel's band-test pretest with a queue of the tasks it cannot rule out
#endif
#ifndef VK_MINW
#define VK_MINW 4
#endif
#ifndef SK_MINW
#define SK_MINW 1
#endif
#ifndef RX_MINW
#define RX_MINW 4   // <= 128 VGPRs (the prefetched task records stay in LDS)
#endif
#ifndef SHORT_COUNT
#define SHORT_COUNT 0
#endif
// waves per SIMD the resolve kernel is compiled for (register budget)
#ifndef FK_TIMING   // developer aid: per-phase cycle counters of the resolve kernel (KW_DUMP_TIMING)
#define FK_TIMING 0
#endif
#define FK_T0(v) const unsigned long long v = FK_TIMING ? __builtin_amdgcn_s_memtime() : 0ull
#define FK_TACC(acc, v) do { if (FK_TIMING) acc += __builtin_amdgcn_s_memtime() - (v); } while (0)
#ifndef EK_TIMING   // developer aid: per-phase cycle counters of the epilogue kernel (KW_DUMP_TIMING, stats 21..31)
#define EK_TIMING 0
#endif
#define EK_T0(v) const unsigned long long v = EK_TIMING ? __builtin_amdgcn_s_memtime() : 0ull
#define EK_TACC(acc, v) do { if (EK_TIMING) (acc) += __builtin_amdgcn_s_memtime() - (v); } while (0)



#ifndef FK_EPI_EDGE   // developer aid: 3 = edge windows in the epilogue; 1 = code present, never run; 0 = absent
#define FK_EPI_EDGE 3
#endif

#ifndef FK_SHORT_LANES   // 1: lane-parallel short-field windows in the short task kernel; 0: wave-serial
#define FK_SHORT_LANES 1
#endif

#ifndef RK_OCC
#define RK_OCC 4
#endif

namespace kw {

// ---------------------------------------------------------------- per-doc state
struct FastDoc {
    const uint8_t *arena;
    int64_t t0, t1, t2;
    int32_t l1, l2;   // t1 - t0, t2 - t0: field ends relative to the document
    uint32_t doc;
};

__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t *__restrict__ a, int64_t p)
{
    const int64_t a0 = p & ~(int64_t)3;
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t x0 = *(const uint32_t *)(a + a0);
    const uint32_t x1 = *(const uint32_t *)(a + a0 + 4);
    return __builtin_amdgcn_alignbyte(x1, x0, s);
}

// the 8 bytes at any byte position (three aligned words)
__device__ __forceinline__ uint64_t ld_u64_unaligned(const uint8_t *__restrict__ a, int64_t p)
{
    const int64_t a0 = p & ~(int64_t)3;
    const uint32_t s = (uint32_t)(p & 3);
    const uint32_t x0 = *(const uint32_t *)(a + a0);
    const uint32_t x1 = *(const uint32_t *)(a + a0 + 4);
    const uint32_t x2 = *(const uint32_t *)(a + a0 + 8);
    return (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, s) << 32);
}

// a 64-bit value of lane l, l varying per lane
__device__ __forceinline__ int64_t rdlane64v(int64_t v, int l)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, l, WAVE);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)v >> 32), l, WAVE);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// a 64-bit value of lane l (wave-uniform result)
__device__ __forceinline__ int64_t rdlane64(int64_t v, int l)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ bool lds_bit(const uint32_t *t, uint32_t idx) { return __builtin_amdgcn_ubfe(t[idx >> 5], idx, 1) != 0u; }

// byte-exact compare of text[p, p+len) with pat[0, len)
__device__ __forceinline__ bool span_equal(const uint8_t *__restrict__ a, int64_t p, const uint8_t *__restrict__ pat,
                                           uint32_t len)
{
    uint32_t i = 0;
    for (; i + 4 <= len; i += 4) {
        const uint32_t t = ld_u32_unaligned(a, p + i);
        const uint32_t q = (uint32_t)pat[i] | ((uint32_t)pat[i + 1] << 8) | ((uint32_t)pat[i + 2] << 16) |
                           ((uint32_t)pat[i + 3] << 24);
        if (t != q) return false;
    }
    for (; i < len; ++i)
        if (a[p + i] != pat[i]) return false;
    return true;
}

// ---------------------------------------------------------------- field helpers
// code points of a field: ASCII fields are their byte length; others are counted
__device__ uint32_t field_cp_count(const uint8_t *__restrict__ arena, int64_t fb, int64_t fe, bool ascii)
{
    const int64_t L = fe - fb;
    if (ascii) return (uint32_t)L;
    const int lane = lane_id();
    uint32_t cnt = 0;
    for (int64_t b0 = 0; b0 < L; b0 += WAVE) {
        const int64_t i = b0 + lane;
        const bool lead = i < L && ((arena[fb + i] & 0xC0) != 0x80);
        cnt += (uint32_t)__popcll(__ballot(lead));
    }
    return cnt;
}

__device__ bool field_is_ascii(const uint8_t *__restrict__ arena, int64_t fb, int64_t fe)
{
    const int lane = lane_id();
    bool hi = false;
    for (int64_t i = fb + lane; i < fe; i += WAVE) hi |= arena[i] >= 0x80;
    return __ballot(hi) == 0;
}

// Decode a non-ASCII field into code points, 16 bytes per lane per step (coalesced), with the
// cumulative lead-byte count at every 64-byte block of the arena from base = fb & ~15 (blkcnt[k] =
// code points of the field before base + 64 k).  Returns the field's code points.
__device__ uint32_t decode_field_fast(const uint8_t *__restrict__ a, int64_t fb, int64_t fe, uint32_t *cps,
                                      uint32_t *blkcnt, uint32_t cap)
{
    const int lane = lane_id();
    const int64_t base = fb & ~(int64_t)15;
    uint32_t count = 0;
    for (int64_t blk = base; blk < fe; blk += 1024) {
        const int64_t lp = blk + 16 * (int64_t)lane;
        uint32_t W[5];
        if (lp < fe) {
            const uint4 v = *(const uint4 *)(a + lp);
            W[0] = v.x; W[1] = v.y; W[2] = v.z; W[3] = v.w;
        } else {
            W[0] = W[1] = W[2] = W[3] = 0;
        }
        W[4] = (uint32_t)__shfl_down((int)W[0], 1, WAVE);
        if (lane == WAVE - 1) W[4] = (blk + 1024 < fe) ? *(const uint32_t *)(a + blk + 1024) : 0u;
        const int64_t r0 = fb - lp, r2 = fe - lp;
        const int jlo = r0 <= 0 ? 0 : (r0 >= 16 ? 16 : (int)r0);
        const int jhi = r2 <= 0 ? 0 : (r2 >= 16 ? 16 : (int)r2);
        const uint32_t valid = (jhi > jlo) ? (((1u << jhi) - 1u) & ~((1u << jlo) - 1u)) : 0u;
        uint32_t lead = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t b = (W[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            lead |= (uint32_t)((b & 0xC0u) != 0x80u) << j;
        }
        lead &= valid;
        int total;
        const int ex = wave_excl_scan(__popc(lead), &total);
        if ((lane & 3) == 0) blkcnt[(lp - base) >> 6] = count + (uint32_t)ex;
        uint32_t idx = count + (uint32_t)ex;
        uint32_t lm = lead;
        while (lm) {
            const int j = __ffs(lm) - 1;
            lm &= lm - 1;
            // bytes j.. of this chunk, continuing into the next lane's first word
            const uint32_t b0 = (W[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            uint32_t c = b0;
            if (b0 >= 0x80u) {
                const uint32_t n = (b0 >= 0xF0u) ? 4u : (b0 >= 0xE0u) ? 3u : 2u;
                c = b0 & (0x7Fu >> n);
                for (uint32_t k = 1; k < n; ++k) {
                    const int jj = j + (int)k;
                    const uint32_t bk = (lp + jj < fe) ? ((W[jj >> 2] >> (8 * (jj & 3))) & 0xFFu) : 0x80u;
                    c = (c << 6) | (bk & 0x3Fu);
                }
            }
            if (idx < cap) cps[idx] = c;
            ++idx;
        }
        count += (uint32_t)total;
    }
    wave_sync_global();
    return count;
}

// code point offset of field byte bpos (non-ASCII fields decoded by decode_field_fast)
__device__ __forceinline__ uint32_t to_cp_fast(const FieldCtx &F, uint32_t bpos)
{
    if (F.ascii) return bpos;
    const int64_t base = F.fb & ~(int64_t)15, p = F.fb + bpos;
    const int64_t b64 = (p - base) & ~(int64_t)63;
    uint32_t c = F.blkcnt[b64 >> 6];
    // leads in [max(base + b64, fb), p)
    for (int64_t q = base + b64; q < p; q += 4) {
        const uint32_t w = *(const uint32_t *)(F.arena + q);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t y = q + k;
            if (y >= F.fb && y < p) c += (((w >> (8 * k)) & 0xC0u) != 0x80u);
        }
    }
    return c;
}

// text code point i of the field (ASCII: byte; else decoded scratch)
__device__ __forceinline__ uint32_t fk_cp(const FieldCtx &F, int64_t i)
{
    if (i < 0 || i >= (int64_t)F.n) return 0xFFFFFFFFu;
    return F.ascii ? (uint32_t)F.arena[F.fb + i] : F.cps[i];
}

// ---------------------------------------------------------------- wave-cooperative LCS (ballot)
// V-update with needle bit-vector from a ballot over lanes holding the needle
__device__ __forceinline__ uint64_t lcs_ballot_step(uint64_t V, uint32_t lanechar, uint32_t c, uint64_t needle_mask)
{
    const uint64_t M = __ballot(lanechar == c) & needle_mask;
    const uint64_t U = V & M;
    return (V + U) | (V - U);
}

// Text code points [lo, lo + 128) of a field staged one per lane in two
// registers (out-of-range positions read as 0xFFFFFFFF, which no name holds).
__device__ __forceinline__ void fk_stage_text(const FieldCtx &F, int64_t lo, uint32_t &ta, uint32_t &tb)
{
    const int lane = lane_id();
    ta = fk_cp(F, lo + lane);
    tb = fk_cp(F, lo + 64 + lane);
}

// staged code point at a wave-uniform index (0..127)
__device__ __forceinline__ uint32_t fk_staged_u(uint32_t ta, uint32_t tb, int idx)
{
    return idx < 64 ? __builtin_amdgcn_readlane(ta, idx) : __builtin_amdgcn_readlane(tb, idx - 64);
}

// staged code point at a per-lane index (0..127); every lane must execute it
__device__ __forceinline__ uint32_t fk_staged_v(uint32_t ta, uint32_t tb, int idx)
{
    const uint32_t a = (uint32_t)__shfl((int)ta, idx & 63, WAVE);
    const uint32_t b = (uint32_t)__shfl((int)tb, idx & 63, WAVE);
    return idx < 64 ? a : b;
}

// Verify one PIECE item of pattern P (needle = name, m < n).  All lanes call.
// nm: lane i holds name[i] (i < m).  base = q - o is the text code point the
// name's first code point aligns with.  Returns true if some window of the
// partial_ratio family containing the piece passes.
__device__ bool fk_verify_piece(const FieldCtx &F, uint32_t nm, uint32_t m, uint32_t q, uint32_t o, uint32_t pl,
                                unsigned long long &nwin)
{
    const int lane = lane_id();
    const uint32_t n = F.n;
    const uint64_t needle = low_mask(m);
    const uint32_t k = kfull(m);
    if (k > 0) {
        // band test: every name char matched by a passing full window lies within +-2k of base+i.
        // The text [base-2k, base+m+2k) (<= 76 code points) is staged in registers.
        const int64_t base = (int64_t)q - (int64_t)o;
        const int64_t lo = base - 2 * (int64_t)k;
        uint32_t ta, tb;
        fk_stage_text(F, lo, ta, tb);
        bool hit = false;
        for (int t = 0; t <= 4 * (int)k; ++t) {
            const uint32_t c = fk_staged_v(ta, tb, lane + t);
            hit |= (lane < (int)m) && c == nm;
        }
        const uint32_t cnt = (uint32_t)__popcll(__ballot(hit));
        if (cnt + k >= m) {
            int64_t pmin = base - k, pmax = base + k;
            if (pmin < 0) pmin = 0;
            if (pmax > (int64_t)(n - m)) pmax = (int64_t)(n - m);
            for (int64_t p = pmin; p <= pmax; ++p) {
                const int i0 = (int)(p - lo);
                uint64_t V = ~0ull;
                for (uint32_t j = 0; j < m; ++j) V = lcs_ballot_step(V, nm, fk_staged_u(ta, tb, i0 + (int)j), needle);
                ++nwin;
                const uint32_t L = (uint32_t)__popcll(~V & needle);
                if (20u * (m - L) < m) return true;
            }
        }
    }
    if (q + pl + 1 <= m) {   // prefixes text[:w], w in [1, m)
        const uint32_t tc = (lane < (int)m) ? fk_cp(F, lane) : 0xFFFFFFFEu;
        uint64_t V = ~0ull;
        ++nwin;
        for (uint32_t w = 1; w < m; ++w) {
            V = lcs_ballot_step(V, nm, __builtin_amdgcn_readlane(tc, w - 1), needle);
            if (passes((uint32_t)__popcll(~V & needle), m, w)) return true;
        }
    }
    if (q + m > n) {         // suffixes text[i:], i in (n-m, n): reversed needle and text
        const uint32_t nr = __shfl(nm, (int)m - 1 - lane, WAVE);
        const uint32_t tc = (lane < (int)m) ? fk_cp(F, (int64_t)n - 1 - lane) : 0xFFFFFFFEu;
        uint64_t V = ~0ull;
        ++nwin;
        for (uint32_t kk = 1; kk < m; ++kk) {
            V = lcs_ballot_step(V, nr, __builtin_amdgcn_readlane(tc, kk - 1), needle);
            if (passes((uint32_t)__popcll(~V & needle), m, kk)) return true;
        }
    }
    return false;
}

// Short field (n <= 64 code points) vs a longer-or-equal name: needle = field.
// fc: lane i holds field[i] (i < n); nmr: lane i holds name[i] (i < m, m >= n).
__device__ bool fk_short_decide(uint32_t fc, uint32_t n, uint32_t nmr, uint32_t m, bool *exact,
                                unsigned long long &nwin)
{
    *exact = false;
    const int lane = lane_id();
    const uint64_t needle = low_mask(n);
    uint64_t Vf = ~0ull;
    for (uint32_t p = 0; p + n <= m; ++p) {        // full windows of the name
        uint64_t V = ~0ull;
        for (uint32_t j = 0; j < n; ++j) V = lcs_ballot_step(V, fc, __builtin_amdgcn_readlane(nmr, p + j), needle);
        ++nwin;
        if (p == 0) Vf = V;
        const uint32_t L = (uint32_t)__popcll(~V & needle);
        if (L == n && m == n) *exact = true;
        if (20u * (n - L) < n) return true;
    }
    {   // prefixes of the name
        uint64_t V = ~0ull;
        for (uint32_t i = 1; i < n; ++i) {
            V = lcs_ballot_step(V, fc, __builtin_amdgcn_readlane(nmr, i - 1), needle);
            if (passes((uint32_t)__popcll(~V & needle), n, i)) return true;
        }
    }
    const uint32_t fr = __shfl(fc, (int)n - 1 - lane, WAVE);
    uint64_t Vr = ~0ull;
    {   // suffixes of the name (reversed needle)
        uint64_t V = ~0ull;
        for (uint32_t kk = 1; kk < n; ++kk) {
            V = lcs_ballot_step(V, fr, __builtin_amdgcn_readlane(nmr, m - kk), needle);
            if (passes((uint32_t)__popcll(~V & needle), n, kk)) return true;
        }
    }
    if (m == n) {   // swapped run: needle = name, windows = prefixes / suffixes of the field
        for (uint32_t j = 0; j < m; ++j) Vr = lcs_ballot_step(Vr, fr, __builtin_amdgcn_readlane(nmr, m - 1 - j), needle);
        for (uint32_t i = 1; i < n; ++i) {
            if (passes((uint32_t)__popcll(~Vf & low_mask(i)), m, i)) return true;
            if (passes((uint32_t)__popcll(~Vr & low_mask(n - i)), m, n - i)) return true;
        }
    }
    (void)lane;
    return false;
}


// ---------------------------------------------------------------- edge windows (11 <= m <= 20)
// A fuzzy name with 11 <= m <= 20 and m < n passes partial_ratio on an edge
// window iff the first or the last m-1 code points of the field equal the
// name with one code point deleted (20*1 < 2m-1; every other window of such a
// name needs an exact occurrence, which the FULL use finds).  Lanes 0..19 take
// (side, L = m-1): hash the window, look it up among the one-deletion variants,
// verify exactly and append an EDGE item.  Returns the number of items added.
#ifndef RK_EDGE_NOINLINE   // 1: fk_edge_items as a called function (its registers stay out of the resolve loop)
#define RK_EDGE_NOINLINE 0
#endif
template <uint32_t ICAP>
#if RK_EDGE_NOINLINE
__device__ __attribute__((noinline))
#else
__device__
#endif
uint32_t fk_edge_items(const FastTables &FT, const FieldCtx &F, uint64_t *items, uint32_t *icnt_f,
                                  uint32_t *dflag)
{
    const int lane = lane_id();
    const uint32_t L = (EDGE_MIN_M - 1) + (uint32_t)(lane % 10);
    const bool act = lane < 20 && L + 2 <= F.n;
    const uint8_t *__restrict__ a = F.arena;
    uint64_t hh = 0;
    int64_t b0 = F.fb;
    if (F.ascii) {
        // bytes are code points: the wave holds the first and the last 20 bytes
        const int64_t flen = F.fe - F.fb;
        const int t20 = flen < 20 ? (int)flen : 20;
        const uint32_t head = (lane < t20) ? a[F.fb + lane] : 0u;
        const uint32_t tail = (lane < t20) ? a[F.fe - t20 + lane] : 0u;
        if (lane >= 10) b0 = F.fe - (int64_t)L;
        const int tbase = t20 - (int)L;   // suffix window = tail[t20-L, t20)
#pragma unroll
        for (int j = 0; j < (int)EDGE_MAX_M - 1; ++j) {
            const uint32_t ch = (uint32_t)__shfl((int)head, j, WAVE);
            const uint32_t ct = (uint32_t)__shfl((int)tail, (tbase + j) & 63, WAVE);
            const uint32_t c = lane >= 10 ? ct : ch;
            if ((uint32_t)j < L) hh = hh * SUB_B + c;
        }
    } else {
        // decoded field: the wave holds the first and the last 20 code points
        const int t20 = F.n < 20u ? (int)F.n : 20;
        const uint32_t head = (lane < t20) ? F.cps[lane] : 0u;
        const uint32_t tail = (lane < t20) ? F.cps[F.n - t20 + lane] : 0u;
        b0 = lane >= 10 ? (int64_t)F.n - (int64_t)L : 0;   // window start, in code points
        const int tbase = t20 - (int)L;
#pragma unroll
        for (int j = 0; j < (int)EDGE_MAX_M - 1; ++j) {
            const uint32_t ch = (uint32_t)__shfl((int)head, j, WAVE);
            const uint32_t ct = (uint32_t)__shfl((int)tail, (tbase + j) & 63, WAVE);
            const uint32_t c = lane >= 10 ? ct : ch;
            if ((uint32_t)j < L) hh = hh * SUB_B + c;
        }
    }
    uint32_t added = 0;
    if (act) {
        const uint64_t key = (hh + (uint64_t)L * 0x9E3779B97F4A7C15ull) | 1ull;
        uint32_t slot = (uint32_t)(key >> 32) & FT.edge_mask;
        uint32_t eb = 0, ec = 0;
        for (;;) {
            const uint64_t kk = FT.edge_key[slot];
            if (kk == key) { eb = FT.edge_begin[slot]; ec = FT.edge_cnt[slot]; break; }
            if (kk == 0) break;
            slot = (slot + 1) & FT.edge_mask;
        }
        for (uint32_t e = 0; e < ec; ++e) {
            const uint32_t ent = FT.edge_ent[eb + e];
            const uint32_t P = ent >> 5, del = ent & 31u;
            if (pi_m(FT.pat_info[P]) != L + 1) continue;
            const uint32_t *nm = FT.pat_cps + FT.pat_cp_off[P];
            bool eq = true;
            for (uint32_t j = 0; j < L && eq; ++j) {
                const uint32_t c = F.ascii ? (uint32_t)a[b0 + j] : F.cps[b0 + j];
                eq = c == nm[j < del ? j : j + 1];
            }
            if (!eq) continue;
            const uint32_t idx = atomicAdd(icnt_f, 1u);
            if (idx < ICAP)
                items[idx] = ((uint64_t)P << IT_PAT_SHIFT) | ((uint64_t)FU_EDGE << IT_KIND_SHIFT) | (uint64_t)IT_USE_MASK;
            else
                atomicOr(dflag, 1u);
            ++added;
        }
    }
    return added;
}

// re.finditer positions of a quantifier-free regex name (literals and '.'):
// shift-and over the field, lane l owning the 32 start positions
// [r0 + 32 l, r0 + 32 l + 32) of each 2048-position round.  tab = this wave's
// LDS copy of the row's 128 ASCII masks; txt = this wave's LDS staging buffer
// (RX_TXT bytes) for the round's text of an ASCII field.  Leftmost
// non-overlapping selection (every match is L code points long).  Returns the
// number of positions emitted.
constexpr int RX_TXT = 2048 + 64 + 16 + 16;   // 2048 starts + L - 1 <= 63 tail bytes + alignment slack

// TAB256 (tab holds 256 entries): a transcoded field's marker bytes get their masks in tab[128, 256) first, so
// its bytes take the unrolled loop like an ASCII field's (one LDS lookup per byte, no per-byte branch)
struct RxfParams {   // a fixed program's length, any-code-point mask and extended code point range
    uint32_t L, eb, ee;
    uint64_t anym;
};
__device__ __forceinline__ RxfParams rxf_params(const FastTables &FT, uint32_t r)
{
    RxfParams p;
    p.L = FT.rxf_len[r];
    p.anym = FT.rxf_any[r];
    p.eb = FT.rxf_ext_off[r];
    p.ee = FT.rxf_ext_off[r + 1];
    return p;
}

template <bool TAB256 = false>
__device__ uint32_t fk_rx_fixed_positions(const FastTables &FT, const DevScratch &GS, const FieldCtx &F, OutCtx &O,
                                          uint32_t P, uint32_t r, const RxfParams &prm, uint64_t *tab, uint8_t *txt)
{
    const int lane = lane_id();
    const uint32_t L = prm.L;
    const uint64_t anym = prm.anym;
    const uint32_t eb = prm.eb, ee = prm.ee;
    wave_sync();
    tab[lane] = FT.rxf_pm[(size_t)r * 128 + lane];
    tab[lane + 64] = FT.rxf_pm[(size_t)r * 128 + 64 + lane];
    const bool fast_tx = TAB256 && F.ascii && F.tx;
    if (fast_tx) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t b = 128u + (uint32_t)lane + 64u * (uint32_t)h;
            const uint32_t c = FT.tx_inv[b & 0x7Fu];
            uint64_t B = anym;
            for (uint32_t e = eb; e < ee; ++e)
                if (FT.rxf_ext_cp[e] == c) B |= FT.rxf_ext_mask[e];
            tab[b] = B;
        }
    }
    wave_sync();
    const int64_t n = F.n;
    if (n < (int64_t)L) return 0;
#if defined(RX_TIMING_SKIP) && RX_TIMING_SKIP == 4
    return 0;
#endif
    // the program's literal head: each of its first min(4, L) positions whose matching bytes are exactly one
    // ASCII byte c (hv byte i = c, hm byte i = 0xFF).  With two or more such bytes a lane tests its 32 starts'
    // 4-byte windows against the head (SWAR, no per-byte lookup chain) and confirms only the candidates
    // position by position against the masks
    uint32_t hv = 0, hm = 0;
    if (F.ascii && (!F.tx || fast_tx)) {
        const uint64_t m0 = tab[lane], m1 = tab[lane + 64];
        const uint64_t mx = fast_tx ? (tab[128 + lane] | tab[192 + lane]) : 0ull;
        for (uint32_t i = 0; i < 4u && i < L; ++i) {
            const uint64_t b0 = __ballot((m0 >> i) & 1ull), b1 = __ballot((m1 >> i) & 1ull);
            const uint64_t bx = __ballot((mx >> i) & 1ull);
            if (!bx && __popcll(b0) + __popcll(b1) == 1) {
                const uint32_t c = b0 ? (uint32_t)__builtin_ctzll(b0) : 64u + (uint32_t)__builtin_ctzll(b1);
                hv |= c << (8 * i);
                hm |= 0xFFu << (8 * i);
            }
        }
    }
    const bool use_head = __popc(hm) >= 16;
    const int64_t nstarts = n - L + 1;
    const uint64_t fin = 1ull << (L - 1);
    uint32_t last_end = 0, emitted = 0;
    for (int64_t r0 = 0; r0 < nstarts; r0 += 64 * 32) {
        int64_t tb = 0;   // txt[k] = field byte tb + k
        if (F.ascii) {
            // stage field bytes [r0, r0 + 2048 + L - 1) with coalesced 16-byte loads (the arena is padded)
            const int64_t a0 = (F.fb + r0) & ~(int64_t)15;
            const int64_t a1 = F.fb + r0 + 2048 + L - 1 < F.fe ? F.fb + r0 + 2048 + L - 1 : F.fe;
            tb = a0 - F.fb;
            wave_sync();
            for (int c = lane; c < RX_TXT / 16; c += WAVE) {
                const int64_t a = a0 + 16 * (int64_t)c;
                if (a < a1) ((uint4 *)txt)[c] = *(const uint4 *)(F.arena + a);
            }
            wave_sync();
        } else {
            // code points [r0, r0 + 2048 + L - 1) as bytes: ASCII as is, the rest as the marker 0x80
            tb = r0;
            const int64_t a1 = r0 + 2048 + L - 1 < n ? r0 + 2048 + L - 1 : n;
            wave_sync();
            for (int c = lane; c < RX_TXT / 16; c += WAVE) {
                const int64_t i0 = r0 + 16 * (int64_t)c;
                uint32_t wv[4] = {0u, 0u, 0u, 0u};
                if (i0 < a1) {
#pragma unroll
                    for (int k4 = 0; k4 < 4; ++k4) {
                        const uint4 v = *(const uint4 *)(F.cps + i0 + 4 * k4);   // the buffer holds FK_CP_CAP code points
                        const uint32_t cc[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                        for (int k = 0; k < 4; ++k) wv[k4] |= (cc[k] < 128u ? cc[k] : 0x80u) << (8 * k);
                    }
                }
                ((uint4 *)txt)[c] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
            }
            wave_sync();
        }
        const int64_t s_lo = r0 + (int64_t)lane * 32;
        uint32_t mask = 0;
#if defined(RX_TIMING_SKIP) && RX_TIMING_SKIP == 3
        if (false) {
#else
        if (s_lo < nstarts) {
#endif
            const int64_t s_hi = s_lo + 32 < nstarts ? s_lo + 32 : nstarts;
            const int c_cnt = (int)(s_hi + L - 1 - s_lo);
            uint64_t D = 0;
            const uint8_t *t = txt + (s_lo - tb);
            if (use_head) {
                const uint32_t o = (uint32_t)(s_lo - tb), sh = o & 3u;
                const uint32_t *tw = (const uint32_t *)txt + (o >> 2);
                uint32_t wd[10];
#pragma unroll
                for (int q = 0; q < 10; ++q) wd[q] = tw[q];
                // windows at every byte b < 36 of the lane's dwords (constant shifts), then the lane's starts
                uint64_t cmb = 0;
#pragma unroll
                for (int q = 0; q < 9; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const uint32_t win = r ? __builtin_amdgcn_alignbyte(wd[q + 1], wd[q], r) : wd[q];
                        cmb |= (uint64_t)(((win ^ hv) & hm) == 0u ? 1u : 0u) << (4 * q + r);
                    }
                uint32_t cm = (uint32_t)(cmb >> sh);
                const int ns = (int)(s_hi - s_lo);
                if (ns < 32) cm &= (1u << ns) - 1u;
                const uint32_t bm = fast_tx ? 0xFFu : 0x7Fu;
                while (cm) {
                    const int j = __builtin_ctz(cm);
                    cm &= cm - 1u;
                    bool ok = true;
                    for (uint32_t i = 0; i < L && ok; ++i) ok = ((tab[t[j + (int)i] & bm] >> i) & 1ull) != 0;
                    if (ok) mask |= 1u << j;
                }
            } else if (F.ascii && !F.tx) {
#pragma unroll 8
                for (int k = 0; k < c_cnt; ++k) {
                    D = ((D << 1) | 1ull) & tab[t[k] & 0x7Fu];
                    if (D & fin) mask |= 1u << (uint32_t)(k - (int)(L - 1));
                }
            } else if (fast_tx) {
#pragma unroll 8
                for (int k = 0; k < c_cnt; ++k) {
                    D = ((D << 1) | 1ull) & tab[t[k]];
                    if (D & fin) mask |= 1u << (uint32_t)(k - (int)(L - 1));
                }
            } else {
                for (int k = 0; k < c_cnt; ++k) {
                    const uint32_t b = t[k];
                    uint64_t B;
                    if (b < 128) {
                        B = tab[b];
                    } else {   // (transcoded view: the marker's code point; 0x80 is none of the names')
                        const uint32_t c = F.tx ? FT.tx_inv[b & 0x7Fu] : F.cps[s_lo + k];
                        B = anym;
                        for (uint32_t e = eb; e < ee; ++e)
                            if (FT.rxf_ext_cp[e] == c) B |= FT.rxf_ext_mask[e];
                    }
                    D = ((D << 1) | 1ull) & B;
                    if (D & fin) mask |= 1u << (uint32_t)(k - (int)(L - 1));
                }
            }
        }
        // greedy selection in position order (lanes in order, bits in order)
        uint64_t lanes = __ballot(mask != 0);
        uint32_t keep = 0;
        while (lanes) {
            const int l = __builtin_ctzll(lanes);
            lanes &= lanes - 1;
            uint32_t mk = (uint32_t)__builtin_amdgcn_readlane((int)mask, l), kp = 0;
            while (mk) {
                const int b = __builtin_ctz(mk);
                mk &= mk - 1;
                const uint32_t st = (uint32_t)(r0 + (int64_t)l * 32 + b);
                if (st >= last_end) { kp |= 1u << b; last_end = st + L; }
            }
            if (lane == l) keep = kp;
        }
        while (__ballot(keep != 0)) {
            const int b = keep ? __builtin_ctz(keep) : 0;
            emit_hits(O, GS, keep != 0, F.doc, P, (uint32_t)(s_lo + b), F.field);
            emitted += (uint32_t)__popcll(__ballot(keep != 0));
            keep &= keep - 1;
        }
    }
    return emitted;
}

// sort the n <= 64 keys held by lanes [0, n) (the other lanes hold ~0): few keys by rank and an
// LDS scatter into buf (n slots, this wave's), more by the register bitonic network
__device__ __forceinline__ uint64_t wave_sort_few(uint64_t x, uint32_t n, uint64_t *buf)
{
    if (n > 24) return wave_sort_reg(x);
    const int lane = lane_id();
    uint32_t r = 0;
    for (uint32_t j = 0; j < n; ++j) {
        const uint64_t y = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), j) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, j);
        r += (y < x || (y == x && (int)j < lane)) ? 1u : 0u;
    }
    wave_sync();
    if (lane < (int)n) buf[r] = x;
    wave_sync();
    return lane < (int)n ? buf[lane] : ~0ull;
}

// wave_sort_reg with a 32-bit payload per key
__device__ __forceinline__ uint64_t wave_sort_reg_kv(uint64_t x, uint32_t &v)
{
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= WAVE; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t y = __shfl_xor(x, j, WAVE);
            const uint32_t w = (uint32_t)__shfl_xor((int)v, j, WAVE);
            const bool take_min = ((lane & j) == 0) == ((lane & k) == 0);
            const bool take_y = take_min ? y < x : x < y;
            x = take_y ? y : x;
            v = take_y ? w : v;
        }
    }
    return x;
}

// sort n <= FK_ITEMS_MAX u64 keys in this wave's LDS buffer (bitonic over the next power of two; pads with ~0)
__device__ void wave_sort_lds(uint64_t *a, uint32_t n)
{
    const int lane = lane_id();
    uint32_t n2 = WAVE;
    while (n2 < n) n2 <<= 1;
    for (uint32_t i = n + (uint32_t)lane; i < n2; i += WAVE) a[i] = ~0ull;
    wave_sync();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = (uint32_t)lane; i < n2; i += WAVE) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t x = a[i], y = a[l];
                    if ((x > y) == ((i & k) == 0)) { a[i] = y; a[l] = x; }
                }
            }
            wave_sync();
        }
    }
}

// Regex-position tasks are queued per wave and run after the wave's last
// document, where few registers are live (a call from inside the resolve
// would spill the caller's state on every decided regex name).
struct RxQueue {
    uint4 *q;
    uint32_t n, cap;
    uint8_t *txt;   // the wave's LDS text staging buffer (RX_TXT bytes)
};

__device__ __forceinline__ void fk_regex_enqueue(const DevScratch &GS, const FieldCtx &F, uint32_t P, RxQueue &Q)
{
    if (Q.n < Q.cap) {
        if (lane_id() == 0) Q.q[Q.n] = make_uint4(F.doc, F.field | (F.ascii ? 2u : 0u), P, F.n);
    } else if (lane_id() == 0) {
        atomicOr(&GS.status[0], ST_RX_OVERFLOW);   // the host grows the queues and scans again
    }
    ++Q.n;
}

// Short field (n <= 64 code points): the field is the needle, the fuzzy names at least as long as
// the field are the haystacks (exact-substring table for n <= 10, signatures + LCS above).
// on_regex(P) receives the decided regex-class names (their positions need the regex search).
template <class RxFn>
__device__ void fk_short_field(const FastTables &FT, const uint32_t *__restrict__ pcps, const DevScratch &GS,
                               const FieldCtx &F, OutCtx &O,
                               unsigned long long &nver, unsigned long long &nwin, RxFn on_regex)
{
    const int lane = lane_id();
    const uint32_t n = F.n;
    if (n == 0) {
        if (FT.empty_pat >= 0) emit_hits(O, GS, lane == 0, F.doc, (uint32_t)FT.empty_pat, 0u, F.field);
        return;
    }
    const uint32_t fc = (lane < (int)n) ? fk_cp(F, lane) : 0xFFFFFFFCu;
    if (n <= (uint32_t)SHORT_EXACT_MAX) {
        uint64_t h = 0;
        for (uint32_t i = 0; i < n; ++i) h = h * SUB_B + (uint32_t)__builtin_amdgcn_readlane(fc, i);
        const uint64_t key = (h + (uint64_t)n * 0x9E3779B97F4A7C15ull) | 1ull;
        uint32_t slot = (uint32_t)(key >> 32) & FT.sub_mask;
        uint32_t b = 0, cnt = 0;
        for (;;) {
            const uint64_t kk = FT.sub_key[slot];
            if (kk == key) { b = FT.sub_begin[slot]; cnt = FT.sub_cnt[slot]; break; }
            if (kk == 0) break;
            slot = (slot + 1) & FT.sub_mask;
        }
        b = __builtin_amdgcn_readfirstlane(b);
        cnt = __builtin_amdgcn_readfirstlane(cnt);
        uint32_t fch[SHORT_EXACT_MAX];
#pragma unroll
        for (int j = 0; j < SHORT_EXACT_MAX; ++j) fch[j] = __builtin_amdgcn_readlane(fc, j);
        for (uint32_t c0 = 0; c0 < cnt; c0 += WAVE) {
            const uint32_t idx = c0 + lane;
            bool hit = false, exact = false;
            uint32_t P = 0, rk = 0;
            if (idx < cnt) {
                const uint32_t e = FT.sub_pat[b + idx];
                P = e & 0xFFFFFu;
                const uint32_t m = pi_m(FT.pat_info[P]);
                rk = FT.pat_rxk[P];
                const uint32_t *nmp = pcps + FT.pat_cp_off[P];
                {   // the substring's recorded offset first (loads in flight together), every offset on a collision
                    const uint32_t p0 = e >> 20;
                    bool eq = p0 + n <= m;
#pragma unroll
                    for (int j = 0; j < SHORT_EXACT_MAX; ++j)
                        if ((uint32_t)j < n) eq = eq && nmp[p0 + j] == fch[j];
                    hit = eq;
                }
                for (uint32_t p = 0; p + n <= m && !hit; ++p) {
                    bool eq = true;
#pragma unroll
                    for (int j = 0; j < SHORT_EXACT_MAX; ++j)
                        if ((uint32_t)j < n) eq = eq && nmp[p + j] == fch[j];
                    hit = eq;
                }
                exact = hit && m == n;
            }
            // literal: position 0 iff the name equals the field
            const bool lit = hit && rk == RXK_LITERAL;
            emit_hits(O, GS, lit, F.doc, P, exact ? 0u : KW_NOPOS, F.field);
            uint64_t rxm = __ballot(hit && rk == RXK_REGEX);
            while (rxm) {
                const int l = __builtin_ctzll(rxm);
                rxm &= rxm - 1;
                on_regex((uint32_t)__shfl((int)P, l, WAVE));
            }
        }
        return;
    }
    // signature of the field's characters
    uint64_t fsig = 0;
    {
        uint64_t bit = (lane < (int)n) ? (1ull << (fc & 63)) : 0ull;
        for (int d = 1; d < WAVE; d <<= 1) bit |= __shfl_xor(bit, d, WAVE);
        fsig = bit;
    }
    const uint32_t allow = (2 * n - 1) / 20;   // unmatched field chars any passing window allows
    const uint32_t count = (uint32_t)FT.f_count_ge[n];
    constexpr int SIG_U = 8;   // signature chunks in flight
    for (uint32_t c00 = 0; c00 < count; c00 += SIG_U * WAVE) {
        uint64_t nsig[SIG_U];
#pragma unroll
        for (int u = 0; u < SIG_U; ++u) {
            const uint32_t idx = c00 + (uint32_t)(u * WAVE + lane);
            nsig[u] = idx < count ? FT.pat_sig[FT.f_first + idx] : ~0ull;
        }
#pragma unroll
      for (int u = 0; u < SIG_U; ++u) {
        const uint32_t c0 = c00 + (uint32_t)(u * WAVE);
        const bool cand = c0 + (uint32_t)lane < count && (uint32_t)__popcll(fsig & ~nsig[u]) <= allow;
        uint64_t cm = __ballot(cand);
        while (cm) {
            const int l = __builtin_ctzll(cm);
            cm &= cm - 1;
            const uint32_t P = (uint32_t)FT.f_first + c0 + (uint32_t)l;
            const uint32_t m = pi_m(FT.pat_info[P]);
            bool exact = false;
            ++nver;
            const uint32_t nmr = (lane < (int)m) ? pcps[FT.pat_cp_off[P] + lane] : 0xFFFFFFFDu;
            if (!fk_short_decide(fc, n, nmr, m, &exact, nwin)) continue;
            if (FT.pat_rxk[P] == RXK_REGEX) on_regex(P);
            else emit_hits(O, GS, lane == 0, F.doc, P, exact ? 0u : KW_NOPOS, F.field);
        }
      }
    }
}

// ---------------------------------------------------------------- fast resolve of one field
// Returns 0 when done, 1 if the field is a long non-ASCII field and 3 if the
// items overflowed: the document then goes to the generic kernel.
template <uint32_t ICAP>
__device__ int fk_resolve_field(const FastTables &FT, const DevTables &T, const DevScratch &GS, FieldCtx &F, OutCtx &O,
                                 uint64_t *items_lds, uint32_t *icnt_f, uint32_t *dflag, uint32_t *cps,
                                 uint32_t *blkcnt, uint64_t *rxtab, RxQueue &RQ, bool maybe_nonascii, bool edge,
                                 unsigned long long &nver,
                                 unsigned long long &nwin, unsigned long long &nedge, unsigned long long *tacc)
{
    const int lane = lane_id();
    // ---- field facts (code points, ASCII) on demand
    const int64_t flen = F.fe - F.fb;
    // the scan's non-ASCII flags are exact per field
    F.ascii = !maybe_nonascii;
    F.n = (uint32_t)flen;
    FK_T0(tr0);
    if (!F.ascii) {
        if (flen > (int64_t)FK_CP_CAP) return 1;
        F.n = decode_field_fast(F.arena, F.fb, F.fe, cps, blkcnt, FK_CP_CAP);
        F.cps = cps;
        F.blkcnt = blkcnt;
    }
    FK_TACC(tacc[0], tr0);
    FK_T0(tr1);
    const bool is_short = F.n <= (uint32_t)MAXM;
    // ---- one-deletion edge windows of the 11..20-code-point names (prefiltered by the scan)
    if (edge && F.n >= EDGE_MIN_M + 1) {
        uint32_t added = fk_edge_items<ICAP>(FT, F, items_lds, icnt_f, dflag);
        added = (uint32_t)wave_sum((int)added);
        if (added) {
            nedge += added;
            wave_sync();
            if (__builtin_amdgcn_readfirstlane(*dflag)) return 3;
        }
    }
    wave_sync();
    FK_TACC(tacc[1], tr1);
    FK_T0(tr2);
    const uint32_t N = __builtin_amdgcn_readfirstlane(*icnt_f);
    if (N == 0 && !is_short) return 0;
    if (N > (uint32_t)WAVE) {
        // more than one register tile: sort in LDS, then take pattern-aligned batches of <= 64 items
        wave_sort_lds(items_lds, N);
    }
    for (uint32_t bs = 0; bs < N;) {
        uint32_t be = N;
        if (N > (uint32_t)WAVE) {
            be = bs + WAVE < N ? bs + WAVE : N;
            if (be < N) {
                while (be > bs && it_pat(items_lds[be]) == it_pat(items_lds[be - 1])) --be;
                if (be == bs) return 3;   // one name with more than 64 items: the generic kernel
            }
        }
        const uint32_t NB = be - bs;
        uint64_t it = (lane < (int)NB) ? items_lds[bs + lane] : ~0ull;
        it = wave_sort_few(it, NB, items_lds + bs);
        bs = be;
        const bool valid = lane < (int)NB;
        const uint32_t pat = valid ? it_pat(it) : 0xFFFFFu;
        const uint32_t kind = it_kind(it);
        const uint32_t bpos = it_pos(it);
        const uint32_t use = it_use(it);
        const uint32_t pi = valid ? FT.pat_info[pat] : 0u;
        const uint32_t rxk = valid ? FT.pat_rxk[pat] : 0u;
        const uint32_t m = pi_m(pi);
        const bool fuzzy = (pi & PI_FUZZY) != 0;
        const uint32_t prev_pat = (uint32_t)__shfl_up((int)pat, 1, WAVE);
        const bool head = valid && (lane == 0 || prev_pat != pat);
        const uint64_t heads = __ballot(head);
        const uint64_t below = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
        const int gs = 63 - __builtin_clzll((heads & below) | 1ull);
        const uint64_t after = heads & ~below;
        const int ge = after ? __builtin_ctzll(after) : (int)NB;
        const uint64_t gmask = (ge >= 64 ? ~0ull : ((1ull << ge) - 1)) & ~((1ull << gs) - 1);
        // the short path owns fuzzy names at least as long as the field
        const bool live = valid && !(fuzzy && m >= F.n);
        // (kind 3 is an edge item here only with use IT_USE_MASK; the probe's RXM items never decide)
        const uint64_t fullm = __ballot(live && (kind == FU_FULL || (kind == FU_EDGE && use == IT_USE_MASK)));
        const bool decided_full = (fullm & gmask) != 0;
        // ---- verification of pieces of undecided fuzzy names (wave-serial over such items)
        const bool vpiece = live && fuzzy && !decided_full && kind == FU_PIECE;
        // every piece lane's use record and code point position at once
        const uint32_t vinfo = vpiece ? FT.use_info1[use] : 0u;
        const uint32_t vq = vpiece ? to_cp_fast(F, bpos) : 0u;
        uint64_t vneed = __ballot(vpiece);
        uint64_t decided_v = 0;   // bit per lane: its group got decided by a window
        uint32_t last_P = 0xFFFFFFFFu, nm = 0xFFFFFFFDu;
        int64_t last_key = -1;
        while (vneed) {
            const int l = __builtin_ctzll(vneed);
            vneed &= vneed - 1;
            const uint64_t lg = __shfl(gmask, l, WAVE);
            if (decided_v & lg) continue;                       // group already decided
            const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)pat, l);
            const uint32_t mm = (uint32_t)__builtin_amdgcn_readlane((int)m, l);
            const uint32_t info1 = (uint32_t)__builtin_amdgcn_readlane((int)vinfo, l);
            const uint32_t o = (info1 >> 16) & 0xFF, pl = info1 >> 24;
            const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)vq, l);
            // pieces of one occurrence share the alignment base = q - o: verify it once
            const int64_t key = piece_window_key(q, o, pl, mm, F.n);
            if (P == last_P && key == last_key) continue;
            if (P != last_P) nm = (lane < (int)mm) ? FT.pat_cps[FT.pat_cp_off[P] + lane] : 0xFFFFFFFDu;
            last_P = P;
            last_key = key;
            ++nver;
            if (fk_verify_piece(F, nm, mm, q, o, pl, nwin)) decided_v |= lg;
        }
        const bool decided = decided_full || ((decided_v >> lane) & 1ull);
        // ---- positions: U names and literal fuzzy names report their exact occurrences
        const bool relevant = live && ((!fuzzy && kind == FU_UPPER) ||
                                       (fuzzy && decided && rxk == RXK_LITERAL && kind == FU_FULL));
        const uint32_t cpos = relevant ? to_cp_fast(F, bpos) : 0u;
        const uint64_t relm = __ballot(relevant);
        // leftmost non-overlapping selection per group (a match spans m code points)
        const uint64_t prevrel = relm & gmask & ((1ull << lane) - 1);
        const int pr = prevrel ? 63 - __builtin_clzll(prevrel) : -1;
        const uint32_t pcpos = (uint32_t)__shfl((int)cpos, pr < 0 ? lane : pr, WAVE);
        const bool overlap = relevant && pr >= 0 && cpos < pcpos + m;
        uint64_t keep = relm;
        if (__ballot(overlap)) {
            // rare: resolve the greedy chain serially
            keep = 0;
            uint64_t mm2 = relm;
            int cur_head = -1;
            uint32_t last_end = 0;
            while (mm2) {
                const int l = __builtin_ctzll(mm2);
                mm2 &= mm2 - 1;
                const int h = __shfl(gs, l, WAVE);
                const uint32_t s = (uint32_t)__shfl((int)cpos, l, WAVE);
                const uint32_t len = (uint32_t)__shfl((int)m, l, WAVE);
                if (h != cur_head) { cur_head = h; last_end = 0; keep |= 1ull << l; last_end = s + len; continue; }
                if (s >= last_end) { keep |= 1ull << l; last_end = s + len; }
            }
        }
        const bool k_me = (keep >> lane) & 1ull;
        emit_hits(O, GS, k_me, F.doc, pat, cpos, F.field);
        // decided literal fuzzy groups without any occurrence: `name: []`
        const bool none_kept = (keep & gmask) == 0;
        emit_hits(O, GS, head && live && fuzzy && decided && rxk == RXK_LITERAL && none_kept, F.doc, pat, KW_NOPOS,
                  F.field);
        // decided regex-class names: re.finditer over the field
        uint64_t rxm = __ballot(head && live && fuzzy && decided && rxk == RXK_REGEX);
        while (rxm) {
            const int l = __builtin_ctzll(rxm);
            rxm &= rxm - 1;
            fk_regex_enqueue(GS, F, (uint32_t)__shfl((int)pat, l, WAVE), RQ);
        }
    }
    FK_TACC(tacc[2], tr2);
    // ---- short field: the field is the needle, the longer names are the haystacks
    FK_T0(tr3);
    if (is_short) fk_short_field(FT, FT.pat_cps, GS, F, O, nver, nwin, [&](uint32_t P) { fk_regex_enqueue(GS, F, P, RQ); });
    FK_TACC(tacc[3], tr3);
    return 0;
}


// ---------------------------------------------------------------- flat resolve (all-ASCII documents)
// The scan kernel finishes an all-ASCII document itself (fk_scan_epilogue): it sorts the document's
// items, emits the positions of uppercase names and of exact occurrences of literal fuzzy names,
// (edge windows included) and leaves the rest as tasks in its wave's task regions for the task kernels
// (kw_verify_kernel, kw_short_kernel, kw_rx_task_kernel):
//   vq  {doc, P << 1 | field, q, o | pl << 8}   a pigeonhole piece of an undecided fuzzy name
//   sq  {doc, field, 0, 0}                       a field of <= 64 code points
//   xq  {doc, P << 1 | field, 0, 0}              a regex-class name decided by an exact occurrence
// A name can be decided by more than one source (an exact occurrence and an edge window; several
// pieces); the decided set makes the first one the only one that emits `name: []` or runs the
// regex search.
__device__ __forceinline__ unsigned long long dset_key(uint32_t doc, uint32_t P, uint32_t field)
{
    return (((unsigned long long)doc << 21) | ((unsigned long long)P << 1) | field) + 1ull;
}

__device__ __forceinline__ unsigned long long dset_slot(unsigned long long key, unsigned long long mask)
{
    return ((key * 0x9E3779B97F4A7C15ull) >> 20) & mask;
}

// true iff this call inserted the key (one lane calls)
__device__ bool dset_insert(const FastScratch &S, unsigned long long key)
{
    unsigned long long slot = dset_slot(key, S.dmask);
    for (unsigned long long probe = 0; probe <= S.dmask; ++probe) {
        const unsigned long long cur = atomicCAS(&S.dset[slot], 0ull, key);
        if (cur == 0ull) return true;
        if (cur == key) return false;
        slot = (slot + 1) & S.dmask;
    }
    atomicOr(&S.status[0], ST_DSET_FULL);
    return false;
}

__device__ bool dset_contains(const FastScratch &S, unsigned long long key)
{
    unsigned long long slot = dset_slot(key, S.dmask);
    for (unsigned long long probe = 0; probe <= S.dmask; ++probe) {
        const unsigned long long cur = __atomic_load_n(&S.dset[slot], __ATOMIC_RELAXED);
        if (cur == key) return true;
        if (cur == 0ull) return false;
        slot = (slot + 1) & S.dmask;
    }
    return false;
}

// wave-uniform decision "insert (doc, field, P)": lane 0 inserts, every lane gets the answer
__device__ __forceinline__ bool dset_insert_wave(const FastScratch &S, uint32_t doc, uint32_t P, uint32_t field)
{
    int ins = 0;
    if (lane_id() == 0) ins = dset_insert(S, dset_key(doc, P, field)) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(ins) != 0;
}

// append one record to a wave's task region (cnt is wave-uniform; lane 0 writes)
__device__ __forceinline__ void task_push(uint4 *region, uint32_t cap, uint32_t &cnt, uint4 rec)
{
    if (cnt < cap && lane_id() == 0) region[cnt] = rec;
    ++cnt;
}

struct TaskCounts {
    uint32_t v, e, s, x;
};

// true iff some name has more than 64 items in the sorted list a[0, n) (lane-parallel)
__device__ __forceinline__ bool fk_long_run(const uint64_t *a, uint32_t n)
{
    bool r = false;
    for (uint32_t i = (uint32_t)lane_id(); i + WAVE < n; i += WAVE) r |= it_pat(a[i]) == it_pat(a[i + WAVE]);
    return __ballot(r) != 0;
}

// Whether a short field (<= MAXM code points, one byte each: ASCII or the transcoded view) needs the short
// kernel: fields of <= SHORT_EXACT_MAX always; longer ones only if some name at least as long passes the
// short kernel's signature test (popcount(field signature & ~name signature) <= (2n - 1) / 20), checked here
// when those names are at most 64.  Whole wave.
__device__ __forceinline__ bool fk_short_has_cand(const FastTables &FT, const FieldCtx &F)
{
    const int lane = lane_id();
    const uint32_t n = F.n;
    if (n <= (uint32_t)SHORT_EXACT_MAX) return true;
    const uint32_t cnt = (uint32_t)FT.f_count_ge[n];
    if (cnt > (uint32_t)WAVE) return true;
    uint64_t fsig = (lane < (int)n) ? 1ull << (F.arena[F.fb + lane] & 63u) : 0ull;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) fsig |= __shfl_xor(fsig, d, WAVE);
    const uint32_t allow = (2 * n - 1) / 20;
    const bool c = lane < (int)cnt && (uint32_t)__popcll(fsig & ~FT.pat_sig[FT.f_first + lane]) <= allow;
    return __ballot(c) != 0;
}

// One-deletion edge windows of a document's 11..20-code-point names (flags: its edge prefilter bits), after its
// items were decided (the decided set then holds every name an exact occurrence decided).
__device__ __forceinline__ void fk_epi_edge(const FastTables &FT, const FastScratch &S, const DevScratch &GS,
                                            const FastDoc &D, uint32_t flags, OutCtx &O, TaskCounts &TC, uint4 *xq)
{
    const int lane = lane_id();
    // ---- one-deletion edge windows of the 11..20-code-point names, both fields at once:
    // lane 20 f + 10 side + (L - 10) hashes the first (side 0) or last (side 1) L bytes of field f
    if ((FK_EPI_EDGE & 1) && (flags & (DH_EDGE0 | DH_EDGE1)) && (FK_EPI_EDGE & 2)) {
        const int f = lane >= 20 ? 1 : 0;
        const int sidx = lane - 20 * f;
        const uint32_t L = (EDGE_MIN_M - 1) + (uint32_t)(sidx % 10);
        const int64_t fb = f ? D.t1 : D.t0, fe = f ? D.t2 : D.t1;
        const bool act = lane < 40 && (flags & (f ? DH_EDGE1 : DH_EDGE0)) && fe - fb >= (int64_t)L + 2;
        const int64_t w0 = sidx >= 10 ? fe - (int64_t)L : fb;
        uint64_t hh = 0;
        uint32_t wb[5] = {0u, 0u, 0u, 0u, 0u};   // the window's first 20 bytes
        if (act) {
            const int64_t a0 = w0 & ~(int64_t)3;
            const uint32_t sh = (uint32_t)(w0 & 3);
            uint32_t dw[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) dw[i] = *(const uint32_t *)(D.arena + a0 + 4 * i);   // the arena is padded
#pragma unroll
            for (int i = 0; i < 5; ++i) wb[i] = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], sh);
#pragma unroll
            for (int j = 0; j < (int)EDGE_MAX_M - 1; ++j)
                if ((uint32_t)j < L) hh = hh * SUB_B + ((wb[j >> 2] >> (8 * (j & 3))) & 0xFFu);
        }
        uint32_t ecur = 0, eend = 0;
        if (act) {
            const uint64_t key = (hh + (uint64_t)L * 0x9E3779B97F4A7C15ull) | 1ull;
            uint32_t slot = (uint32_t)(key >> 32) & FT.edge_mask;
            for (;;) {
                const uint64_t kk = FT.edge_key[slot];
                if (kk == key) { ecur = FT.edge_begin[slot]; eend = ecur + FT.edge_cnt[slot]; break; }
                if (kk == 0) break;
                slot = (slot + 1) & FT.edge_mask;
            }
        }
        // one matching variant per lane per round (a lane rarely has two)
        while (__ballot(ecur < eend)) {
            uint32_t P = 0;
            bool hit = false;
            while (ecur < eend && !hit) {
                const uint32_t ent = FT.edge_ent[ecur++];
                P = ent >> 5;
                const uint32_t del = ent & 31u;
                const uint32_t pi = FT.pat_info[P], co = FT.pat_cp_off[P];
                if (pi_m(pi) != L + 1) continue;
                // the name's code points, all loads in flight together; the window is in wb
                uint32_t nmv[EDGE_MAX_M];
#pragma unroll
                for (int k = 0; k < (int)EDGE_MAX_M; ++k) nmv[k] = (uint32_t)k <= L ? FT.pat_tcps[co + k] : 0u;
                bool eq = true;
#pragma unroll
                for (int j = 0; j < (int)EDGE_MAX_M - 1; ++j) {
                    const uint32_t want = (uint32_t)j < del ? nmv[j] : nmv[j + 1];
                    if ((uint32_t)j < L) eq = eq && ((wb[j >> 2] >> (8 * (j & 3))) & 0xFFu) == want;
                }
                hit = eq;
            }
            const bool first = hit && dset_insert(S, dset_key(D.doc, P, (uint32_t)f));
            const bool rx = first && FT.pat_rxk[P] == RXK_REGEX;
            emit_hits(O, GS, first && !rx, D.doc, P, KW_NOPOS, (uint32_t)f);
            const uint64_t xm = __ballot(rx);
            if (xm) {
                const uint32_t xi = TC.x + mbcnt(xm);
                if (rx && xi < S.xcap) xq[xi] = make_uint4(D.doc, (P << 1) | (uint32_t)f, 0u, 0u);
                TC.x += (uint32_t)__popcll(xm);
            }
            TC.e += (uint32_t)__popcll(__ballot(hit));   // edge items found (statistics)
        }
    }
}

// Finish an all-ASCII document in the scan kernel.  items: the wave's LDS item lists (field 0 at 0,
// field 1 at f1off; each buffer holds the next power of two of its count), n0 / n1 items.  Returns
// false, before anything is emitted, when a name has more than 64 items in a field (the generic kernel
// takes the document).
template <uint32_t F1OFF = FK_ITEMS0>
__device__ bool fk_scan_epilogue(const FastTables &FT, const FastScratch &S, const DevScratch &GS, const FastDoc &D,
                                 uint64_t *items, uint32_t n0, uint32_t n1, uint32_t flags, int64_t wave, OutCtx &O,
                                 TaskCounts &TC, unsigned long long *ekt = nullptr)
{
    constexpr uint32_t f1off = F1OFF;
    const int lane = lane_id();
    unsigned long long ekt_dummy[8];
    if (!ekt) ekt = ekt_dummy;
    EK_T0(te0);
    // the fields' items sorted first: the deferral test precedes every emission
    if (n0 > (uint32_t)WAVE) {
        wave_sort_lds(items, n0);
        if (fk_long_run(items, n0)) return false;
    }
    if (F1OFF != FK_ITEMS0 && n1 > (uint32_t)WAVE) {   // (big documents only: the epilogue kernel holds <= 64)
        wave_sort_lds(items + f1off, n1);
        if (fk_long_run(items + f1off, n1)) return false;
    }
    uint4 *vq = S.vq + (size_t)wave * S.vcap;
    uint4 *sq = S.sq + (size_t)wave * S.scap, *xq = S.xq + (size_t)wave * S.xcap;
    EK_TACC(ekt[0], te0);
    for (uint32_t f = 0; f < 2; ++f) {
        FieldCtx F;
        F.arena = D.arena;
        F.fb = f ? D.t1 : D.t0;
        F.fe = f ? D.t2 : D.t1;
        F.n = (uint32_t)(F.fe - F.fb);
        F.ascii = true;
        F.cps = nullptr;
        F.blkcnt = nullptr;
        F.doc = D.doc;
        F.field = f;
        const uint32_t N = f ? n1 : n0;
        uint64_t *its = items + (f ? f1off : 0);
        // (RXM items are exact regex matches in an ASCII field only; a transcoded field's regex names are searched)
        const bool rxm_ok = !(flags & (f ? DH_NA1 : DH_NA0));
        if (F.n <= (uint32_t)MAXM && fk_short_has_cand(FT, F)) {
            if (SHORT_COUNT && lane == 0) atomicAdd(&S.stats[27 + (flags & (DH_NA0 | DH_NA1) ? 1 : 0)], 1ull);
            task_push(sq, S.scap, TC.s, make_uint4(D.doc, f, 0u, 0u));
        }
        if (N == 0) continue;
        for (uint32_t bs = 0; bs < N;) {
            uint32_t be = N;
            if (N > (uint32_t)WAVE) {
                be = bs + WAVE < N ? bs + WAVE : N;
                if (be < N)
                    while (be > bs && it_pat(its[be]) == it_pat(its[be - 1])) --be;
                if (be == bs) be = bs + WAVE;   // (cannot happen: fk_long_run deferred such documents)
            }
            const uint32_t NB = be - bs;
            EK_T0(te1);
            uint64_t it = (lane < (int)NB) ? its[bs + lane] : ~0ull;
            it = wave_sort_few(it, NB, its + bs);
            bs = be;
            EK_TACC(ekt[1], te1);
            EK_T0(te2);
            const bool valid = lane < (int)NB;
            const uint32_t pat = valid ? it_pat(it) : 0xFFFFFu;
            const uint32_t kind = it_kind(it);
            const uint32_t bpos = it_pos(it);
            const uint32_t use = it_use(it);
            // the name's info, regex class and (pieces) use record: all lanes' loads in flight at once
            const uint32_t pi = valid ? FT.pat_info[pat] : 0u;
            const uint32_t rxk = valid ? FT.pat_rxk[pat] : 0u;
            const uint32_t rxl = valid ? FT.pat_rxl[pat] : 0u;
            const uint32_t uinfo = (valid && kind == FU_PIECE) ? FT.use_info1[use] : 0u;
            const uint32_t m = pi_m(pi);
            // a regex name with an RXM use: its positions are its RXM items (matches of rxl code points)
            const bool rxi = rxk == RXK_REGEX && rxl != 0u && rxm_ok;
            const uint32_t mlen = rxi ? rxl : m;
            const bool fuzzy = (pi & PI_FUZZY) != 0;
            const uint32_t prev_pat = (uint32_t)__shfl_up((int)pat, 1, WAVE);
            const bool head = valid && (lane == 0 || prev_pat != pat);
            const uint64_t heads = __ballot(head);
            const uint64_t below = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
            const int gs = 63 - __builtin_clzll((heads & below) | 1ull);
            const uint64_t after = heads & ~below;
            const int ge = after ? __builtin_ctzll(after) : (int)NB;
            const uint64_t gmask = (ge >= 64 ? ~0ull : ((1ull << ge) - 1)) & ~((1ull << gs) - 1);
            // the short path owns fuzzy names at least as long as the field
            const bool live = valid && !(fuzzy && m >= F.n);
            const uint64_t fullm = __ballot(live && kind == FU_FULL);
            EK_TACC(ekt[2], te2);
            EK_T0(te3);
            const bool decided = (fullm & gmask) != 0;
            // pieces of undecided fuzzy names -> verify tasks (one per alignment base)
            const bool vpiece = live && fuzzy && !decided && kind == FU_PIECE;
            const uint32_t vinfo = vpiece ? uinfo : 0u;
            uint64_t vneed = __ballot(vpiece);
            uint32_t last_P = 0xFFFFFFFFu;
            int64_t last_key = -1;
            while (vneed) {
                const int l = __builtin_ctzll(vneed);
                vneed &= vneed - 1;
                const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)pat, l);
                const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)bpos, l);   // ASCII: byte = code point
                const uint32_t info1 = (uint32_t)__builtin_amdgcn_readlane((int)vinfo, l);
                const uint32_t o = (info1 >> 16) & 0xFF, pl = info1 >> 24;
                const uint32_t mP = (uint32_t)__builtin_amdgcn_readlane((int)m, l);
                const int64_t key = piece_window_key(q, o, pl, mP, F.n);
                if (P == last_P && key == last_key) continue;
                last_P = P;
                last_key = key;
                task_push(vq, S.vcap, TC.v, make_uint4(D.doc, (P << 1) | f, q, o | (pl << 8)));
            }
            // positions: uppercase names, exact occurrences of decided literal fuzzy names, RXM matches of
            // decided regex names
            const bool relevant = live && ((!fuzzy && kind == FU_UPPER) ||
                                           (fuzzy && decided && ((rxk == RXK_LITERAL && kind == FU_FULL) ||
                                                                 (rxi && kind == FU_RXM))));
            const uint32_t cpos = bpos;
            const uint64_t relm = __ballot(relevant);
            const uint64_t prevrel = relm & gmask & ((1ull << lane) - 1);
            const int pr = prevrel ? 63 - __builtin_clzll(prevrel) : -1;
            const uint32_t pcpos = (uint32_t)__shfl((int)cpos, pr < 0 ? lane : pr, WAVE);
            const bool overlap = relevant && pr >= 0 && cpos < pcpos + mlen;
            uint64_t keep = relm;
            if (__ballot(overlap)) {
                keep = 0;
                uint64_t mm2 = relm;
                int cur_head = -1;
                uint32_t last_end = 0;
                while (mm2) {
                    const int l = __builtin_ctzll(mm2);
                    mm2 &= mm2 - 1;
                    const int hh = __shfl(gs, l, WAVE);
                    const uint32_t st = (uint32_t)__shfl((int)cpos, l, WAVE);
                    const uint32_t len = (uint32_t)__shfl((int)mlen, l, WAVE);
                    if (hh != cur_head) { cur_head = hh; keep |= 1ull << l; last_end = st + len; continue; }
                    if (st >= last_end) { keep |= 1ull << l; last_end = st + len; }
                }
            }
            emit_hits(O, GS, (keep >> lane) & 1ull, F.doc, pat, cpos, F.field);
            // exactly decided fuzzy names: an edge window (11 <= m <= 20) may decide them again -> the set;
            // regex-class ones get their re.finditer search unless their RXM items gave the positions
            const bool dec_head = head && live && fuzzy && decided;
            if (dec_head && m >= EDGE_MIN_M && m <= EDGE_MAX_M) (void)dset_insert(S, dset_key(D.doc, pat, f));
            emit_hits(O, GS, dec_head && rxi && (keep & gmask) == 0, F.doc, pat, KW_NOPOS, F.field);
            const bool xrx = dec_head && rxk == RXK_REGEX && !rxi;
            const uint64_t xm = __ballot(xrx);
            if (xm) {
                const uint32_t xi = TC.x + mbcnt(xm);
                if (xrx && xi < S.xcap) xq[xi] = make_uint4(D.doc, (pat << 1) | f, 0u, 0u);
                TC.x += (uint32_t)__popcll(xm);
            }
            EK_TACC(ekt[3], te3);
        }
    }
    EK_T0(te4);
    fk_epi_edge(FT, S, GS, D, flags, O, TC, xq);
    EK_TACC(ekt[4], te4);
    return true;
}

// ---------------------------------------------------------------- kernel: the tasks of the flat resolve
// Task wave t works the task regions of scan wave t: verify, edge, short, then regex tasks.
// field of an epilogue document through its view record (the arena, or the transcoded view of a document
// with a non-ASCII field: one byte per code point)
__device__ __forceinline__ void fk_field_ctx(FieldCtx &F, const uint8_t *arena, const FastScratch &S, uint32_t doc,
                                             uint32_t field)
{
    const uint4 v = S.vrec[doc];
    F.tx = (v.y >> 31) != 0;
    F.arena = F.tx ? S.tarena : arena;
    F.fb = (int64_t)(((uint64_t)(v.y & 0x7FFFFFFFu) << 32) | v.x) + (field ? (int64_t)v.z : 0);
    F.n = field ? v.w : v.z;
    F.fe = F.fb + F.n;
    F.ascii = true;
    F.cps = nullptr;
    F.blkcnt = nullptr;
    F.doc = doc;
    F.field = field;
}

// a decided regex-class name: re.finditer over the field, or `name: []` (rxtab: 256 entries); the program's
// index and parameters come prefetched (the regex task kernel's records)
__device__ __forceinline__ void fk_regex_pre(const FastTables &FT, const DevTables &T, const DevScratch &GS,
                                             const FieldCtx &F, OutCtx &O, uint32_t P, int32_t r, const RxfParams &prm,
                                             uint64_t *rxtab, uint8_t *txt, unsigned long long &nrx,
                                             unsigned long long &nrx_bt, unsigned long long &nrx_rounds)
{
    ++nrx;
    nrx_bt += r < 0;
    nrx_rounds += r >= 0 ? (F.n + 2047) / 2048 : 0;
#if defined(RX_TIMING_SKIP) && RX_TIMING_SKIP == 5   // (timing variant: no backtracking engine in the kernel)
    const uint32_t cnt = r >= 0 ? fk_rx_fixed_positions<true>(FT, GS, F, O, P, (uint32_t)r, prm, rxtab, txt) : 1u;
#else
    const uint32_t cnt = r >= 0 ? fk_rx_fixed_positions<true>(FT, GS, F, O, P, (uint32_t)r, prm, rxtab, txt)
                                : rx_positions(T, GS, F, O, P);
#endif
    if (cnt == 0) emit_hits(O, GS, lane_id() == 0, F.doc, P, KW_NOPOS, F.field);
}

// ---- lane-parallel verification of a piece of an ASCII name in an ASCII field (one lane = one task)
// exact zero-byte flags (the high bit of every zero byte) of a 64-bit word
__device__ __forceinline__ uint64_t zb64(uint64_t x)
{
    return ~(((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x | 0x7F7F7F7F7F7F7F7Full);
}
// the 8 byte flags of zb64 -> bits 0..7
__device__ __forceinline__ uint32_t hb8(uint64_t z)
{
    return (uint32_t)((((z >> 7) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
}

constexpr int LV_WIN = 23;   // dwords of text per lane in LDS (stride 23: no bank conflicts between lanes)

// 8 text bytes at byte d of the lane's window: one ds_read_b64 at any byte address (LDS runs in unaligned mode on
// gfx950: scripts/probe/lds_unaligned.hip)
__device__ __forceinline__ uint64_t lv_text8(const uint32_t *win, int64_t d)
{
    return *(const uint64_t *)((const uint8_t *)win + d);
}

// positions of byte c in the name (bit i = name[i] == c), name in 8 little-endian words
__device__ __forceinline__ uint64_t lv_match(const uint64_t (&NW)[8], uint32_t c, uint64_t needle)
{
    const uint64_t cc = (uint64_t)c * 0x0101010101010101ull;
    uint64_t M = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) M |= (uint64_t)hb8(zb64(NW[w] ^ cc)) << (8 * w);
    return M & needle;
}

// Band test of one lane's verify task (the text [base - 2k, base + m + 2k) staged in the lane's
// LDS window): every name byte matched by a passing full window lies within +-2k of its aligned
// text byte.  Returns the number of full windows [pmin, pmin + nwj) left to evaluate.  The window's bytes
// outside the field are staged as 0 (no name byte is 0; a 0 could only let a task through to the exact window
// jobs), so the shifts need no field-bound masks.
__device__ uint32_t lv_band(const uint8_t *__restrict__ arena, int64_t fb, uint32_t n, const uint64_t (&NW)[8],
                            uint32_t m, int64_t base, uint32_t k, uint32_t *win, int64_t &pmin)
{
    pmin = 0;
    if (k == 0) return 0;
    const uint64_t needle = low_mask(m);
    const int64_t lo = base - 2 * (int64_t)k;
    const int64_t A = (fb + lo) & ~(int64_t)3;
    const int64_t fe = fb + n;
#pragma unroll
    for (int j = 0; j < LV_WIN; ++j) {   // only dwords that overlap the field; their bytes outside it cleared
        const int64_t ad = A + 4 * j;
        uint32_t x = (ad + 4 > fb && ad < fe) ? *(const uint32_t *)(arena + ad) : 0u;
        if (ad < fb) x &= ~0u << (8 * (uint32_t)(fb - ad) & 31u);
        if (ad + 4 > fe) x &= fe > ad ? ~(~0u << (8 * (uint32_t)(fe - ad) & 31u)) : 0u;
        win[j] = x;
    }
    uint64_t hit[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t d0 = fb + base - A;   // window byte of name byte 0 at shift 0
    for (int t = -2 * (int)k; t <= 2 * (int)k; ++t) {
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            if (8 * w >= (int)m) break;
            hit[w] |= zb64(lv_text8(win, d0 + 8 * w + t) ^ NW[w]);
        }
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) cnt += (uint32_t)__popcll(hb8(hit[w]) & (uint32_t)((needle >> (8 * w)) & 0xFFu));
    if (cnt + k < m) return 0;
    int64_t pmax = base + k;
    pmin = base - k;
    if (pmin < 0) pmin = 0;
    if (pmax > (int64_t)(n - m)) pmax = (int64_t)(n - m);
    return pmax >= pmin ? (uint32_t)(pmax - pmin + 1) : 0u;
}

// The band test on the name's first 16 bytes alone (m > 16): those bytes matched within +-2k of their aligned text
// bytes must number >= 16 - k, or the whole test fails (the other m - 16 bytes can add at most m - 16).  Stages
// only the window's first dwords.  A task failing it has no full window to evaluate.
__device__ bool lv_pretest(const uint8_t *__restrict__ arena, int64_t fb, uint32_t n, uint64_t w0, uint64_t w1,
                           int64_t base, uint32_t k, uint32_t *win)
{
    const int64_t lo = base - 2 * (int64_t)k;
    const int64_t A = (fb + lo) & ~(int64_t)3;
    const int64_t fe = fb + n;
    const int nd = (int)((4 * k + 3 + 16 + 7) / 4) + 1;   // dwords the shifts read (<= 12 for k <= 3)
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        if (j >= nd) break;
        const int64_t ad = A + 4 * j;
        uint32_t x = (ad + 4 > fb && ad < fe) ? *(const uint32_t *)(arena + ad) : 0u;
        if (ad < fb) x &= ~0u << (8 * (uint32_t)(fb - ad) & 31u);
        if (ad + 4 > fe) x &= fe > ad ? ~(~0u << (8 * (uint32_t)(fe - ad) & 31u)) : 0u;
        win[j] = x;
    }
    uint64_t h0 = 0, h1 = 0;
    const int64_t d0 = fb + base - A;
    for (int t = -2 * (int)k; t <= 2 * (int)k; ++t) {
        h0 |= zb64(lv_text8(win, d0 + t) ^ w0);
        h1 |= zb64(lv_text8(win, d0 + 8 + t) ^ w1);
    }
    const uint32_t cnt = (uint32_t)__popcll(hb8(h0)) + (uint32_t)__popcll(hb8(h1));
    return cnt + k >= 16u;
}

// regex-class names decided in the task kernels -> the region's regex queue (xq), lane-parallel;
// several waves may append to one region (atomic count)
struct XPush {
    uint4 *q;
    uint32_t cap;
    uint32_t *cnt;
    uint32_t *tmax;
    uint32_t *status;
};

__device__ __forceinline__ void xq_push(XPush &X, bool pred, uint32_t doc, uint32_t P, uint32_t field)
{
    const uint64_t m = __ballot(pred);
    if (!m) return;
    uint32_t b = 0;
    if (lane_id() == 0) b = atomicAdd(X.cnt, (uint32_t)__popcll(m));
    b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
    const uint32_t idx = b + mbcnt(m);
    if (pred) {
        if (idx < X.cap) {
            X.q[idx] = make_uint4(doc, (P << 1) | field, 0u, 0u);
        } else {
            atomicOr(X.status, ST_TASK_OVERFLOW);
            atomicMax(X.tmax, idx + 1);
        }
    }
}

__device__ __forceinline__ XPush xq_region(const FastScratch &S, int64_t t)
{
    XPush X;
    X.q = S.xq + (size_t)t * S.xcap;
    X.cap = S.xcap;
    X.cnt = S.xcnt + t;
    X.tmax = S.tmax + 3;
    X.status = S.status;
    return X;
}

// region t's result list, shared by the waves working the region
__device__ __forceinline__ OutCtx tout_region(const FastScratch &S, int64_t t)
{
    OutCtx O;
    O.shared = nullptr;
    O.out = S.tout + (size_t)t * S.out_cap;
    O.cap = S.out_cap;
    O.n = 0;
    O.shared = S.tout_cnt + t;
    return O;
}

// a name decided without an exact occurrence (edge window): the first decision emits `name: []`
// or queues the regex search.  Wave-uniform.
__device__ __forceinline__ void fk_decide_queue(const FastTables &FT, const FastScratch &S, const DevScratch &GS,
                                                const FieldCtx &F, OutCtx &O, XPush &X, uint32_t P)
{
    if (!dset_insert_wave(S, F.doc, P, F.field)) return;
    const bool rx = FT.pat_rxk[P] == RXK_REGEX;
    xq_push(X, rx && lane_id() == 0, F.doc, P, F.field);
    emit_hits(O, GS, !rx && lane_id() == 0, F.doc, P, KW_NOPOS, F.field);
}

__device__ __forceinline__ void task_stats(const FastScratch &S, unsigned long long v, unsigned long long w,
                                           unsigned long long e, unsigned long long rx, unsigned long long rxbt,
                                           unsigned long long rxr)
{
    if (lane_id() == 0) {
        if (w) atomicAdd(&S.stats[2], w);
        if (v) atomicAdd(&S.stats[3], v);
        if (e) atomicAdd(&S.stats[7], e);
        if (rx) atomicAdd(&S.stats[10], rx);
        if (rxbt) atomicAdd(&S.stats[11], rxbt);
        if (rxr) atomicAdd(&S.stats[12], rxr);
    }
}

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v)
{
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) v += __shfl_xor(v, dd, WAVE);
    return v;
}

constexpr int LV_MAXJ = 16;   // window jobs per verify task: <= 2 kfull(64) + 1 full windows + prefix + suffix

// ---------------------------------------------------------------- kernels: the tasks of the flat resolve
// Task kernels run one wave per scan wave t over the task regions that scan wave wrote, in stream
// order verify -> edge -> short -> regex; each appends to region t's result list (tout) and the
// first three append regex-class decisions to region t's regex queue (xq).

// Verify tasks.  Lanes take 64 tasks at a time: band test per lane, then the surviving windows
// (full windows, prefixes, suffixes) of all 64 tasks as one flat job list, 64 jobs a round, each
// job's text staged in its lane's LDS window.  Names with non-ASCII code points wave-serially.
__global__ __launch_bounds__(RK_BLOCK, VK_MINW) void kw_verify_kernel(FastTables FT, DevTables T, const uint8_t *__restrict__ arena,
                                                             const int64_t *__restrict__ off, int n_regions, int G,
                                                             FastScratch S, DevScratch GS)
{
    __shared__ uint32_t lvwin_all[RK_BLOCK * LV_WIN];
    __shared__ uint16_t jobs_all[RK_BLOCK * LV_MAXJ];
    __shared__ uint32_t okf_all[RK_BLOCK];
    __shared__ uint32_t vsel_all[RK_BLOCK * 2];   // per wave: a ring of 128 task indices that passed the pretest
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t gw = (int64_t)blockIdx.x * RK_WAVES + wib;   // G waves per region
    const int64_t t = gw / G;
    const uint32_t sub = (uint32_t)(gw % G);
    if (t >= n_regions) return;
    uint32_t *win = lvwin_all + threadIdx.x * LV_WIN;
    uint16_t *jobs = jobs_all + wib * WAVE * LV_MAXJ;
    uint32_t *okf = okf_all + wib * WAVE;
    OutCtx O = tout_region(S, t);
    XPush X = xq_region(S, t);
    unsigned long long nver = 0, nwin = 0, nver_w = 0, nwin_w = 0;
    const uint32_t nv = min(S.vcnt[t], S.vcap);
    const uint4 *vq = S.vq + (size_t)t * S.vcap;
    uint32_t *vsel = vsel_all + wib * 2 * WAVE;
    auto run = [&](uint32_t kk, bool valid) {
        const uint4 tk = valid ? vq[kk] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t doc = tk.x, P = tk.y >> 1, field = tk.y & 1u;
        const bool todo = valid && !dset_contains(S, dset_key(doc, P, field));
        const uint32_t pi = todo ? FT.pat_info[P] : 0u;
        const uint32_t m = pi_m(pi);
        const bool lanewise = todo && (pi & PI_ASCII) != 0;
        int64_t fb = 0;
        uint32_t n = 0;
        bool tx = false;
        if (todo) {
            const uint4 v = S.vrec[doc];
            tx = (v.y >> 31) != 0;
            fb = (int64_t)(((uint64_t)(v.y & 0x7FFFFFFFu) << 32) | v.x) + (field ? (int64_t)v.z : 0);
            n = field ? v.w : v.z;
        }
        const uint8_t *la = tx ? S.tarena : arena;
        const uint32_t q = tk.z, o = tk.w & 0xFFu, pl = (tk.w >> 8) & 0xFFu;
        uint64_t NW[8];
        {
            const int64_t nb = lanewise ? FT.pat_boff[P] : 0;
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                uint64_t x = 0;
                if (lanewise && 8 * w < (int)m) x = load8(FT.pat_bytes, nb + 8 * w);
                const int rem = (int)m - 8 * w;
                if (rem < 8) x &= rem <= 0 ? 0ull : ((1ull << (8 * rem)) - 1);
                NW[w] = x;
            }
        }
        // band test -> this lane's window jobs
        int64_t pmin = 0;
        uint32_t nwj = 0, pre = 0, cj = 0;
        if (lanewise) {
            ++nver;
#if defined(VK_TIMING_SKIP)   // (timing variants only, results void: 1 no band test, 2 no band test and no jobs)
            nwj = 0;
            pre = VK_TIMING_SKIP == 1 && q + pl + 1 <= m ? 1u : 0u;
            cj = VK_TIMING_SKIP == 1 ? nwj + pre + (q + m > n ? 1u : 0u) : 0u;
#else
            nwj = lv_band(la, fb, n, NW, m, (int64_t)q - (int64_t)o, kfull(m), win, pmin);
            pre = q + pl + 1 <= m ? 1u : 0u;
            cj = nwj + pre + (q + m > n ? 1u : 0u);
#endif
        }
        int J = 0;
        const int ex = wave_excl_scan((int)cj, &J);
        okf[lane] = 0;
        for (uint32_t j = 0; j < cj; ++j) jobs[ex + j] = (uint16_t)(lane | (j << 6));
        wave_sync();
        for (int g0 = 0; g0 < J; g0 += WAVE) {
            const int g = g0 + lane;
            const bool jv = g < J;
            const uint32_t e = jv ? jobs[g] : 0u;
            const int l = (int)(e & 63u);
            const uint32_t j = e >> 6;
            // the owner's task (every lane shuffles)
            const uint32_t jm = (uint32_t)__shfl((int)m, l, WAVE);
            const uint32_t jn = (uint32_t)__shfl((int)n, l, WAVE);
            const uint32_t jnwj = (uint32_t)__shfl((int)nwj, l, WAVE);
            const uint32_t jpre = (uint32_t)__shfl((int)pre, l, WAVE);
            const uint32_t jpmin = (uint32_t)__shfl((int)(uint32_t)pmin, l, WAVE);
            const uint32_t jP = (uint32_t)__shfl((int)P, l, WAVE);
            const uint32_t fbl = (uint32_t)__shfl((int)(uint32_t)fb, l, WAVE);
            const uint32_t fbh = (uint32_t)__shfl((int)(uint32_t)((uint64_t)fb >> 32), l, WAVE);
            const int64_t jfb = (int64_t)(((uint64_t)fbh << 32) | fbl);
            const uint8_t *ja = __shfl((int)tx, l, WAVE) ? S.tarena : arena;
            if (!jv) continue;
            // job kind: full window at pmin + j, prefix text[:w] (w < m), suffix text[i:] (reversed)
            const bool full = j < jnwj;
            const bool rev = !full && !(j == jnwj && jpre);
            const uint32_t len = full ? jm : jm - 1;
            const int64_t start = full ? (int64_t)jpmin + j : (rev ? (int64_t)jn - len : 0);
            const int64_t A = (jfb + start) & ~(int64_t)3;
            const int64_t fe = jfb + jn;
#pragma unroll
            for (int w = 0; w < 17; ++w) {
                const int64_t ad = A + 4 * w;
                win[w] = (ad + 4 > jfb && ad < fe) ? *(const uint32_t *)(ja + ad) : 0u;
            }
            const uint32_t d0 = (uint32_t)(jfb + start - A);
            const uint64_t needle = low_mask(jm);
            // the name's match vectors from the compiled table (bit i = name[i] == c), eight text bytes'
            // loads in flight at a time
            const uint64_t *pmr = T.pm_ascii + (size_t)jP * 128;
            uint64_t V = ~0ull;
            bool ok = false;
            for (uint32_t s0 = 0; s0 < len && !ok; s0 += VK_U) {
                uint64_t Mb[VK_U];
#pragma unroll
                for (int u = 0; u < VK_U; ++u) {
                    const uint32_t s2 = s0 + (uint32_t)u;
                    const uint32_t bi = d0 + (rev ? len - 1 - s2 : s2);
                    const uint32_t c = s2 < len ? (win[bi >> 2] >> (8 * (bi & 3))) & 0xFFu : 0x80u;
                    Mb[u] = c < 0x80u ? pmr[c] : 0ull;   // (ASCII names never match a non-ASCII byte)
                }
#pragma unroll
                for (int u = 0; u < VK_U; ++u) {
                    const uint32_t s2 = s0 + (uint32_t)u;
                    if (s2 >= len) break;
                    uint64_t M = Mb[u];
                    if (rev) M = __builtin_bitreverse64(M) >> (64 - jm);   // bit i = name[m - 1 - i] == c
                    const uint64_t U = V & M;
                    V = (V + U) | (V - U);
                    if (!full && passes((uint32_t)__popcll(~V & needle), jm, s2 + 1)) { ok = true; break; }
                }
            }
            if (full) ok = 20u * (jm - (uint32_t)__popcll(~V & needle)) < jm;
            ++nwin;
            if (ok) okf[l] = 1u;
        }
        wave_sync();
        bool pass = lanewise && okf[lane] != 0;
        // names lanes cannot take (non-ASCII code points), wave-serially
        uint64_t wm = __ballot(todo && !lanewise);
        while (wm) {
            const int l = __builtin_ctzll(wm);
            wm &= wm - 1;
            FieldCtx F;
            fk_field_ctx(F, arena, S, (uint32_t)__builtin_amdgcn_readlane((int)doc, l),
                         (uint32_t)__builtin_amdgcn_readlane((int)field, l));
            const uint32_t lP = (uint32_t)__builtin_amdgcn_readlane((int)P, l);
            const uint32_t lm = (uint32_t)__builtin_amdgcn_readlane((int)m, l);
            const uint32_t nm = (lane < (int)lm) ? FT.pat_tcps[FT.pat_cp_off[lP] + lane] : 0xFFFFFFFDu;
            const uint32_t lw = (uint32_t)__builtin_amdgcn_readlane((int)tk.w, l);
            const uint32_t lq = (uint32_t)__builtin_amdgcn_readlane((int)tk.z, l);
            ++nver_w;
            const bool dec = fk_verify_piece(F, nm, lm, lq, lw & 0xFFu, (lw >> 8) & 0xFFu, nwin_w);
            if (lane == l) pass = dec;
        }
        // decisions, lane-parallel: the first decision of (doc, name, field) emits or queues the regex search
        const bool first = pass && dset_insert(S, dset_key(doc, P, field));
        const bool rx = first && FT.pat_rxk[P] == RXK_REGEX;
        emit_hits(O, GS, first && !rx, doc, P, KW_NOPOS, field);
        xq_push(X, rx, doc, P, field);
    };
#if VK_PRETEST
    // the tasks 64 at a time through the pretest; the ones it cannot rule out queue up and run the full test (and
    // their window jobs) 64 at a time, so those rounds run on full waves (~90 % of the tasks fail the band test)
    uint32_t qh = 0, qn = 0;
    for (uint32_t k0 = sub * WAVE; k0 < nv; k0 += (uint32_t)G * WAVE) {
        const uint32_t kk = k0 + (uint32_t)lane;
        bool keep = kk < nv;
        if (keep) {
            const uint4 tk = vq[kk];
            const uint32_t P = tk.y >> 1, field = tk.y & 1u;
            const uint32_t pi = FT.pat_info[P];
            const uint32_t m = pi_m(pi);
            if ((pi & PI_ASCII) != 0) {
                const uint4 v = S.vrec[tk.x];
                const bool tx = (v.y >> 31) != 0;
                const int64_t fb = (int64_t)(((uint64_t)(v.y & 0x7FFFFFFFu) << 32) | v.x) + (field ? (int64_t)v.z : 0);
                const uint32_t n = field ? v.w : v.z;
                const uint32_t q = tk.z, o = tk.w & 0xFFu, pl = (tk.w >> 8) & 0xFFu;
                const uint32_t k = kfull(m);
                // (a prefix or suffix job runs whatever the band test says; k = 0: no full window at all, m <= 20)
                if (q + pl + 1 > m && q + m <= n) {
                    if (k == 0) {
                        keep = false;
                    } else if (m > 16u) {
                        const int64_t nb = FT.pat_boff[P];
                        keep = lv_pretest(tx ? S.tarena : arena, fb, n, load8(FT.pat_bytes, nb),
                                          load8(FT.pat_bytes, nb + 8), (int64_t)q - (int64_t)o, k, win);
                    }
                    if (!keep) ++nver;   // (verified: no full window passes)
                }
            }
        }
        const uint64_t km = __ballot(keep);
        wave_sync();
        if (keep) vsel[(qh + qn + mbcnt(km)) & (2u * WAVE - 1u)] = kk;
        qn += (uint32_t)__popcll(km);
        wave_sync();
        if (qn >= (uint32_t)WAVE) {
            const uint32_t kq = vsel[(qh + (uint32_t)lane) & (2u * WAVE - 1u)];
            qh = (qh + WAVE) & (2u * WAVE - 1u);
            qn -= WAVE;
            run(kq, true);
        }
    }
    if (qn) {
        wave_sync();
        const uint32_t kq = vsel[(qh + (uint32_t)lane) & (2u * WAVE - 1u)];
        run(kq, (uint32_t)lane < qn);
    }
#else
    for (uint32_t k0 = sub * WAVE; k0 < nv; k0 += (uint32_t)G * WAVE) run(k0 + (uint32_t)lane, k0 + (uint32_t)lane < nv);
#endif
    task_stats(S, wave_sum64(nver) + nver_w, wave_sum64(nwin) + nwin_w, 0, 0, 0, 0);
}

// ---------------------------------------------------------------- lane-parallel short fields
// An ASCII field of SHORT_EXACT_MAX < n <= 64 bytes against the fuzzy names at least as long
// (the field is the needle).  Candidates come from the signature filter as in fk_short_field;
// then every window of every candidate (full windows of the name, its prefixes, its suffixes and,
// when m == n, the swapped run) is a job on its own lane: a bit-parallel LCS whose match vectors
// come from the field's 128-entry table in LDS (pm), the candidate names staged in LDS (names,
// SL_NAME bytes each).  Names with non-ASCII code points take the wave-serial fk_short_decide.
constexpr int SL_NAME = 64;

__device__ __forceinline__ void fk_short_run(const FastTables &FT, const DevScratch &GS, const FieldCtx &F, OutCtx &O,
                                             XPush &X, const uint64_t *pm, uint8_t *names, uint32_t *cand,
                                             uint32_t nc, uint32_t fc, unsigned long long &nver,
                                             unsigned long long &nwin, unsigned long long &nwin_w)
{
    const int lane = lane_id();
    const uint32_t n = F.n;
    const uint64_t needle = low_mask(n);
    // lane k holds candidate k
    const bool has = lane < (int)nc;
    const uint32_t P = has ? cand[lane] : 0u;
    const uint32_t pi = has ? FT.pat_info[P] : 0u;
    const uint32_t m = pi_m(pi);
    // every name on lanes: its code points as one byte each (ASCII, or the transcoded view's markers), the
    // field's match vectors cover all 256 byte values
    const bool lanes_ok = has && (SHORT_TB || (pi & PI_ASCII) != 0) && m <= (uint32_t)SL_NAME;
    const int64_t boff = lanes_ok ? (SHORT_TB ? (int64_t)FT.pat_cp_off[P] : FT.pat_boff[P]) : 0;
    nver += has ? 1u : 0u;
    // stage the names: 16 dwords per candidate
    for (uint32_t i0 = 0; i0 < nc * (SL_NAME / 4); i0 += WAVE) {
        const uint32_t idx = i0 + (uint32_t)lane;
        const int k = (int)(idx / (SL_NAME / 4));
        const uint32_t w = idx % (SL_NAME / 4);
        const uint32_t blo = (uint32_t)__shfl((int)(uint32_t)boff, k & 63, WAVE);
        const uint32_t bhi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)boff >> 32), k & 63, WAVE);
        const int32_t km = __shfl((int)m, k & 63, WAVE);
        if (idx < nc * (SL_NAME / 4) && 4 * w < (uint32_t)km)
            ((uint32_t *)names)[idx] = ld_u32_unaligned(SHORT_TB ? FT.pat_tbytes : FT.pat_bytes, (int64_t)(((uint64_t)bhi << 32) | blo) + 4 * w);
    }
    // jobs per candidate: m - n + 1 full windows, the prefixes, the suffixes, the swapped run (m == n)
    const uint32_t nj = lanes_ok ? (m - n + 3 + (m == n ? 1u : 0u)) : 0u;
    int J = 0;
    const int ex = wave_excl_scan((int)nj, &J);
    uint32_t okm = 0, exm = 0;   // per candidate lane: decided / equal to the field
    wave_sync();
    for (int g0 = 0; g0 < J; g0 += WAVE) {
        const int g = g0 + lane;
        int owner = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
            const int c = owner + step;
            const int e = __shfl(ex, c & 63, WAVE);
            if (c < WAVE && e <= g) owner = c;
        }
        const int exo = __shfl(ex, owner, WAVE);
        const uint32_t om = (uint32_t)__shfl((int)m, owner, WAVE);
        bool ok = false, exact = false;
        if (g < J) {
            const uint32_t j = (uint32_t)(g - exo);
            const uint8_t *nm = names + owner * SL_NAME;
            const uint32_t nfull = om - n + 1;
            uint64_t V = ~0ull;
            ++nwin;
            if (j < nfull) {
                // full window name[j, j + n)
                for (uint32_t s = 0; s < n; ++s) {
                    const uint64_t U = V & pm[nm[j + s]];
                    V = (V + U) | (V - U);
                }
                const uint32_t L = (uint32_t)__popcll(~V & needle);
                ok = 20u * (n - L) < n;
                exact = om == n && L == n;
                if (!ok && om == n && j == 0) {   // swapped: needle = name, windows = prefixes of the field
                    for (uint32_t i = 1; i < n && !ok; ++i) ok = passes((uint32_t)__popcll(~V & low_mask(i)), om, i);
                }
            } else if (j == nfull) {
                // prefixes name[:i], i < n
                for (uint32_t i = 1; i < n && !ok; ++i) {
                    const uint64_t U = V & pm[nm[i - 1]];
                    V = (V + U) | (V - U);
                    ok = passes((uint32_t)__popcll(~V & needle), n, i);
                }
            } else {
                // suffixes name[m-k:] (j == nfull + 1) or the swapped run over the whole reversed name:
                // reversed needle
                const bool sw = j == nfull + 2;
                const uint32_t steps = sw ? om : n - 1;
                for (uint32_t t = 1; t <= steps && !ok; ++t) {
                    const uint64_t R = __builtin_bitreverse64(pm[nm[om - t]]) >> (64 - n);
                    const uint64_t U = V & R;
                    V = (V + U) | (V - U);
                    if (!sw) ok = passes((uint32_t)__popcll(~V & needle), n, t);
                }
                if (sw) {   // needle = name, windows = suffixes of the field: field[i:] ~ fr[:n-i]
                    for (uint32_t t = 1; t < n && !ok; ++t) ok = passes((uint32_t)__popcll(~V & low_mask(t)), om, t);
                }
            }
        }
        // fold the job results into the owners' bits
        const uint64_t okb = __ballot(ok), exb = __ballot(exact);
        uint64_t rest = okb | exb;
        while (rest) {
            const int l = __builtin_ctzll(rest);
            rest &= rest - 1;
            const int ow = __shfl(owner, l, WAVE);
            if (lane == ow) {
                if ((okb >> l) & 1ull) okm = 1u;
                if ((exb >> l) & 1ull) exm = 1u;
            }
        }
    }
    // candidates lanes cannot take (non-ASCII names), wave-serially
    uint64_t slow = __ballot(has && !lanes_ok);
    while (slow) {
        const int l = __builtin_ctzll(slow);
        slow &= slow - 1;
        const uint32_t lP = (uint32_t)__builtin_amdgcn_readlane((int)P, l);
        const uint32_t lm = (uint32_t)__builtin_amdgcn_readlane((int)m, l);
        const uint32_t nmr = (lane < (int)lm) ? FT.pat_tcps[FT.pat_cp_off[lP] + lane] : 0xFFFFFFFDu;
        bool exact = false;
        const bool dec = fk_short_decide(fc, n, nmr, lm, &exact, nwin_w);
        if (lane == l) {
            okm = dec ? 1u : 0u;
            exm = exact ? 1u : 0u;
        }
    }
    const bool dec = has && okm != 0;
    const bool rx = dec && FT.pat_rxk[P] == RXK_REGEX;
    emit_hits(O, GS, dec && !rx, F.doc, P, exm ? 0u : KW_NOPOS, F.field);
    xq_push(X, rx, F.doc, P, F.field);
    wave_sync();
}

__device__ void fk_short_lanes(const FastTables &FT, const DevScratch &GS, const FieldCtx &F, OutCtx &O, XPush &X,
                               uint64_t *pm, uint8_t *names, uint32_t *cand, unsigned long long &nver,
                               unsigned long long &nwin, unsigned long long &nver_w, unsigned long long &nwin_w)
{
    const int lane = lane_id();
    const uint32_t n = F.n;
    if (n <= (uint32_t)SHORT_EXACT_MAX) {
        fk_short_field(FT, FT.pat_tcps, GS, F, O, nver_w, nwin_w, [&](uint32_t P) { xq_push(X, lane == 0, F.doc, P, F.field); });
        return;
    }
    // the field's signature first (bit c & 63 of every byte): most fields have no candidate name at all
    const uint32_t fc = (lane < (int)n) ? (uint32_t)F.arena[F.fb + lane] : 0xFFFFFFFCu;
    uint64_t fsig = (lane < (int)n) ? 1ull << (fc & 63u) : 0ull;
    // and its bigram signature: a window alignment within partial_ratio's bound d <= allow keeps all but
    // 2d of the field's bigram positions in the name (3d when the name is the needle, m == n), so a name
    // missing more than 3 * allow of the field's bigram bits has no window
    uint64_t fb0 = 0, fb1 = 0;
    {
        const uint32_t nx = (uint32_t)__shfl((int)fc, (lane + 1) & (WAVE - 1), WAVE);
        if (SHORT_BG && lane + 1 < (int)n) {
            const uint32_t h = fk_bg_bit(fc, nx);
            (h & 64u ? fb1 : fb0) = 1ull << (h & 63u);
        }
    }
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        fsig |= __shfl_xor(fsig, d, WAVE);
        fb0 |= __shfl_xor(fb0, d, WAVE);
        fb1 |= __shfl_xor(fb1, d, WAVE);
    }
    bool have_pm = false;
    auto run = [&](uint32_t nc) {
        if (!have_pm) {   // the field's match vectors for every ASCII byte (LDS pm), built for the first candidates
            const uint64_t needle = low_mask(n);
            uint64_t FW[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                uint64_t x = 0;
                if (8 * w < (int)n) x = load8(F.arena, F.fb + 8 * w);
                const int rem = (int)n - 8 * w;
                if (rem < 8) x &= rem <= 0 ? 0ull : ((1ull << (8 * rem)) - 1);
                FW[w] = x;
            }
#pragma unroll
            for (int q = 0; q < (SHORT_TB ? 4 : 2); ++q) pm[lane + 64 * q] = lv_match(FW, (uint32_t)lane + 64u * q, needle);
            have_pm = true;
            wave_sync();
        }
        fk_short_run(FT, GS, F, O, X, pm, names, cand, nc, fc, nver, nwin, nwin_w);
    };
    wave_sync();
    const uint32_t allow = (2 * n - 1) / 20;
    const uint32_t count = (uint32_t)FT.f_count_ge[n];
    uint32_t nc = 0;
    constexpr int SIG_U = 8;
    for (uint32_t c00 = 0; c00 < count; c00 += SIG_U * WAVE) {
        uint64_t nsig[SIG_U];
        ulonglong2 nbs[SIG_U];
#pragma unroll
        for (int u = 0; u < SIG_U; ++u) {
            const uint32_t idx = c00 + (uint32_t)(u * WAVE + lane);
            nsig[u] = idx < count ? FT.pat_sig[FT.f_first + idx] : ~0ull;
            nbs[u] = (SHORT_BG && idx < count) ? ((const ulonglong2 *)FT.pat_bsig)[FT.f_first + idx] : make_ulonglong2(~0ull, ~0ull);
        }
#pragma unroll
        for (int u = 0; u < SIG_U; ++u) {
            const uint32_t c0 = c00 + (uint32_t)(u * WAVE);
            const bool cnd = c0 + (uint32_t)lane < count && (uint32_t)__popcll(fsig & ~nsig[u]) <= allow &&
                             (uint32_t)(__popcll(fb0 & ~nbs[u].x) + __popcll(fb1 & ~nbs[u].y)) <= 3 * allow;
            const uint64_t cm = __ballot(cnd);
            if (!cm) continue;
            if (nc + (uint32_t)__popcll(cm) > (uint32_t)WAVE) {
                run(nc);
                nc = 0;
            }
            if (cnd) cand[nc + mbcnt(cm)] = (uint32_t)FT.f_first + c0 + (uint32_t)lane;
            nc += (uint32_t)__popcll(cm);
            wave_sync();
        }
    }
    if (nc) run(nc);
}

// Short fields: the field is the needle, the fuzzy names at least as long as the field the haystacks.
__global__ __launch_bounds__(RK_BLOCK, SK_MINW) void kw_short_kernel(FastTables FT, DevTables T, const uint8_t *__restrict__ arena,
                                                            const int64_t *__restrict__ off, int n_regions, int G,
                                                            FastScratch S, DevScratch GS)
{
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t gw = (int64_t)blockIdx.x * RK_WAVES + wib;   // G waves per region
    const int64_t t = gw / G;
    const uint32_t sub = (uint32_t)(gw % G);
    if (t >= n_regions) return;
    (void)T;
    __shared__ uint64_t pm_all[RK_WAVES * (SHORT_TB ? 256 : 128)];
    __shared__ uint32_t names_all[RK_WAVES * WAVE * SL_NAME / 4];
    __shared__ uint32_t cand_all[RK_WAVES * WAVE];
    uint64_t *pm = pm_all + wib * (SHORT_TB ? 256 : 128);
    uint8_t *names = (uint8_t *)(names_all + wib * WAVE * SL_NAME / 4);
    uint32_t *cand = cand_all + wib * WAVE;
    OutCtx O = tout_region(S, t);
    XPush X = xq_region(S, t);
    unsigned long long nver = 0, nwin = 0, nver_w = 0, nwin_w = 0;
    FieldCtx F;
    const uint32_t ns = min(S.scnt[t], S.scap);
    const uint4 *sq = S.sq + (size_t)t * S.scap;
    for (uint32_t k = sub; k < ns; k += (uint32_t)G) {
        const uint4 tk = sq[k];
        fk_field_ctx(F, arena, S, (uint32_t)__builtin_amdgcn_readfirstlane((int)tk.x),
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)tk.y));
        if (FK_SHORT_LANES)
        {
            if (SHORT_COUNT && lane == 0) {   // developer aid: short tasks by length class (stats 21..24)
                atomicAdd(&S.stats[21 + (F.n <= (uint32_t)SHORT_EXACT_MAX ? 0 : F.n < 40u ? 1 : 2)], 1ull);
                atomicAdd(&S.stats[24], (unsigned long long)FT.f_count_ge[F.n]);
            }
            fk_short_lanes(FT, GS, F, O, X, pm, names, cand, nver, nwin, nver_w, nwin_w);
        }
        else
            fk_short_field(FT, FT.pat_tcps, GS, F, O, nver_w, nwin_w,
                           [&](uint32_t P) { xq_push(X, lane == 0, F.doc, P, F.field); });
    }
    task_stats(S, wave_sum64(nver) + nver_w, wave_sum64(nwin) + nwin_w, 0, 0, 0, 0);
}

// re.finditer positions of a decided regex name P with an RXM use (program length L) in an ASCII field: the
// leftmost non-overlapping of the field's RXM items of P (the probe's exact matches of the program).  Returns
// false, having emitted nothing, when P has more than 64 of them (the field search takes it).
// (b, n: the field's items in S.items)
__device__ bool fk_rx_items(const FastScratch &S, const DevScratch &GS, const FieldCtx &F, OutCtx &O, uint32_t P,
                            uint32_t L, uint32_t b, uint32_t n)
{
    const int lane = lane_id();
    uint64_t key = ~0ull;   // (position, lane slot) of this lane's match
    uint32_t k = 0;
    for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
        const uint32_t i = i0 + (uint32_t)lane;
        const uint64_t it = i < n ? S.items[b + i] : 0ull;
        const bool mine = i < n && it_pat(it) == P && it_kind(it) == FU_RXM && it_use(it) != IT_USE_MASK;
        const uint64_t bm = __ballot(mine);
        const uint32_t c = (uint32_t)__popcll(bm);
        if (k + c > (uint32_t)WAVE) return false;
        // gather this round's matches into lanes k .. k + c
        const uint32_t pos = it_pos(it);
        uint64_t rest = bm;
        for (uint32_t q = 0; q < c; ++q) {
            const int l = __builtin_ctzll(rest);
            rest &= rest - 1;
            const uint32_t pq = (uint32_t)__shfl((int)pos, l, WAVE);
            if ((uint32_t)lane == k + q) key = pq;
        }
        k += c;
    }
    key = wave_sort_reg(key);
    // greedy leftmost non-overlapping selection (matches are L code points long)
    uint64_t keep = 0;
    uint32_t last_end = 0;
    for (uint32_t q = 0; q < k; ++q) {
        const uint32_t pq = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, (int)q);
        if (q == 0 || pq >= last_end) { keep |= 1ull << q; last_end = pq + L; }
    }
    const bool kq = (keep >> lane) & 1ull;
    emit_hits(O, GS, kq, F.doc, P, (uint32_t)key, F.field);
    emit_hits(O, GS, k == 0 && lane == 0, F.doc, P, KW_NOPOS, F.field);
    return true;
}

// Regex-class names decided (by the scan or the task kernels): re.finditer positions or `name: []`.  phase 0:
// every task of the region; 1: the tasks the epilogue queued (xmark, beside the verify / short kernels); 2: the
// ones the verify / short kernels queued after them.
__global__ __launch_bounds__(RK_BLOCK, RX_MINW) void kw_rx_task_kernel(FastTables FT, DevTables T, const uint8_t *__restrict__ arena,
                                                              const int64_t *__restrict__ off, int n_regions, int G,
                                                              FastScratch S, DevScratch GS, int phase)
{
    __shared__ uint64_t rxtab_all[RK_WAVES * 256];
    __shared__ uint4 rxtxt_all[RK_WAVES * (RX_TXT / 16)];
    __shared__ uint4 rxpre_all[RK_WAVES * WAVE * 5];   // per wave: the next 64 tasks' records, fetched lane-parallel
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t gw = (int64_t)blockIdx.x * RK_WAVES + wib;   // G waves per region
    const int64_t t = gw / G;
    const uint32_t sub = (uint32_t)(gw % G);
    if (t >= n_regions) return;
    uint64_t *rxtab = rxtab_all + wib * 256;
    uint8_t *txt = (uint8_t *)(rxtxt_all + wib * (RX_TXT / 16));
    uint4 *pre = rxpre_all + wib * WAVE * 5;
    OutCtx O = tout_region(S, t);
    unsigned long long nrx = 0, nrx_bt = 0, nrx_rounds = 0;
    FieldCtx F;
    const uint32_t xall = min(S.xcnt[t], S.xcap), xm = phase ? min(S.xmark[t], xall) : 0u;
    const uint32_t x0 = phase == 2 ? xm : 0u, nx = (phase == 1 ? xm : xall) - x0;
    const uint4 *xq = S.xq + (size_t)t * S.xcap + x0;
    for (uint32_t k0 = sub; k0 < nx; k0 += (uint32_t)G * WAVE) {
        // lane j fetches task k0 + j G and its document's view record, flags and item range (one dependent
        // round for all 64 instead of two per task)
        {
            const uint32_t k = k0 + (uint32_t)lane * (uint32_t)G;
            const bool has = k < nx;
            const uint4 tk = has ? xq[k] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t doc = tk.x, P = tk.y >> 1, f = tk.y & 1u;
            const uint4 v = has ? S.vrec[doc] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t L = has ? FT.pat_rxl[P] : 0u;
            const uint32_t na = has ? (S.dflags[doc] & (f ? DH_NA1 : DH_NA0)) : 0u;
            const uint2 h = has ? S.hdr[doc] : make_uint2(0u, 0u), nc = has ? S.ncnt[doc] : make_uint2(0u, 0u);
            const int32_t rr = has ? FT.rxf_idx[P] : -1;   // the field search's program, when it comes to that
            RxfParams prm = {0u, 0u, 0u, 0ull};
            if (rr >= 0) prm = rxf_params(FT, (uint32_t)rr);
            wave_sync();
            pre[5 * lane] = v;
            pre[5 * lane + 1] = make_uint4(doc, tk.y, na ? 0u : L, h.x + (f ? nc.x : 0u));
            pre[5 * lane + 2] = make_uint4(f ? nc.y : nc.x, (uint32_t)rr, prm.L, 0u);
            pre[5 * lane + 3] = make_uint4(prm.eb, prm.ee, (uint32_t)prm.anym, (uint32_t)(prm.anym >> 32));
            wave_sync();
        }
        const uint32_t nj = min((uint32_t)WAVE, (nx - k0 + (uint32_t)G - 1) / (uint32_t)G);
        for (uint32_t j = 0; j < nj; ++j) {
            const uint4 vv = pre[5 * j], q = pre[5 * j + 1];
            const uint4 v = make_uint4((uint32_t)__builtin_amdgcn_readfirstlane((int)vv.x),
                                       (uint32_t)__builtin_amdgcn_readfirstlane((int)vv.y),
                                       (uint32_t)__builtin_amdgcn_readfirstlane((int)vv.z),
                                       (uint32_t)__builtin_amdgcn_readfirstlane((int)vv.w));
            const uint32_t y = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.y);
            const uint32_t f = y & 1u, P = y >> 1;
            const uint32_t L = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.z);
            F.tx = (v.y >> 31) != 0;
            F.arena = F.tx ? S.tarena : arena;
            F.fb = (int64_t)(((uint64_t)(v.y & 0x7FFFFFFFu) << 32) | v.x) + (f ? (int64_t)v.z : 0);
            F.n = f ? v.w : v.z;
            F.fe = F.fb + F.n;
            F.ascii = true;
            F.cps = nullptr;
            F.blkcnt = nullptr;
            F.doc = (uint32_t)__builtin_amdgcn_readfirstlane((int)q.x);
            F.field = f;
            // a name with an RXM use in an ASCII field: the probe's RXM items are its matches, no search
            if (L && fk_rx_items(S, GS, F, O, P, L, (uint32_t)__builtin_amdgcn_readfirstlane((int)q.w),
                                 (uint32_t)__builtin_amdgcn_readfirstlane((int)pre[5 * j + 2].x)))
                continue;
#if defined(RX_TIMING_SKIP) && RX_TIMING_SKIP <= 2   // (timing variants only: 1 skips the backtracking
                                                      // searches, 2 every search, 3 the shift-and loops, 4 all
                                                      // but the mask table load)
            if (RX_TIMING_SKIP == 2 || FT.rxf_idx[P] < 0) continue;
#endif
            const uint4 q2 = pre[5 * j + 2], q3 = pre[5 * j + 3];
            RxfParams prm;
            prm.L = (uint32_t)__builtin_amdgcn_readfirstlane((int)q2.z);
            prm.eb = (uint32_t)__builtin_amdgcn_readfirstlane((int)q3.x);
            prm.ee = (uint32_t)__builtin_amdgcn_readfirstlane((int)q3.y);
            prm.anym = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)q3.z) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)q3.w) << 32);
            fk_regex_pre(FT, T, GS, F, O, P, (int32_t)__builtin_amdgcn_readfirstlane((int)q2.y), prm, rxtab, txt, nrx,
                         nrx_bt, nrx_rounds);
        }
    }
    task_stats(S, 0, 0, 0, nrx, nrx_bt, nrx_rounds);
}


// ---------------------------------------------------------------- kernel 2: resolve
#ifndef RK_NOINLINE   // 1: the resolve kernels call fk_resolve_field (fewer spills, a call frame); 0: inlined
#define RK_NOINLINE 0
#endif
template <uint32_t ICAP>
__device__ __attribute__((noinline)) int fk_resolve_field_call(const FastTables &FT, const DevTables &T, const DevScratch &GS,
                                                               FieldCtx &F, OutCtx &O, uint64_t *items_lds,
                                                               uint32_t *icnt_f, uint32_t *dflag, uint32_t *cps,
                                                               uint32_t *blkcnt, uint64_t *rxtab, RxQueue &RQ,
                                                               bool maybe_nonascii, bool edge, unsigned long long &nver,
                                                               unsigned long long &nwin, unsigned long long &nedge,
                                                               unsigned long long *tacc)
{
    return fk_resolve_field<ICAP>(FT, T, GS, F, O, items_lds, icnt_f, dflag, cps, blkcnt, rxtab, RQ, maybe_nonascii, edge,
                                  nver, nwin, nedge, tacc);
}

struct RkCounters {   // (per wave: the uniform ones in 32 bits, fewer scalar registers to spill)
    unsigned long long nver, nwin, nedge;
    uint32_t ndefer, ndef_cp, ndef_items, nres, nrx, nrx_bt, nrx_rounds;
};

// Resolve one document with a non-ASCII field (n0 / n1 items from hx in the probe's item list, header
// flags hy), field by field through an ICAP-item LDS buffer; on a field the fast path cannot finish, the
// document's records and regex tasks are rolled back and it goes to the generic kernel.
template <uint32_t ICAP>
__device__ __forceinline__ void rk_resolve_doc(const FastTables &FT, const DevTables &T, const DevScratch &GS,
                                               const FastScratch &S, const uint8_t *__restrict__ arena,
                                               const int64_t *__restrict__ off, int64_t d, uint32_t hx, uint32_t n0,
                                               uint32_t n1, uint32_t hy, uint64_t *items, uint32_t *icnt, uint32_t *cps,
                                               uint32_t *blkcnt, uint64_t *rxtab, OutCtx &O, RxQueue &RQ, RkCounters &C,
                                               unsigned long long *tacc)
{
    const int lane = lane_id();
    const int64_t t0 = off[2 * d], t1 = off[2 * d + 1], t2 = off[2 * d + 2];
    const uint32_t nf[2] = {n0, n1};
    const uint32_t out_mark = O.n, rq_mark = RQ.n;
    bool defer = false;
    ++C.nres;
    for (int f = 0; f < 2 && !defer; ++f) {
        const uint32_t N = nf[f];
        const uint64_t *src = S.items + hx + (f ? nf[0] : 0u);
        for (uint32_t i = (uint32_t)lane; i < N; i += WAVE) items[i] = src[i];
        if (lane == 0) { icnt[0] = N; icnt[1] = 0; }
        wave_sync();
        FieldCtx F;
        F.arena = arena;
        F.fb = f ? t1 : t0;
        F.fe = f ? t2 : t1;
        F.cps = cps;
        F.blkcnt = blkcnt;
        F.doc = (uint32_t)d;
        F.field = (uint32_t)f;
        F.ascii = true;
        F.n = 0;
        const bool na = (hy & (f ? DH_NA1 : DH_NA0)) != 0;
        const bool edge = (hy & (f ? DH_EDGE1 : DH_EDGE0)) != 0;
        int rs = 0;
        if constexpr (RK_NOINLINE)
            rs = fk_resolve_field_call<ICAP>(FT, T, GS, F, O, items, &icnt[0], &icnt[1], cps, blkcnt, rxtab, RQ, na,
                                             edge, C.nver, C.nwin, C.nedge, tacc);
        else
            rs = fk_resolve_field<ICAP>(FT, T, GS, F, O, items, &icnt[0], &icnt[1], cps, blkcnt, rxtab, RQ, na, edge,
                                        C.nver, C.nwin, C.nedge, tacc);
        if (rs) {
            defer = true;
            if (rs == 1) ++C.ndef_cp;
            else ++C.ndef_items;
        }
        wave_sync();
    }
    if (defer) {
        O.n = out_mark;   // drop this doc's partial records; the generic kernel redoes it
        RQ.n = rq_mark;
        ++C.ndefer;
        if (lane == 0) {
            const uint32_t i = atomicAdd(S.defer_cnt, 1u);
            if (i < S.defer_cap) S.defer_list[i] = (uint32_t)d;
            else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
        }
    }
}

// After a resolve wave's last document: its queued regex-position tasks, its record count, the statistics.
__device__ __forceinline__ void rk_wave_tail(const FastTables &FT, const DevTables &T, const DevScratch &GS,
                                             const FastScratch &S, const uint8_t *__restrict__ arena,
                                             const int64_t *__restrict__ off, int64_t wave, uint32_t *cps,
                                             uint32_t *blkcnt, uint64_t *rxtab, OutCtx &O, RxQueue &RQ, RkCounters &C,
                                             unsigned long long *tacc, unsigned long long tall0)
{
    const int lane = lane_id();
    wave_sync_global();
    if (RQ.n > RQ.cap && lane == 0) atomicMax(&GS.status[2], RQ.n);   // the queue size a rescan needs
    const uint32_t n_rx = RQ.n < RQ.cap ? RQ.n : RQ.cap;
    FK_T0(trx0);
    uint32_t dec_d = 0xFFFFFFFFu, dec_f = 0;   // the field whose code points cps holds (tasks come in doc order)
    for (uint32_t t = 0; t < n_rx; ++t) {
        const uint4 tk = RQ.q[t];
        const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk.x);
        const uint32_t fy = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk.y);
        const uint32_t P = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk.z);
        FieldCtx F;
        F.arena = arena;
        F.field = fy & 1u;
        F.fb = off[2 * (int64_t)d + F.field];
        F.fe = off[2 * (int64_t)d + F.field + 1];
        F.ascii = (fy & 2u) != 0;
        F.n = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk.w);
        F.cps = cps;
        F.blkcnt = blkcnt;
        F.doc = d;
        if (!F.ascii && (d != dec_d || F.field != dec_f)) {
            decode_field_fast(arena, F.fb, F.fe, cps, blkcnt, FK_CP_CAP);
            dec_d = d;
            dec_f = F.field;
        }
        const int32_t r = FT.rxf_idx[P];
        ++C.nrx;
        C.nrx_bt += r < 0;
        C.nrx_rounds += r >= 0 ? (F.n + 2047) / 2048 : 0;
        const uint32_t cnt = r >= 0 ? fk_rx_fixed_positions(FT, GS, F, O, P, (uint32_t)r, rxf_params(FT, (uint32_t)r), rxtab, RQ.txt)
                                    : rx_positions(T, GS, F, O, P);
        if (cnt == 0) emit_hits(O, GS, lane == 0, d, P, KW_NOPOS, F.field);
    }
    FK_TACC(tacc[4], trx0);
    FK_TACC(tacc[5], tall0);
    if (FK_TIMING && lane == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(&S.stats[21 + i], tacc[i]);
    if (lane == 0) S.out_cnt[wave] = O.n;
    unsigned long long v = C.nver, w = C.nwin;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) {
        v += __shfl_xor(v, dd, WAVE);
        w += __shfl_xor(w, dd, WAVE);
    }
    if (lane == 0 && (C.nres | C.ndefer)) {   // (a wave without documents adds nothing: no same-address atomics)
        atomicAdd(&S.stats[2], w / WAVE);
        atomicAdd(&S.stats[3], v / WAVE);
        atomicAdd(&S.stats[4], (unsigned long long)C.ndefer);
        atomicAdd(&S.stats[5], (unsigned long long)C.ndef_items);
        atomicAdd(&S.stats[6], (unsigned long long)C.ndef_cp);
        atomicAdd(&S.stats[7], C.nedge);
        atomicAdd(&S.stats[9], (unsigned long long)C.nres);
        atomicAdd(&S.stats[10], (unsigned long long)C.nrx);
        atomicAdd(&S.stats[11], (unsigned long long)C.nrx_bt);
        atomicAdd(&S.stats[12], (unsigned long long)C.nrx_rounds);
    }
}



__global__ __launch_bounds__(RK_BLOCK, RK_OCC) void kw_resolve_kernel(FastTables FT, DevTables T,
                                                              const uint8_t *__restrict__ arena,
                                                              const int64_t *__restrict__ off, int64_t n_docs,
                                                              FastScratch S, DevScratch GS)
{
    __shared__ uint64_t items_all[RK_WAVES * FK_ITEMS_MAX];
    __shared__ uint64_t rxtab_all[RK_WAVES * 128];
    __shared__ uint4 rxtxt_all[RK_WAVES * (RX_TXT / 16)];
    __shared__ uint32_t cnt_all[RK_WAVES * 4];
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t wave = (int64_t)blockIdx.x * RK_WAVES + wib;
    const int64_t n_waves = (int64_t)gridDim.x * RK_WAVES;
    uint64_t *items = items_all + wib * FK_ITEMS_MAX;
    uint64_t *rxtab = rxtab_all + wib * 128;
    uint32_t *icnt = cnt_all + wib * 4;
    uint32_t *cps = S.cps + (size_t)wave * FK_CP_CAP;
    uint32_t *blkcnt = S.cpbase + (size_t)wave * (CP_CAP / 16 + 2);
    OutCtx O;
    O.shared = nullptr;
    O.out = S.out + (size_t)wave * S.out_cap;
    O.cap = S.out_cap;
    O.n = 0;
    RxQueue RQ;
    RQ.q = S.rx_tasks + (size_t)wave * S.rx_cap;
    RQ.cap = S.rx_cap;
    RQ.n = 0;
    RQ.txt = (uint8_t *)(rxtxt_all + wib * (RX_TXT / 16));
    RkCounters C = {};
    unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0};   // FK_TIMING: decode, edge, items, short, regex, all
    FK_T0(tall0);

    const int64_t n_list = (int64_t)min(*S.res_cnt, S.defer_cap);
    // chunks of up to 64 documents per wave, fewer when the list is short (each wave finishes its chunk's
    // documents one after another: a short list spread over every wave)
    const int64_t ch = max((int64_t)1, min((int64_t)WAVE, (n_list + n_waves - 1) / n_waves));
    for (int64_t c0 = wave * ch; c0 < n_list; c0 += n_waves * ch) {
        // lane = document: this kernel owns the documents the epilogue left to it (res_list, DH_RESOLVE: a
        // non-ASCII field its transcoded view cannot take); it runs beside the task kernels, after the epilogue
        const int64_t dl = (lane < ch && c0 + lane < n_list) ? (int64_t)S.res_list[c0 + lane] : n_docs;
        uint2 hl = make_uint2(0u, 0u);
        bool dfr = false, dfr_items = false;
        {
            const uint32_t fl = dl < n_docs ? S.dflags[dl] : 0u;
            if (fl & DH_RESOLVE) {   // (the epilogue's non-ASCII documents its transcoded view cannot take)
                const uint2 nc = S.ncnt[dl];
                const uint32_t ibeg = S.hdr[dl].x;
                const int64_t t0 = off[2 * dl], t1 = off[2 * dl + 1], t2 = off[2 * dl + 2];
                uint32_t flags = fl & (DH_NA0 | DH_NA1);
                // edge prefilter: the first / last eight bytes of each field against the global bitmaps
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int f = k >> 1;
                    const int64_t fb = f ? t1 : t0, fe = f ? t2 : t1;
                    if (fe - fb < (int64_t)EDGE_MIN_M + 1) continue;
                    const int64_t a = (k & 1) ? fe - 8 : fb;
                    const uint64_t key8 = (uint64_t)ld_u32_unaligned(arena, a) | ((uint64_t)ld_u32_unaligned(arena, a + 4) << 32);
                    const uint32_t idx = fk_edge_index(key8);
                    if ((((k & 1) ? FT.edge_suf : FT.edge_pre)[idx >> 5] >> (idx & 31u)) & 1u) flags |= f ? DH_EDGE1 : DH_EDGE0;
                }
                const bool over = nc.x > (uint32_t)FK_ITEMS0 || nc.y > (uint32_t)FK_ITEMS1;
                bool defer = (fl & DH_DEFER) || t1 - t0 > MAX_FIELD_BYTES || t2 - t1 > MAX_FIELD_BYTES;
                bool big = false;
                if (!defer && over) {
                    // more items than this kernel's LDS holds: the big-document resolve (list at the tail end
                    // of big_list, the epilogue's big documents fill it from the head), beyond it the generic kernel
                    if (nc.x <= (uint32_t)FK_BIG0 && nc.y <= (uint32_t)FK_BIG0) {
                        const uint32_t bi = atomicAdd(&S.big_cnt[1], 1u);
                        if (bi < S.defer_cap) {
                            S.big_list[S.defer_cap - 1 - bi] = (uint32_t)dl;
                            big = true;
                        }
                    }
                    defer = !big;
                }
                const int64_t l0 = t1 - t0, l1 = t2 - t1;
                const bool s0 = l0 <= MAXM || ((flags & DH_NA0) && l0 <= 4 * MAXM);
                const bool s1 = l1 <= MAXM || ((flags & DH_NA1) && l1 <= 4 * MAXM);
                const bool need = !big && ((nc.x + nc.y) > 0 || (flags & (DH_EDGE0 | DH_EDGE1)) || s0 || s1);
                hl.x = ibeg;
                // (a big document's header keeps the flags only: its kernel reads the counts from ncnt)
                hl.y = defer ? (DH_DEFER | flags) : big ? flags : (nc.x | (nc.y << DH_N1_SHIFT) | flags | (need ? DH_NEED : 0u));
                S.hdr[dl] = hl;
                if (defer) {
                    const uint32_t i = atomicAdd(S.defer_cnt, 1u);
                    if (i < S.defer_cap) S.defer_list[i] = (uint32_t)dl;
                    else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
                }
                dfr = defer;
                dfr_items = defer && over;
            }
        }
        C.ndefer += (uint32_t)__popcll(__ballot(dfr));
        C.ndef_items += (uint32_t)__popcll(__ballot(dfr_items));
        uint64_t todo = __ballot((hl.y & DH_NEED) != 0 && (hl.y & DH_DEFER) == 0);
        while (todo) {
            const int l = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int64_t d = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)dl, l);
            const uint32_t hx = (uint32_t)__shfl((int)hl.x, l, WAVE);
            const uint32_t hy = (uint32_t)__shfl((int)hl.y, l, WAVE);
            rk_resolve_doc<FK_ITEMS_MAX>(FT, T, GS, S, arena, off, d, hx, hy & 1023u, (hy >> DH_N1_SHIFT) & 127u, hy,
                                         items, icnt, cps, blkcnt, rxtab, O, RQ, C, tacc);
        }
    }
    rk_wave_tail(FT, T, GS, S, arena, off, wave, cps, blkcnt, rxtab, O, RQ, C, tacc, tall0);
}

// ---------------------------------------------------------------- kernel 2b: big non-ASCII documents
// The documents with a non-ASCII field and more items than kw_resolve_kernel's LDS holds (FK_ITEMS0 in the
// text, FK_ITEMS1 in the title), up to FK_BIG0 per field: the same per-document resolve with one wave per
// workgroup and a 32 KiB item buffer.  Launched after kw_resolve_kernel on its stream, at most one
// workgroup per resolve wave: wave w continues resolve wave w's hit region and regex queue.
__global__ __launch_bounds__(WAVE) void kw_resolve_big_kernel(FastTables FT, DevTables T, const uint8_t *__restrict__ arena,
                                                            const int64_t *__restrict__ off, FastScratch S, DevScratch GS)
{
    __shared__ uint64_t items[FK_BIG0];
    __shared__ uint64_t rxtab[128];
    __shared__ uint4 rxtxt[RX_TXT / 16];
    __shared__ uint32_t icnt[4];
    const int64_t wave = blockIdx.x;
    const uint32_t nbig = min(S.big_cnt[1], S.defer_cap);
    if (wave >= (int64_t)nbig) return;
    uint32_t *cps = S.cps + (size_t)wave * FK_CP_CAP;
    uint32_t *blkcnt = S.cpbase + (size_t)wave * (CP_CAP / 16 + 2);
    OutCtx O;
    O.shared = nullptr;
    O.out = S.out + (size_t)wave * S.out_cap;
    O.cap = S.out_cap;
    O.n = S.out_cnt[wave];
    RxQueue RQ;
    RQ.q = S.rx_tasks + (size_t)wave * S.rx_cap;
    RQ.cap = S.rx_cap;
    RQ.n = 0;
    RQ.txt = (uint8_t *)rxtxt;
    RkCounters C = {};
    unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0};
    FK_T0(tall0);
    for (int64_t i = wave; i < (int64_t)nbig; i += gridDim.x) {
        const uint32_t d = S.big_list[S.defer_cap - 1 - i];   // (the list's tail end: see kw_resolve_kernel)
        const uint2 h = S.hdr[d];
        const uint2 nc = S.ncnt[d];
        rk_resolve_doc<FK_BIG0>(FT, T, GS, S, arena, off, d, h.x, nc.x, nc.y, h.y, items, icnt, cps, blkcnt, rxtab, O,
                                RQ, C, tacc);
    }
    rk_wave_tail(FT, T, GS, S, arena, off, wave, cps, blkcnt, rxtab, O, RQ, C, tacc, tall0);
    if (wave == 0 && lane_id() == 0) atomicAdd(&S.stats[16], (unsigned long long)nbig);
}
}  // namespace kw
