// The fast path's byte scan as three kernels (gfx950).  Included after kwmatch_fast_kernel.hpp, whose
// probe, epilogue and field helpers it reuses.
//
//   kw_filter_kernel  a wave per 32-document group (grid-stride): the LDS filters over every byte position; the
//                     stage-2 survivors ("candidates", 4 bytes: position in the document << 8 | document
//                     in its group << 3 | key lengths to probe, after a header record per group) go to the
//                     wave's region in HBM in document and position order, with the document's flags (non-ASCII fields, edge prefilter, field
//                     too long) in its header.  132 KiB of LDS: one 16-wave workgroup per CU.
//   kw_probe_kernel   one wave per filter region: the region's candidates 64 at a time, whatever document
//                     they belong to (a document averages ~13 candidates, so per-document batches left most
//                     lanes idle): anchor hash probe, head compare, then the (candidate, use) pairs spread
//                     over the lanes to compare spans and test \b.  The batch's verified uses ("items") are
//                     appended to a wave-wide LDS pool (ballot ranks, any candidate may own hundreds of
//                     them: a 50k-name KB has pieces shared by many names) and scattered to HBM grouped by
//                     candidate, so a document's items are contiguous, the text's before the title's; the
//                     header gets the first item's index, the per-field counts are added up in ncnt.
//   kw_epi_kernel     one wave per document: all-ASCII documents are finished by the epilogue
//                     (fk_scan_epilogue: sort, emit, queue the verify / short / regex tasks), the others get
//                     their header for the resolve kernel; documents with more items than a wave's LDS
//                     holds are finished after the workgroup's loop with the whole workgroup's LDS (epi_big_doc;
//                     up to EK_BIGQ, the rest: kw_resolve_big_kernel), oversize ones go to the generic kernel.
//
// Reference: the per-article x per-name loop of match_keywords.py:159-180 (see kwmatch_fast.hpp for the
// anchors and filters).
#pragma once
#include "kwmatch_fast_kernel.hpp"

namespace kw {

#ifndef FS_WAVES_CFG
#define FS_WAVES_CFG 16
#endif
#ifndef FS_MINW
#define FS_MINW 1
#endif
#ifndef FS_EQ_TRIGGER
#define FS_EQ_TRIGGER 32   // queued entries that start a stage-2 round: a round then takes ~2 tiles of survivors
                           // while their bytes are still in L2 (64: filter reads 4.03 GB a launch, 48: 3.59, 32: 3.08
                           // for 1.103 / 1.111 / 1.112 ms; 24: 1.145 ms, 16: 1.238 ms)
#endif
#ifndef FS_AHEAD
#define FS_AHEAD 3       // 1 KiB tiles each filter wave keeps in flight
#endif

constexpr int FS_WAVES = FS_WAVES_CFG;   // waves per filter workgroup
constexpr int FS_BLOCK = FS_WAVES * WAVE;
constexpr int PK_WAVES = 4;              // waves per probe workgroup
constexpr int PK_BLOCK = PK_WAVES * WAVE;
#ifndef PK_POOL_CFG
#define PK_POOL_CFG 768   // (with PK_MINW 5: 5 probe waves per SIMD; 1024 / 4: 6.15 vs 5.97 ms per step)
#endif
constexpr int PK_POOL = PK_POOL_CFG;     // items one batch of 64 candidates may stage (more: their documents defer)
#ifndef FK_TX
#define FK_TX 1     // 0: every document with a non-ASCII field goes to the resolve kernel
#endif
#ifndef EK_MINW
#define EK_MINW 4   // 128 VGPRs, no spill (5 waves per SIMD spills 96 B per lane: epilogue 2.08 vs 1.98 ms)
#endif
#ifndef PK_MINW
#define PK_MINW 5   // <= 102 VGPRs: the probe and the transcoding kernel beside it share the CUs better
#endif
constexpr int EK_WAVES = 8;              // waves per epilogue workgroup
constexpr int EK_BIGQ = 64;              // big documents one epilogue workgroup finishes itself (more: resolve)
constexpr int EK_BLOCK = EK_WAVES * WAVE;

constexpr int FG_DOCS = 32;              // documents per filter group (one flat byte range; 5 bits of a candidate)
#ifndef EF_TX_FLAT
#define EF_TX_FLAT 1   // kw_epi_flat_kernel<true> batches the transcoded documents too (KBs without PI_TXUNSAFE names)
#endif

struct __attribute__((aligned(16))) FilterLds {
    uint32_t s1[FK_S1_WORDS];
    uint32_t p2[FK_P2_WORDS];
    uint32_t l2[FK_L2_WORDS];
    uint32_t t3[FK_T3_WORDS];
    uint32_t b2[FK_B2_WORDS];
    uint32_t dstart[FS_WAVES][FG_DOCS + 1];   // group-relative document starts (+ the group end)
    uint32_t dtitle[FS_WAVES][FG_DOCS];       // group-relative title starts
    uint2 sent[FS_WAVES][2 * WAVE];           // stage 2: the queue of entries {group-relative byte of the lane's
                                              // position 0, transposed survivor mask} (a ring)
    uint32_t spos[FS_WAVES][WAVE];            // a round's survivors' group-relative positions
};

// the group document holding group-relative byte r (dstart[0] = 0 <= r < dstart[nd])
__device__ __forceinline__ uint32_t fg_doc(const uint32_t *dstart, uint32_t nd, uint32_t r)
{
    uint32_t lo = 0, n = nd;
    while (n > 1) {
        const uint32_t h = n >> 1;
        if (dstart[lo + h] <= r) lo += h;
        n -= h;
    }
    return lo;
}

// pair-table bit index: the low 16 bits of a 24-bit product equal fk_b2_index's (key2 * 40503) & 0xFFFF.  As
// inline asm: left to itself the compiler sees that only the low 16 bits are used and emits a quarter-rate
// v_mul_lo_u32 (twice: once for the word, once for the bit)
__device__ __forceinline__ uint32_t fk_b2_mul(uint32_t key)
{
    uint32_t r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(40503u), "v"(key));
    return r;
}

// Stage-1 masks use the transposed bit order of a lane's 16 positions: position j = 4 q + r (q = its word, r =
// its byte) is bit q + 8 r, the order in which the pair box's per-byte flags of the four words combine with
// one shift each.
__device__ __forceinline__ constexpr uint32_t fk_tbit(int j) { return (uint32_t)((j >> 2) + 8 * (j & 3)); }
__device__ __forceinline__ uint32_t fk_tpos(uint32_t b) { return ((b & 7u) << 2) + (b >> 3); }
// position order of a transposed mask: the bytes' nibbles packed (row r = byte, column q), then a 4 x 4 bit
// transpose by two delta swaps
__device__ __forceinline__ uint32_t fk_untranspose(uint32_t t)
{
    uint32_t x = (t & 0xFu) | ((t >> 4) & 0xF0u) | ((t >> 8) & 0xF00u) | ((t >> 12) & 0xF000u);
    uint32_t d = (x ^ (x >> 3)) & 0x0A0Au;
    x ^= d ^ (d << 3);
    d = (x ^ (x >> 6)) & 0x00CCu;
    x ^= d ^ (d << 6);
    return x;
}
__device__ __forceinline__ uint32_t fk_transpose16(uint32_t v)
{
    uint32_t t = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) t |= ((v >> j) & 1u) << fk_tbit(j);
    return t;
}

// the pair box's byte flags of a word: bit 7 of byte i set iff byte i is in the box's range {A, B, N}
__device__ __forceinline__ uint32_t fk_in_box(uint32_t x, uint32_t A, uint32_t B, uint32_t N)
{
    const uint32_t t = x & 0x7F7F7F7Fu;
    return (((t + A) & ~(t + B) & ~x) | (x & N)) & 0x80808080u;
}

// Stage 1 of one lane's 16 bytes W[0..3] (+ W[4]): `hit` = positions where an anchor of >= 4 bytes may start
// (its first four bytes' bit in the 4-gram table; also the fuzzy 3-byte anchors' 4-grams), `gate` = positions
// whose first two bytes lie in the pair box of the other 2-3 byte anchors (SWAR, no lookup; SH = 2: one box
// for both bytes, the byte flags of each word computed once; SH = 3: two ranges below 0x80); transposed bit order (fk_tbit).  Per position:
// one v_mad_u32_u24 (fk_s1_hash), the address, the lookup, v_bfe_u32 and v_lshl_or_b32.
template <int SH>
__device__ __forceinline__ void fk_stage1(const FastTables &FT, const FilterLds &L, const uint32_t (&W)[5],
                                          uint32_t &hit, uint32_t &gate)
{
    uint32_t k[17];
#pragma unroll
    for (int j = 0; j < 16; ++j) k[j] = (j & 3) ? __builtin_amdgcn_alignbyte(W[(j >> 2) + 1], W[j >> 2], j & 3) : W[j >> 2];
    k[16] = W[4];
    uint32_t hh[16], sw[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        hh[j] = __umul24(k[j], FK_S1_M1) + __umul24(k[j + 1], FK_S1_M2);
        sw[j] = lds_word_at(L.s1, (hh[j] >> 16) & (4u * FK_S1_WORDS - 4u));
    }
    uint32_t g = 0;
    if (SH == 1) {
        uint32_t f0[4], f1[5];
#pragma unroll
        for (int q = 0; q < 4; ++q) f0[q] = fk_in_box(W[q], FT.gate[0], FT.gate[1], FT.gate[2]);
#pragma unroll
        for (int q = 0; q < 5; ++q) f1[q] = fk_in_box(W[q], FT.gate[3], FT.gate[4], FT.gate[5]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t pr = f0[q] & __builtin_amdgcn_alignbyte(f1[q + 1], f1[q], 1);   // byte i: b[i], b[i+1]
            g |= pr >> (7 - q);
        }
    } else if (SH == 3) {
        // both ranges below 0x80 (no N term): a byte >= 0x80 may be flagged too (a superset; the exact pair
        // table decides in stage 2), so each flag is two additions and one v_bitop3_b32
        uint32_t t[5], f1[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) t[q] = W[q] & 0x7F7F7F7Fu;
#pragma unroll
        for (int q = 0; q < 5; ++q) f1[q] = (t[q] + FT.gate[3]) & ~(t[q] + FT.gate[4]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t f0 = (t[q] + FT.gate[0]) & ~(t[q] + FT.gate[1]);
            const uint32_t pr = f0 & __builtin_amdgcn_alignbyte(f1[q + 1], f1[q], 1) & 0x80808080u;
            g |= pr >> (7 - q);
        }
    } else if (SH == 2) {
        uint32_t f[5];
#pragma unroll
        for (int q = 0; q < 5; ++q) f[q] = fk_in_box(W[q], FT.gate[0], FT.gate[1], FT.gate[2]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t pr = f[q] & __builtin_amdgcn_alignbyte(f[q + 1], f[q], 1);
            g |= pr >> (7 - q);
        }
    }
    uint32_t h = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t b = __builtin_amdgcn_ubfe(sw[j], hh[j], 1);
        h |= b << fk_tbit(j);
    }
    hit = h;
    gate = g;
}

// ---------------------------------------------------------------- kernel 1: the filters
// A wave takes groups of FG_DOCS consecutive documents and streams each group's bytes as one flat range
// (1 KiB tiles, 16 bytes per lane, the next tiles' loads in flight): no per-document tile shapes or
// set-up.  Keys that run over a field or document end are kept (a superset): the probe checks every
// anchor against its field.  Non-ASCII bytes mark their field in dflags (rare: an LDS lookup of the
// document, one atomic per field).
template <int SH>
__device__ __forceinline__ void fk_filter_groups(const FastTables &FT, FilterLds &L, const uint8_t *__restrict__ arena,
                                                 const int64_t *__restrict__ off, int64_t n_docs, const FastScratch &S,
                                                 int64_t region, int64_t g_lo, int64_t g_hi, int wib, uint32_t &ncand,
                                                 uint32_t &ncand2, uint32_t &ccur)
{
    const int lane = lane_id();
    const uint32_t *l2 = L.l2, *t3 = L.t3, *b2 = L.b2;
    uint32_t *dstart = L.dstart[wib], *dtitle = L.dtitle[wib];
    uint32_t *spos = L.spos[wib];
    uint32_t *cand = S.cand + (size_t)region * S.cand_cap;
    const uint32_t ccap = S.cand_cap;
    const uint32_t t3on = FT.has_t3 ? 1u : 0u;
    for (int64_t g = g_lo; g < g_hi; ++g) {
        const int64_t d0 = g * FG_DOCS;
        const int nd = (int)(n_docs - d0 < FG_DOCS ? n_docs - d0 : FG_DOCS);
        const int64_t o0 = lane <= nd ? off[2 * (d0 + lane)] : 0;
        const int64_t o1 = lane < nd ? off[2 * (d0 + lane) + 1] : 0;
        const int64_t gb = rdlane64(o0, 0), ge = rdlane64(o0, nd);
        if (ge - gb > 0x7FFFFFFFll) {   // group-relative positions are 32-bit: such groups go to the generic kernel
            if (lane < nd) atomicOr(&S.dflags[d0 + lane], DH_DEFER);
            continue;
        }
        if (ge <= gb) continue;   // every field of the group is empty
        wave_sync();
        if (lane <= nd) dstart[lane] = (uint32_t)(o0 - gb);
        if (lane < nd) dtitle[lane] = (uint32_t)(o1 - gb);
        wave_sync();
        // byte offsets below are 32-bit, from the group's first 16-byte block gbase (groups are < 2^31 bytes):
        // the loads take the SGPR base and a VGPR offset, no 64-bit address arithmetic per tile
        const uint8_t *gbase = arena + (gb & ~(int64_t)15);
        const uint32_t g0 = (uint32_t)(gb & 15), gl = (uint32_t)(ge - (gb & ~(int64_t)15));
        uint32_t blk = 0;   // the tile's offset from gbase
        uint32_t kdoc = 0;   // document of the current stage-2 round's first survivor (candidate emission)
        bool ghdr = true;    // the group's header record is not written yet
        // FS_AHEAD tiles in flight per wave, each in its own registers (the loop is unrolled by FS_AHEAD, so no
        // register copy waits for a load).  Loads are unconditional: an address past the group's last
        // 16-byte block is clamped to it (the arena is padded; such lanes' positions are masked).  A tile
        // comes with the word after it (lane 63's fifth word).
        const uint32_t glast = (gl - 1u) & ~15u;
        auto load = [&](uint4 &v, uint32_t &w, uint32_t tb) {
            const uint32_t a = tb + 16u * (uint32_t)lane, e = tb + 1024u;
            v = *(const uint4 *)(gbase + (a < glast ? a : glast));
            w = *(const uint32_t *)(gbase + (e < glast ? e : glast));
        };
        // Stage 2, one round: the queue's first n (<= 64) survivors, lane = survivor, in position order; the
        // three second filters (every key length's: a superset of what the stage-1 family asked for, the short
        // keys behind the exact pair table); the final survivors ("candidates") ranked by ballot and written
        // with their document
        // (r: the lane's survivor position, lanes < n)
        // (key: the 4-byte key at the position, loaded when the round was formed; see round())
        auto round_at = [&](uint32_t n, uint32_t r, uint32_t key) {
            const bool act = (uint32_t)lane < n;
            const uint32_t b4 = (uint32_t)lds_bit(l2, fk_l2_index(key));
            const uint32_t pr = (uint32_t)lds_bit(L.p2, fk_b2_index(key));
            const uint32_t b3 = pr & t3on & (uint32_t)lds_bit(t3, fk_t3_index(key));
            const uint32_t bb = pr & (uint32_t)lds_bit(b2, fk_b2h_index(key));
            const uint32_t fl = b4 | (b3 << 1) | (bb << 2);
            {
                const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)r);   // the round's first position
                while (dstart[kdoc + 1] <= r0) ++kdoc;
            }
            bool keep = act && fl != 0u;
            uint32_t k = kdoc, pd = 0;
            if (keep) {
                while (dstart[k + 1] <= r) ++k;
                pd = r - dstart[k];
                keep = pd < (1u << 24);   // (a longer document has a field over 8 MiB: the generic kernel's)
            }
            const uint64_t pm = __ballot(keep);
            if (pm) {
                // the group's header record precedes its first candidate (fl = 0: the group index)
                if (ghdr) {
                    if (lane == 0 && ccur < ccap) cand[ccur] = (uint32_t)g << 3;
                    ++ccur;
                    ghdr = false;
                }
                const uint32_t kk = ccur + mbcnt(pm);
                if (keep && kk < ccap) cand[kk] = (pd << 8) | (k << 3) | fl;
            }
            const uint32_t np = (uint32_t)__popcll(pm);
            ccur += np;
            ncand2 += (lane == 0) ? np : 0u;
        };
        uint2 *sent = L.sent[wib];
        uint32_t eh = 0, en = 0;   // the entry ring's head and length (wave-uniform)
        // the round formed last: its survivors' keys are in flight while the next tiles' stage 1 runs (the
        // re-read of bytes streamed a few tiles earlier often misses L2), it finishes when the next round forms
        uint32_t qn = 0, qr = 0, qx0 = 0, qx1 = 0;
        // one round: lane = entry, the ring's first E entries whose survivors add up to <= 64 (E >= 1: an entry
        // holds <= 16); each expands its survivors in position order into spos at its rank, then lane = survivor
        auto round = [&]() {
            wave_sync();
            const bool ein = (uint32_t)lane < en;
            const uint2 ent = ein ? sent[(eh + (uint32_t)lane) & (2u * WAVE - 1u)] : make_uint2(0u, 0u);
            const int c = __popc(ent.y);
            int tot;
            const int ex = wave_excl_scan_dpp(c, &tot);
            const uint64_t tm = __ballot(ein && ex + c <= WAVE);
            const int E = __popcll(tm);
            if ((tm >> lane) & 1ull) {
                uint32_t m = fk_untranspose(ent.y);
                uint32_t o = (uint32_t)ex;
                while (m) {
                    spos[o++] = ent.x + (uint32_t)(__ffs(m) - 1);
                    m &= m - 1u;
                }
            }
            const uint32_t n = (uint32_t)__shfl(ex + c, E - 1, WAVE);
            eh = (eh + (uint32_t)E) & (2u * WAVE - 1u);
            en -= (uint32_t)E;
            wave_sync();
            const uint32_t r = spos[lane];
            wave_sync();
            // the key's two aligned words (joined when the round finishes: no wait for them here)
            uint32_t x0 = 0, x1 = 0;
#if defined(FS_TIMING_SKIP) && FS_TIMING_SKIP == 2   // (traffic calibration only, results void: no key re-read)
            x0 = r * 0x9E3779B1u;
#else
            if ((uint32_t)lane < n) {
                const int64_t a0 = (gb + (int64_t)r) & ~(int64_t)3;
                x0 = *(const uint32_t *)(arena + a0);
                x1 = *(const uint32_t *)(arena + a0 + 4);
            }
#endif
            if (qn) round_at(qn, qr, __builtin_amdgcn_alignbyte(qx1, qx0, (uint32_t)(gb + qr) & 3u));
            qn = n;
            qr = r;
            qx0 = x0;
            qx1 = x1;
        };
        auto tile = [&](const uint4 &v, uint32_t w4, uint32_t tb) {
            const uint32_t lp = tb + 16u * (uint32_t)lane;
            uint32_t W[5];
            W[0] = v.x;
            W[1] = v.y;
            W[2] = v.z;
            W[3] = v.w;
            {
                const uint32_t nx = (uint32_t)__shfl_down((int)v.x, 1, WAVE);
                W[4] = lane == WAVE - 1 ? w4 : nx;
            }
            uint32_t valid = 0xFFFFu;
            if (tb < g0 || tb + 1024u > gl) {   // (uniform: only a group's first and last tiles)
                const int32_t rlo = (int32_t)(g0 - lp), rhi = (int32_t)(gl - lp);
                const int jlo = rlo <= 0 ? 0 : (rlo >= 16 ? 16 : rlo);
                const int jhi = rhi <= 0 ? 0 : (rhi >= 16 ? 16 : rhi);
                valid = (jhi > jlo) ? (((1u << jhi) - 1u) & ~((1u << jlo) - 1u)) : 0u;
            }
            const uint32_t rel = lp - g0;   // group-relative byte of this lane's position 0 (wraps below the
                                            // group start: only valid positions are used)
            if ((W[0] | W[1] | W[2] | W[3]) & 0x80808080u) {
                uint32_t hb = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t x = (W[k] >> 7) & 0x01010101u;
                    hb |= ((x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u)) << (4 * k);
                }
                hb &= valid;
                while (hb) {   // one atomic per (document, field) the lane's non-ASCII bytes fall in
                    const uint32_t r = rel + (uint32_t)(__ffs(hb) - 1);
                    const uint32_t k = fg_doc(dstart, (uint32_t)nd, r);
                    const uint32_t tb2 = dtitle[k];
                    const bool title = r >= tb2;
                    atomicOr(&S.dflags[d0 + k], title ? DH_NA1 : DH_NA0);
                    const uint32_t fend = title ? dstart[k + 1] : tb2;   // group-relative end of that field
                    const int64_t skip = (int64_t)fend - (int64_t)(int32_t)rel;
                    hb &= skip >= 16 ? 0u : ~((1u << (uint32_t)skip) - 1u);
                }
            }
            uint32_t hit, gate;
            fk_stage1<SH>(FT, L, W, hit, gate);
            const uint32_t tvalid = valid == 0xFFFFu ? 0x0F0F0F0Fu : fk_transpose16(valid);
            const uint32_t sm = (hit | gate) & tvalid;
            ncand += (uint32_t)__popc(sm);
            // the lanes with survivors join the entry ring in lane (= position) order: no per-survivor work here
            // (the per-lane survivor loop, the DPP scan and the untranspose were ~60 VALU a tile); stage 2 runs
            // whenever 64 entries (>= 64 survivors) are queued (en < 64 before: the ring of 128 never overflows)
            const uint64_t em = __ballot(sm != 0u);
            if (!em) return;
            if (sm != 0u) sent[(eh + en + mbcnt(em)) & (2u * WAVE - 1u)] = make_uint2(rel, sm);
            en += (uint32_t)__popcll(em);
#if defined(FS_TIMING_SKIP) && FS_TIMING_SKIP == 1   // (traffic calibration only, results void: no stage 2)
            en = 0;
#endif
            while (en >= (uint32_t)FS_EQ_TRIGGER) round();
        };
        uint4 v[FS_AHEAD];
        uint32_t w[FS_AHEAD];
#pragma unroll
        for (int k = 0; k < FS_AHEAD; ++k) {   // in tile order: the first tile's wait then leaves the others in flight
            load(v[k], w[k], blk + 1024 * k);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (bool more = true; more;) {
#pragma unroll
            for (int k = 0; k < FS_AHEAD; ++k) {   // (unrolled: each tile in flight keeps its own registers)
                if (blk >= gl) { more = false; break; }
                tile(v[k], w[k], blk);
                load(v[k], w[k], blk + 1024 * FS_AHEAD);
                blk += 1024;
            }
        }
        while (en) round();   // the group's last survivors
        if (qn) round_at(qn, qr, __builtin_amdgcn_alignbyte(qx1, qx0, (uint32_t)(gb + qr) & 3u));
    }
}

__global__ __launch_bounds__(FS_BLOCK, FS_MINW) void kw_filter_kernel(FastTables FT, const uint8_t *__restrict__ arena,
                                                             const int64_t *__restrict__ off, int64_t n_docs,
                                                             FastScratch S)
{
    __shared__ FilterLds L;
    {
        const uint4 *src = (const uint4 *)FT.s1;
        uint4 *dst = (uint4 *)L.s1;
        for (int i = threadIdx.x; i < FK_S1_WORDS / 4; i += FS_BLOCK) dst[i] = src[i];
    }
    for (int i = threadIdx.x; i < FK_P2_WORDS; i += FS_BLOCK) L.p2[i] = FT.p2[i];
    for (int i = threadIdx.x; i < FK_L2_WORDS; i += FS_BLOCK) L.l2[i] = FT.l2[i];
    for (int i = threadIdx.x; i < FK_T3_WORDS; i += FS_BLOCK) L.t3[i] = FT.t3[i];
    for (int i = threadIdx.x; i < FK_B2_WORDS; i += FS_BLOCK) L.b2[i] = FT.b2[i];
    __syncthreads();
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t wave = (int64_t)blockIdx.x * FS_WAVES + wib;
    const int64_t n_waves = (int64_t)gridDim.x * FS_WAVES;
    uint32_t ncand = 0, ncand2 = 0;
    // work units ("chunks", one candidate region each): S.chunk_groups consecutive 32-document groups; a wave
    // claims the next chunk from a counter when it finishes one (S.dyn; else grid-stride), so the waves end
    // together, and the probe's regions stay small and even
    const int64_t n_groups = (n_docs + FG_DOCS - 1) / FG_DOCS;
    const int64_t K = S.chunk_groups;
    const int64_t n_chunks = (n_groups + K - 1) / K;
    const bool gate_one = FT.gate[0] == FT.gate[3] && FT.gate[1] == FT.gate[4] && FT.gate[2] == FT.gate[5];
    for (int64_t c = S.dyn ? fk_next_group(S.gnext, true, 0, 0) : wave; c < n_chunks;
         c = fk_next_group(S.gnext, S.dyn, c, n_waves)) {
        uint32_t ccur = 0;
        const int64_t g_lo = c * K, g_hi = g_lo + K < n_groups ? g_lo + K : n_groups;
        if (!FT.has_short)
            fk_filter_groups<0>(FT, L, arena, off, n_docs, S, c, g_lo, g_hi, wib, ncand, ncand2, ccur);
        else if (gate_one)
            fk_filter_groups<2>(FT, L, arena, off, n_docs, S, c, g_lo, g_hi, wib, ncand, ncand2, ccur);
        else if (FT.gate[2] == 0u && FT.gate[5] == 0u)
            fk_filter_groups<3>(FT, L, arena, off, n_docs, S, c, g_lo, g_hi, wib, ncand, ncand2, ccur);
        else
            fk_filter_groups<1>(FT, L, arena, off, n_docs, S, c, g_lo, g_hi, wib, ncand, ncand2, ccur);
        if (lane == 0) {
            S.ccnt[c] = ccur;
            if (ccur > S.cand_cap) {
                atomicOr(&S.status[0], ST_CAND_OVERFLOW);
                atomicMax(&S.cmax[0], ccur);
            }
        }
    }
    unsigned long long c1 = ncand;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) c1 += __shfl_xor(c1, dd, WAVE);
    if (lane == 0) {
        atomicAdd(&S.stats[0], c1);
        atomicAdd(&S.stats[8], (unsigned long long)ncand2);
    }
}

// An RXM use's program string (L <= 64 bytes, '.' atoms as wildcard bits wm) against the text at s0: every
// literal byte equal, every wildcard byte other than '\n' (re's '.'; non-ASCII fields never use these items).
__device__ __forceinline__ bool rxm_match(const uint8_t *__restrict__ a, int64_t s0, const uint8_t *__restrict__ prog,
                                          uint32_t L, uint64_t wm)
{
    for (uint32_t k = 0; k < L; k += 8) {
        const uint64_t t = load8(a, s0 + k), p = load8(prog, k);
        const uint32_t nb = L - k < 8 ? L - k : 8;
        const uint64_t valid = nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1);
        uint64_t wb = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) wb |= ((wm >> (k + j)) & 1ull) ? (0xFFull << (8 * j)) : 0ull;
        wb &= valid;
        if (((t ^ p) & valid & ~wb) != 0 || (zb64(t ^ 0x0A0A0A0A0A0A0A0Aull) & wb) != 0) return false;
    }
    return true;
}

// ---------------------------------------------------------------- kernel 2: the anchor probe
__global__ __launch_bounds__(PK_BLOCK, PK_MINW) void kw_probe_kernel(FastTables FT, DevTables T, const uint8_t *__restrict__ arena,
                                                            const int64_t *__restrict__ off, int32_t n_regions,
                                                            FastScratch S)
{
    __shared__ uint64_t pool_all[PK_WAVES * PK_POOL];
    __shared__ uint8_t pown_all[PK_WAVES * PK_POOL];
    __shared__ uint32_t scnt_all[PK_WAVES * WAVE];
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    uint64_t *pool = pool_all + wib * PK_POOL;
    uint8_t *pown = pown_all + wib * PK_POOL;
    uint32_t *scnt = scnt_all + wib * WAVE;
    uint32_t nanchor = 0;
    // regions (the filter's work units, a few groups each) claimed from a counter: the waves end together
    const int64_t n_waves = (int64_t)gridDim.x * PK_WAVES;
    for (int64_t region = S.dyn ? fk_next_group(S.gnext + 1, true, 0, 0) : (int64_t)blockIdx.x * PK_WAVES + wib;
         region < n_regions; region = fk_next_group(S.gnext + 1, S.dyn, region, n_waves)) {
    const uint32_t *cand = S.cand + (size_t)region * S.cand_cap;
    int32_t cur_group = -1;                 // group of the region's last header record so far (wave-uniform)
    const uint32_t nc = min(S.ccnt[region], S.cand_cap);
    uint64_t *items = S.items + (size_t)region * S.item_cap;
    const uint32_t icap = S.item_cap;
    const uint32_t ibase = (uint32_t)((size_t)region * S.item_cap);
    uint32_t icur = 0;                      // items of this region (wave-uniform)
    uint32_t last_doc = 0xFFFFFFFFu;        // document of the region's last item so far
    scnt[lane] = 0;
    for (uint32_t c0 = 0; c0 < nc; c0 += WAVE) {
        const bool inb = c0 + (uint32_t)lane < nc;
        const uint32_t e = inb ? cand[c0 + lane] : 0u;
        // records: a group header (low 3 bits 0: the group index above them) before the group's candidates
        // (position in the document << 8 | document in the group << 3 | key lengths to probe)
        const bool is_hdr = inb && (e & 7u) == 0u;
        int32_t grp = is_hdr ? (int32_t)(e >> 3) : -1;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {   // the last header at or before each lane (groups ascend)
            const int32_t y = __shfl_up(grp, d, WAVE);
            if (lane >= d) grp = max(grp, y);
        }
        grp = max(grp, cur_group);
        cur_group = __shfl(grp, WAVE - 1, WAVE);
        const bool inr = inb && !is_hdr;
        const uint32_t doc = (uint32_t)grp * FG_DOCS + ((e >> 3) & (FG_DOCS - 1));
        const int64_t t0 = inr ? off[2 * (int64_t)doc] : 0;
        const int64_t t1 = inr ? off[2 * (int64_t)doc + 1] : 0;
        const int64_t t2 = inr ? off[2 * (int64_t)doc + 2] : 0;
        // fields beyond MAX_FIELD_BYTES (item positions are 23-bit) are the generic kernel's
        const bool valid = inr && t1 - t0 <= MAX_FIELD_BYTES && t2 - t1 <= MAX_FIELD_BYTES;
        const int32_t l1 = (int32_t)(t1 - t0), l2 = (int32_t)(t2 - t0);
        const int32_t pr = (int32_t)(e >> 8);
        const int f = pr < l1 ? 0 : 1;
        const int32_t fbr = f ? l1 : 0, fer = f ? l2 : l1;
        const int64_t p = t0 + pr;
        const uint64_t h8 = valid ? ld_u64_unaligned(arena, p) : 0ull;
        // hash lookups of the lane's key lengths 4, 3, 2 (try bits 0, 1, 2), all in flight together
        uint32_t rb[3], re[3];
        {
            uint4 hs[3];
            uint64_t key[3];
            uint32_t slot[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int Lk = 4 - i;
                const bool want = valid && ((e >> i) & 1u) && pr + Lk <= fer;
                key[i] = ((uint64_t)Lk << 32) | (h8 & ((1ull << (8 * Lk)) - 1));
                slot[i] = fk_ht_slot(key[i], FT.ht_mask);
                hs[i] = want ? FT.ht4[slot[i]] : make_uint4(~0u, ~0u, 0u, 0u);
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                rb[i] = re[i] = 0;
                for (;;) {
                    const uint64_t kk = (uint64_t)hs[i].x | ((uint64_t)hs[i].y << 32);
                    if (kk == key[i]) { rb[i] = hs[i].z; re[i] = hs[i].z + hs[i].w; break; }
                    if (kk == ~0ull) break;
                    slot[i] = (slot[i] + 1) & FT.ht_mask;
                    hs[i] = FT.ht4[slot[i]];
                }
            }
        }
        uint32_t tcur = rb[0], tend = re[0], b1 = rb[1], e1 = re[1], b2 = rb[2], e2 = re[2];
#if defined(PK_TIMING_SKIP) && PK_TIMING_SKIP == 2
        bool more = false;
        if (__ballot(valid && (tcur | b1 | b2) == 0xFFFFFFFFu)) nanchor += 1;   // (keeps the lookups)
#else
        bool more = valid;
#endif
        uint32_t pn = 0;                    // items in the pool (wave-uniform)
        while (__ballot(more)) {
            // stage A: up to two matching anchors of this lane's candidate
            uint32_t ub = 0, uc = 0, ub1 = 0, uc1 = 0, nm = 0;
            while (more && nm < 2) {
                if (tcur < tend) {
                    const uint4 ar0 = FT.arec[tcur];
                    const bool two = tcur + 1 < tend;
                    const uint4 ar1 = two ? FT.arec[tcur + 1] : make_uint4(0u, 0u, 0u, 0u);
                    auto take = [&](const uint4 &ar) {
                        const uint32_t alen = ar.w & 0xFFu;
                        if (pr + (int32_t)alen > fer) return;
                        const uint64_t m8 = alen >= 8 ? ~0ull : ((1ull << (8 * alen)) - 1);
                        if ((h8 ^ ((uint64_t)ar.x | ((uint64_t)ar.y << 32))) & m8) return;
                        ++nanchor;
                        if (nm == 0) { ub = ar.z; uc = ar.w >> 8; }
                        else { ub1 = ar.z; uc1 = ar.w >> 8; }
                        ++nm;
                    };
                    take(ar0);
                    ++tcur;
                    if (two && nm < 2) {
                        take(ar1);
                        ++tcur;
                    }
                    continue;
                }
                if (b1 >= e1 && b2 >= e2) { more = false; break; }
                tcur = b1; tend = e1;
                b1 = b2; e1 = e2;
                b2 = e2 = 0;
            }
            // a lane that took its last anchor records is done (no extra round of the wave for it)
            if (more && tcur >= tend && b1 >= e1 && b2 >= e2) more = false;
            // stage B: (candidate, use) pairs over the lanes
            int total;
            const int ex = wave_excl_scan_dpp((int)(uc + uc1), &total);
#if defined(PK_TIMING_SKIP)   // (timing variants only, results void: 1 no stage B, 2 no stage A or B)
            total = 0;
#endif
            for (int g0 = 0; g0 < total; g0 += WAVE) {
                const int g = g0 + lane;
                bool pass = false;
                uint64_t item = 0;
                int owner = 0;
#pragma unroll
                for (int step = 32; step >= 1; step >>= 1) {
                    const int cnd = owner + step;
                    const int exc = __shfl(ex, cnd & 63, WAVE);
                    if (cnd < WAVE && exc <= g) owner = cnd;
                }
                const int exo = __shfl(ex, owner, WAVE);
                const uint32_t oub = (uint32_t)__shfl((int)ub, owner, WAVE);
                const uint32_t ouc = (uint32_t)__shfl((int)uc, owner, WAVE);
                const uint32_t oub1 = (uint32_t)__shfl((int)ub1, owner, WAVE);
                const uint32_t loc = (uint32_t)(g - exo);
                const uint32_t u = loc < ouc ? oub + loc : oub1 + (loc - ouc);
                const int32_t ppr = __shfl(pr, owner, WAVE);
                const int32_t ofbr = __shfl(fbr, owner, WAVE), ofer = __shfl(fer, owner, WAVE);
                const int64_t ot0 = rdlane64v(t0, owner);
                do {
                if (g >= total) break;
                const uint4 ur = FT.urec[u];
                const uint32_t kind = ur.x & 0xFF, aoff = (ur.x >> 8) & 0xFF;
                const uint32_t sblen = ur.y & 0xFFFF;
                const uint32_t pat = ur.z;
                const int32_t s0r = ppr - (int32_t)aoff;
                if (s0r < ofbr || s0r + (int32_t)sblen > ofer) break;
                const int64_t s0 = ot0 + s0r, fb = ot0 + ofbr, fe2 = ot0 + ofer;
                const uint4 u2 = FT.urec2[u];
                const uint64_t th = load8(arena, s0);
                const uint64_t tt = load8(arena, s0 + (sblen > 8 ? sblen - 8 : 0));
                const uint32_t pi = kind == FU_UPPER ? FT.pat_info[pat] : 0u;
                const bool hasp = kind == FU_UPPER && s0 > fb, hasn = kind == FU_UPPER && s0 + (int64_t)sblen < fe2;
                const uint32_t prevb = hasp ? (uint32_t)arena[s0 - 1] : 0u;
                const uint32_t nextb = hasn ? (uint32_t)arena[s0 + sblen] : 0u;
                const uint32_t hl = sblen < 8 ? sblen : 8;
                const uint64_t hm = hl >= 8 ? ~0ull : ((1ull << (8 * hl)) - 1);
                if (kind == FU_RXM) {
                    // a regex program's match: literal bytes equal, '.' wildcards any byte but '\n'
                    if (!rxm_match(arena, s0, FT.pat_bytes + ur.w, sblen, FT.use_wild[u])) break;
                } else {
                    if ((th ^ ((uint64_t)u2.x | ((uint64_t)u2.y << 32))) & hm) break;
                    if (sblen > 8 && tt != ((uint64_t)u2.z | ((uint64_t)u2.w << 32))) break;
                    if (sblen > 16 && !span_equal(arena, s0 + 8, FT.pat_bytes + ur.w + 8, sblen - 16)) break;
                }
                if (kind == FU_UPPER) {
                    const bool wf = (pi & PI_WORD_FIRST) != 0, wl = (pi & PI_WORD_LAST) != 0;
                    bool wp = false;
                    if (hasp) wp = is_word_cp(T, prevb < 0x80u ? prevb : decode_before(arena, fb, s0));
                    if (wp == wf) break;
                    bool wn = false;
                    if (hasn) {
                        uint32_t ch = nextb;
                        if (nextb >= 0x80u) decode_at(arena, s0 + sblen, fe2, &ch);
                        wn = is_word_cp(T, ch);
                    }
                    if (wn == wl) break;
                }
                item = ((uint64_t)pat << IT_PAT_SHIFT) | ((uint64_t)(uint32_t)(s0r - ofbr) << IT_POS_SHIFT) |
                       ((uint64_t)kind << IT_KIND_SHIFT) | (uint64_t)u;
                pass = true;
                } while (0);
                // append to the pool: rank by ballot, the owner's count by an LDS atomic
                const uint64_t pm = __ballot(pass);
                if (pass) {
                    const uint32_t k = pn + (uint32_t)__builtin_popcountll(pm & ((1ull << lane) - 1));
                    if (k < (uint32_t)PK_POOL) { pool[k] = item; pown[k] = (uint8_t)owner; }
                    atomicAdd(&scnt[owner], 1u);
                }
                pn += (uint32_t)__builtin_popcountll(pm);
            }
            wave_sync();
        }
        // the batch's items grouped by candidate (candidate order; any order within a candidate, the
        // epilogue sorts): lane L's items start at icur + (items of lanes < L)
        const uint32_t nmine = scnt[lane];
        int itotal;
        const int iex = wave_excl_scan_dpp((int)nmine, &itotal);
        // the pool dropped items, or the batch's items do not fit the region (the scan is redone with larger
        // regions, ST_CAND_OVERFLOW, unless S.item_grow is 0): the batch's documents defer, so nothing reads
        // items that were not written
        const bool ovf = pn > (uint32_t)PK_POOL || icur + (uint32_t)itotal > icap;
        const uint64_t withm = __ballot(nmine > 0);
        if (withm) {
            const uint64_t below = (1ull << lane) - 1;
            const uint64_t prevm = withm & below;
            const uint32_t pdoc = (uint32_t)__shfl((int)doc, prevm ? 63 - __builtin_clzll(prevm) : 0, WAVE);
            const uint32_t prev_doc = prevm ? pdoc : last_doc;
            if (nmine > 0) {
                if (doc != prev_doc) S.hdr[doc].x = ibase + icur + (uint32_t)iex;
                atomicAdd(f ? &S.ncnt[doc].y : &S.ncnt[doc].x, nmine);
                if (ovf) atomicOr(&S.dflags[doc], DH_DEFER);
            }
            last_doc = (uint32_t)__shfl((int)doc, 63 - __builtin_clzll(withm), WAVE);
            if (!ovf) {
                scnt[lane] = icur + (uint32_t)iex;   // the next free slot of the lane's items
                wave_sync();
                for (uint32_t j = (uint32_t)lane; j < pn; j += WAVE) {
                    const uint32_t idx = atomicAdd(&scnt[pown[j]], 1u);
                    if (idx < icap) items[idx] = pool[j];
                }
                wave_sync();
            }
        }
        icur += (uint32_t)itotal;
        scnt[lane] = 0;
        wave_sync();
    }
    if (lane == 0 && icur > icap && S.item_grow) {   // (clamped: the deferred documents are the generic kernel's)
        atomicOr(&S.status[0], ST_CAND_OVERFLOW);
        atomicMax(&S.cmax[1], icur);
    }
    wave_sync();
    }
    unsigned long long a = nanchor;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) a += __shfl_xor(a, dd, WAVE);
    if (lane == 0) atomicAdd(&S.stats[1], a);
}

// the edge-prefilter flags of a document: first / last eight bytes of each field (lanes 0..3) against
// the global one-deletion prefix / suffix bitmaps
__device__ __forceinline__ uint32_t fk_edge_flags(const FastTables &FT, const FastDoc &D)
{
    const int lane = lane_id();
    const int f = lane >> 1;
    const int64_t fb = f ? D.t1 : D.t0, fe = f ? D.t2 : D.t1;
    bool e = false;
    if (lane < 4 && fe - fb >= (int64_t)EDGE_MIN_M + 1) {
        const int64_t a = (lane & 1) ? fe - 8 : fb;
        const uint64_t k = (uint64_t)ld_u32_unaligned(D.arena, a) | ((uint64_t)ld_u32_unaligned(D.arena, a + 4) << 32);
        const uint32_t idx = fk_edge_index(k);
        e = (((lane & 1) ? FT.edge_suf : FT.edge_pre)[idx >> 5] >> (idx & 31u)) & 1u;
    }
    const uint64_t em = __ballot(e);
    return ((em & 3ull) ? DH_EDGE0 : 0u) | ((em & 12ull) ? DH_EDGE1 : 0u);
}

// fk_edge_flags with the keys already loaded (lanes 0..3: epi_prefetch)
__device__ __forceinline__ uint32_t fk_edge_flags_key(const FastTables &FT, const FastDoc &D, uint64_t k)
{
    const int lane = lane_id();
    const int f = lane >> 1;
    const int64_t fb = f ? D.t1 : D.t0, fe = f ? D.t2 : D.t1;
    bool e = false;
    if (lane < 4 && fe - fb >= (int64_t)EDGE_MIN_M + 1) {
        const uint32_t idx = fk_edge_index(k);
        e = (((lane & 1) ? FT.edge_suf : FT.edge_pre)[idx >> 5] >> (idx & 31u)) & 1u;
    }
    const uint64_t em = __ballot(e);
    return ((em & 3ull) ? DH_EDGE0 : 0u) | ((em & 12ull) ? DH_EDGE1 : 0u);
}

// ---------------------------------------------------------------- transcoded view of non-ASCII documents
// A document with a non-ASCII field is rewritten to one byte per code point (ASCII as is, the non-ASCII code
// points of the fuzzy names as their markers 0x81..0xFF, any other code point 0x80) in S.tarena by
// kw_tx_kernel (side stream, beside the probe); the epilogue turns its items' byte positions into code point
// positions and finishes it exactly like an all-ASCII document: every comparison the epilogue and the task
// kernels make is then code point against code point (names through pat_tcps, positions are code point
// indices as re.finditer reports them).  Documents the view cannot decide (an item of a PI_TXUNSAFE name,
// more items than the epilogue holds, a non-ASCII field over FK_CP_CAP bytes, no room left) go to the resolve
// kernel (DH_RESOLVE).
//
// Per transcoded document, one tarena allocation (16-byte aligned): the text's then the title's code point
// bytes (tx_bytes), then per non-ASCII field the code points before each 16-byte chunk of the field's arena
// bytes (u16, chunks counted from fb & ~15); vrec[d] = {start lo, start hi | 1 << 31, text cps, title cps}
// (vrec[d].y = ~0: not transcoded).
#ifndef TX_MINW
#define TX_MINW 8   // 64 VGPRs (a 56-byte spill): 0.57 vs 0.60 ms isolated
#endif
constexpr int TX_WAVES = 4;
constexpr int TX_BLOCK = TX_WAVES * WAVE;
constexpr uint32_t TX_NONE = 0xFFFFFFFFu;
constexpr unsigned long long TX_SLAB = 16384;   // bytes of tarena a transcoding wave takes at a time

__device__ __forceinline__ uint64_t tx_bytes(int64_t l0, int64_t l1)
{
    return ((uint64_t)(l0 + l1) + 16ull + 15ull) & ~15ull;   // (+16: unaligned reads past the end)
}
__device__ __forceinline__ uint32_t tx_nchunks(int64_t fb, int64_t fe) { return (uint32_t)((fe - (fb & ~(int64_t)15) + 15) >> 4) + 1u; }

// the marker of code point cp (txk / txv: the 256-entry marker table, staged in LDS)
__device__ __forceinline__ uint32_t tx_marker(const uint32_t *txk, const uint32_t *txv, uint32_t cp)
{
    uint32_t s = (cp * 0x9E3779B1u) >> 24;
    for (int k = 0; k < 256; ++k) {
        const uint32_t kk = txk[s];
        if (kk == cp) return txv[s];
        if (kk == 0xFFFFFFFFu) break;
        s = (s + 1) & 255u;
    }
    return 0x80u;
}

// Field bytes [fb, fe) of the arena -> out[o0, o0 + n) (one byte per code point; out 16-byte aligned); chunk
// (may be null) [k] = code points of the field before its 16-byte chunk k.  stg: the wave's 1040-byte LDS
// staging buffer (each 1 KiB block's output leaves with 16-byte stores).  Returns n.  Whole wave.
__device__ uint32_t tx_field(const uint32_t *txk, const uint32_t *txv, const uint8_t *__restrict__ a, int64_t fb, int64_t fe,
                             uint8_t *__restrict__ out, uint32_t o0, uint16_t *__restrict__ chunk, uint8_t *stg)
{
    const int lane = lane_id();
    const int64_t base = fb & ~(int64_t)15;
    uint32_t count = 0;
    // the next block's loads are issued before this block's work
    auto ld = [&](int64_t b, uint4 &v, uint32_t &w4) {
        const int64_t p = b + 16 * (int64_t)lane;
        v = p < fe ? *(const uint4 *)(a + p) : make_uint4(0u, 0u, 0u, 0u);
        w4 = (lane == WAVE - 1 && b + 1024 < fe) ? *(const uint32_t *)(a + b + 1024) : 0u;
    };
    uint4 vn;
    uint32_t wn;
    ld(base, vn, wn);
    for (int64_t blk = base; blk < fe; blk += 1024) {
        const int64_t lp = blk + 16 * (int64_t)lane;
        const uint4 v = vn;
        const uint32_t w4 = wn;
        if (blk + 1024 < fe) ld(blk + 1024, vn, wn);
        uint32_t W[5];
        W[0] = v.x; W[1] = v.y; W[2] = v.z; W[3] = v.w;
        W[4] = (uint32_t)__shfl_down((int)W[0], 1, WAVE);
        if (lane == WAVE - 1) W[4] = w4;
        const int64_t r0 = fb - lp, r2 = fe - lp;
        const int jlo = r0 <= 0 ? 0 : (r0 >= 16 ? 16 : (int)r0);
        const int jhi = r2 <= 0 ? 0 : (r2 >= 16 ? 16 : (int)r2);
        const uint32_t valid = (jhi > jlo) ? (((1u << jhi) - 1u) & ~((1u << jlo) - 1u)) : 0u;
        // a lane whose 16 bytes are ASCII (most of them: a non-ASCII field has a few multi-byte characters) has
        // every byte a lead byte and copies them with one 16-byte LDS store below
        const bool asc = ((W[0] | W[1] | W[2] | W[3]) & 0x80808080u) == 0u;
        uint32_t lead = 0xFFFFu, high = 0;
        if (!asc) {
            lead = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t b = (W[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                lead |= (uint32_t)((b & 0xC0u) != 0x80u) << j;
                high |= (uint32_t)(b >= 0x80u) << j;
            }
        }
        lead &= valid;
        high &= valid;
        int total;
        const int ex = wave_excl_scan_dpp(__popc(lead), &total);
        if (chunk && lp < fe) chunk[(lp - base) >> 4] = (uint16_t)(count + (uint32_t)ex);
        // the block's output, staged at the output's alignment (stg byte (g0 & 15) + k = output byte g0 + k):
        // lanes without a multi-byte character copy their bytes
        wave_sync();
        const uint32_t g0 = o0 + count, g1 = g0 + (uint32_t)total, sh = g0 & 15u;
        const uint32_t k = (uint32_t)ex + sh;
        // every lead byte's output at its rank among the lane's lead bytes: the ASCII ones unrolled (one
        // predicated store each), then a loop over the lane's few multi-byte characters only (decode, marker)
        const uint32_t hl = lead & high;
        if (asc && valid == 0xFFFFu) {
            *(uint4 *)(stg + k) = v;   // (any byte address: LDS runs in unaligned mode, scripts/probe/lds_unaligned.hip)
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (((lead & ~hl) >> j) & 1u) stg[k + (uint32_t)__popc(lead & ((1u << j) - 1u))] = (uint8_t)(W[j >> 2] >> (8 * (j & 3)));
        }
        for (uint32_t lm = hl; lm; lm &= lm - 1) {
            const int j = __ffs(lm) - 1;
            const uint32_t b0 = (W[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t n = (b0 >= 0xF0u) ? 4u : (b0 >= 0xE0u) ? 3u : 2u;
            uint32_t c = b0 & (0x7Fu >> n);
            for (uint32_t q = 1; q < n; ++q) {
                const int jj = j + (int)q;
                const uint32_t bk = (lp + jj < fe) ? ((W[jj >> 2] >> (8 * (jj & 3))) & 0xFFu) : 0x80u;
                c = (c << 6) | (bk & 0x3Fu);
            }
            stg[k + (uint32_t)__popc(lead & ((1u << j) - 1u))] = (uint8_t)tx_marker(txk, txv, c);
        }
        wave_sync();
        // out[g0, g1): 16-byte stores of aligned staged chunks (ds_read_b128) for the body, byte stores at the
        // two ends
        const uint32_t gb = g0 & ~15u;
        const uint32_t a0 = (g0 + 15u) & ~15u, a1 = g1 & ~15u;
        if (a0 < a1) {
            if ((uint32_t)lane < a0 - g0) out[g0 + lane] = stg[g0 - gb + lane];
            if ((uint32_t)lane < g1 - a1) out[a1 + lane] = stg[a1 - gb + lane];
            for (uint32_t q = a0 + 16u * (uint32_t)lane; q < a1; q += 16u * WAVE)
                *(uint4 *)(out + q) = *(const uint4 *)(stg + (q - gb));
        } else {
            for (uint32_t q = g0 + (uint32_t)lane; q < g1; q += WAVE) out[q] = stg[q - gb];
        }
        count += (uint32_t)total;
    }
    wave_sync();
    return count;
}

// Transcode the documents with a non-ASCII field (the filter's dflags) into the view.  One wave takes 64
// documents at a time (lane = document), then their non-ASCII ones in turn.
__global__ __launch_bounds__(TX_BLOCK, TX_MINW) void kw_tx_kernel(FastTables FT, const uint8_t *__restrict__ arena,
                                                         const int64_t *__restrict__ off, int64_t n_docs, FastScratch S)
{
    __shared__ __attribute__((aligned(16))) uint32_t stg_all[TX_WAVES * (1040 / 4)];   // (16-byte chunks: ds_read_b128)
    __shared__ uint32_t txk[256], txv[256];
    for (int i = threadIdx.x; i < 256; i += TX_BLOCK) {
        txk[i] = FT.tx_key[i];
        txv[i] = FT.tx_val[i];
    }
    __syncthreads();
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t wave = (int64_t)blockIdx.x * TX_WAVES + wib;
    const int64_t n_waves = (int64_t)gridDim.x * TX_WAVES;
    uint8_t *stg = (uint8_t *)(stg_all + wib * (1040 / 4));
    // the view's space: the wave takes TX_SLAB-byte slabs of tarena (one atomic each, not one per document)
    unsigned long long slab = 0, slab_end = 0;
    for (int64_t c0 = wave * WAVE; c0 < n_docs; c0 += n_waves * WAVE) {
        const int64_t dl = c0 + lane;
        const uint32_t fl = dl < n_docs ? S.dflags[dl] : 0u;
        const bool na = (fl & (DH_NA0 | DH_NA1)) != 0;
        // every lane's offsets at once (lane = document)
        const int64_t lt0 = na ? off[2 * dl] : 0, lt1 = na ? off[2 * dl + 1] : 0, lt2 = na ? off[2 * dl + 2] : 0;
        uint64_t todo = __ballot(na);
        while (todo) {
            const int l = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int64_t d = c0 + l;
            const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)fl, l);
            const int64_t t0 = rdlane64(lt0, l), t1 = rdlane64(lt1, l), t2 = rdlane64(lt2, l);
            const int64_t l0 = t1 - t0, l1 = t2 - t1;
            bool ok = !(f & DH_DEFER) && l0 <= MAX_FIELD_BYTES && l1 <= MAX_FIELD_BYTES &&
                      !((f & DH_NA0) && l0 > FK_CP_CAP) && !((f & DH_NA1) && l1 > FK_CP_CAP);
            const uint64_t nb = tx_bytes(l0, l1);
            const uint32_t nc0 = (f & DH_NA0) ? tx_nchunks(t0, t1) : 0u, nc1 = (f & DH_NA1) ? tx_nchunks(t1, t2) : 0u;
            const unsigned long long need = nb + ((2ull * (nc0 + nc1) + 15ull) & ~15ull);
            unsigned long long tb = 0;
            if (ok) {
                if (slab + need > slab_end) {
                    const unsigned long long take = need > TX_SLAB ? need : TX_SLAB;
                    unsigned long long b0 = 0;
                    if (lane == 0) b0 = atomicAdd(S.tx_used, take);
                    b0 = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b0 >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b0);
                    slab = b0;
                    slab_end = b0 + take;
                }
                tb = slab;
                slab += need;
                ok = tb + need <= S.tx_cap;
            }
            if (!ok) {
                if (lane == 0) S.vrec[d] = make_uint4(0u, TX_NONE, 0u, 0u);
                continue;
            }
            uint8_t *out = S.tarena + tb;
            uint16_t *ch = (uint16_t *)(S.tarena + tb + nb);
            const uint32_t n0 = tx_field(txk, txv, arena, t0, t1, out, 0u, (f & DH_NA0) ? ch : nullptr, stg);
            const uint32_t n1 = tx_field(txk, txv, arena, t1, t2, out, n0, (f & DH_NA1) ? ch + nc0 : nullptr, stg);
            if (lane == 0) S.vrec[d] = make_uint4((uint32_t)tb, (uint32_t)(tb >> 32) | 0x80000000u, n0, n1);
        }
    }
}

// code point position of field byte bpos (field [fb, ...) of the arena; chunk from tx_field)
__device__ __forceinline__ uint32_t tx_pos(const uint8_t *__restrict__ a, int64_t fb, const uint16_t *chunk,
                                           uint32_t bpos)
{
    const int64_t base = fb & ~(int64_t)15, p = fb + bpos;
    const int64_t k = (p - base) >> 4, cs = base + 16 * k;
    const uint4 v = *(const uint4 *)(a + cs);
    const uint32_t W[4] = {v.x, v.y, v.z, v.w};
    const int jlo = fb > cs ? (int)(fb - cs) : 0, jhi = (int)(p - cs);
    uint32_t c = chunk[k];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t b = (W[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        c += (j >= jlo && j < jhi && (b & 0xC0u) != 0x80u) ? 1u : 0u;
    }
    return c;
}

__device__ __forceinline__ uint64_t it_with_pos(uint64_t it, uint32_t pos)
{
    return (it & ~((uint64_t)IT_POS_MASK << IT_POS_SHIFT)) | ((uint64_t)pos << IT_POS_SHIFT);
}

// Whether a name the transcoded view cannot decide (PI_TXUNSAFE) and at least as long as a short field of n
// code points (tf: its transcoded bytes) passes the short kernel's signature test for it (popcount(field
// signature & ~name signature) <= (2n - 1) / 20: a name's signature has the bits of its code points and of
// their transcoded bytes, so a code point the two share never counts); only then may the field decide such a
// name, which the resolve kernel must do.  Whole wave.
__device__ __forceinline__ bool fk_txu_short(const FastTables &FT, const uint8_t *tf, uint32_t n)
{
    const int lane = lane_id();
    if (n == 0 || n > (uint32_t)MAXM) return false;
    if (FT.n_txu > 8u * WAVE) return true;
    uint64_t fsig = (uint32_t)lane < n ? 1ull << (tf[lane] & 63u) : 0ull;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) fsig |= __shfl_xor(fsig, d, WAVE);
    const uint32_t allow = (2 * n - 1) / 20;
    bool c = false;
    for (uint32_t i = (uint32_t)lane; i < FT.n_txu; i += WAVE) {
        const uint32_t p = FT.txu_pat[i];
        c |= pi_m(FT.pat_info[p]) >= n && (uint32_t)__popcll(fsig & ~FT.pat_sig[p]) <= allow;
    }
    return __ballot(c) != 0;
}

// Whether a name the transcoded view cannot decide, of EDGE_MIN_M..EDGE_MAX_M code points, may have a one-deletion
// edge window in a field of n code points (tf: its transcoded bytes): the window (its first or last m - 1 code
// points) holds only code points of the name, so its signature has no bit the name's lacks.  Whole wave.
__device__ __forceinline__ bool fk_txu_edge(const FastTables &FT, const uint8_t *tf, uint32_t n)
{
    const int lane = lane_id();
    if (n + 1 < EDGE_MIN_M) return false;
    if (FT.n_txu > 8u * WAVE) return true;
    const uint32_t w = n < EDGE_MAX_M ? n : EDGE_MAX_M;   // (a window has at most EDGE_MAX_M - 1 code points)
    uint64_t bp = (uint32_t)lane < w ? 1ull << (tf[lane] & 63u) : 0ull;
    uint64_t bs = (uint32_t)lane < w ? 1ull << (tf[n - 1 - lane] & 63u) : 0ull;
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) {   // inclusive prefix OR: lane k - 1 = the first / last k code points
        const uint64_t up = __shfl_up(bp, d, WAVE), us = __shfl_up(bs, d, WAVE);
        if (lane >= d) { bp |= up; bs |= us; }
    }
    bool c = false;
    for (uint32_t k = EDGE_MIN_M - 1; k < EDGE_MAX_M && k <= n; ++k) {
        const uint64_t sp = __shfl(bp, (int)k - 1, WAVE), ss = __shfl(bs, (int)k - 1, WAVE);
        for (uint32_t i = (uint32_t)lane; i < FT.n_txu; i += WAVE) {
            const uint32_t p = FT.txu_pat[i];
            const uint64_t sg = FT.pat_sig[p];
            c |= pi_m(FT.pat_info[p]) == k + 1 && ((sp & ~sg) == 0ull || (ss & ~sg) == 0ull);
        }
    }
    return __ballot(c) != 0;
}

// Finish a transcoded document (V = its vrec) in the epilogue.  D0: the document in the arena, flags: its
// dflags | edge flags (of the arena bytes).  Returns false, before anything is emitted, when the resolve
// kernel must take it; otherwise *done = the epilogue's result (false: the generic kernel).
// CAP0 / CAP1: the item buffers' sizes (one wave's, or a big document's: the workgroup's LDS).
template <uint32_t CAP0 = FK_ITEMS0, uint32_t CAP1 = FK_ITEMS1>
__device__ bool epi_tx_doc(const FastTables &FT, const FastScratch &S, const DevScratch &GS, const FastDoc &D0, uint4 V,
                           uint32_t ibeg, uint32_t n0, uint32_t n1, uint32_t flags, uint64_t *items, int64_t wave,
                           OutCtx &O, TaskCounts &TC, bool *done)
{
    const int lane = lane_id();
    if (V.y == TX_NONE || (flags & DH_DEFER) || n0 > CAP0 || n1 > CAP1) return false;
    const uint32_t c0 = V.z, c1 = V.w;
    const int64_t tb = (int64_t)(((uint64_t)(V.y & 0x7FFFFFFFu) << 32) | V.x);
    // an edge-flagged non-ASCII field: a one-deletion edge window of a name the view cannot decide may be there
    if (FT.tx_unsafe_edge && (((flags & DH_NA0) && (flags & DH_EDGE0) && fk_txu_edge(FT, S.tarena + tb, c0)) ||
                              ((flags & DH_NA1) && (flags & DH_EDGE1) && fk_txu_edge(FT, S.tarena + tb + c0, c1))))
        return false;
    // a short non-ASCII field meets every name at least as long: one the view cannot decide may be among them
    if (FT.tx_unsafe_short && (((flags & DH_NA0) && fk_txu_short(FT, S.tarena + tb, c0)) ||
                               ((flags & DH_NA1) && fk_txu_short(FT, S.tarena + tb + c0, c1))))
        return false;
    const uint64_t nb = tx_bytes(D0.t1 - D0.t0, D0.t2 - D0.t1);
    const uint16_t *ch0 = (const uint16_t *)(S.tarena + tb + nb);
    const uint16_t *ch1 = ch0 + ((flags & DH_NA0) ? tx_nchunks(D0.t0, D0.t1) : 0u);
    // the items at code point positions; a name the view cannot decide sends the document to the resolve kernel
    const uint64_t *src = S.items + ibeg;
    bool unsafe = false;
    for (uint32_t i = (uint32_t)lane; i < n0 + n1; i += WAVE) {
        uint64_t it = src[i];
        const bool t = i < n0;
        unsafe |= (FT.pat_info[it_pat(it)] & PI_TXUNSAFE) != 0;
        if (flags & (t ? DH_NA0 : DH_NA1))
            it = it_with_pos(it, tx_pos(D0.arena, t ? D0.t0 : D0.t1, t ? ch0 : ch1, it_pos(it)));
        items[t ? i : CAP0 + (i - n0)] = it;
    }
    if (__ballot(unsafe)) return false;
    wave_sync();
    FastDoc D;
    D.arena = S.tarena;
    D.t0 = tb;
    D.t1 = D.t0 + c0;
    D.t2 = D.t1 + c1;
    D.doc = D0.doc;
    D.l1 = (int32_t)c0;
    D.l2 = (int32_t)(c0 + c1);
    *done = fk_scan_epilogue<CAP0>(FT, S, GS, D, items, n0, n1, flags, wave, O, TC);
    return true;
}

constexpr uint32_t EK_TXBIG = 0x80000000u;   // blk_docs entry: a transcoded big document (epi_big_doc)

// ---------------------------------------------------------------- big documents
// A document with more items than one epilogue wave's LDS holds (FK_ITEMS0 / FK_ITEMS1; a 50k-name KB has
// pieces that many names share), up to FK_BIG0 / FK_BIG1: finished by the same epilogue after the
// workgroup's loop, by its wave 0 with the whole workgroup's LDS (items), in wave 0's hit and task regions.
// An entry with EK_TXBIG is a document with a non-ASCII field: finished on its transcoded view (epi_tx_doc's
// tests and item positions), else left to the resolve kernel.  Returns bit 0: the document went to the
// generic kernel (a name with > 64 items), bit 1: finished on its transcoded view, bit 2: left to the
// resolve kernel, bit 3: a deferral of the transcoded view's.
#ifndef EK_BIG_NOINLINE   // 1: epi_big_doc as a called function (a call frame; 0: inlined into the epilogue)
#define EK_BIG_NOINLINE 0
#endif
#if EK_BIG_NOINLINE
__device__ __attribute__((noinline))
#else
__device__ __forceinline__
#endif
uint32_t epi_big_doc(const FastTables &FT, const FastScratch &S, const DevScratch &GS,
                                                          const uint8_t *__restrict__ arena, const int64_t *__restrict__ off,
                                                          uint32_t e, uint64_t *items, int64_t wave, OutCtx &O,
                                                          TaskCounts &TC)
{
    const int lane = lane_id();
    const bool tx = (e & EK_TXBIG) != 0;
    const uint32_t d = e & ~EK_TXBIG;
    const int64_t ov = lane < 3 ? off[2 * (int64_t)d + lane] : 0;
    const uint2 hv = lane == 3 ? S.hdr[d] : (lane == 4 ? S.ncnt[d] : (lane == 5 ? make_uint2(0u, S.dflags[d]) :
                                                                    make_uint2(0u, 0u)));
    FastDoc D;
    D.arena = arena;
    D.t0 = rdlane64(ov, 0);
    D.t1 = rdlane64(ov, 1);
    D.t2 = rdlane64(ov, 2);
    D.doc = d;
    D.l1 = (int32_t)(D.t1 - D.t0);
    D.l2 = (int32_t)(D.t2 - D.t0);
    const uint32_t ibeg = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 3);
    const uint32_t dfl = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 5);
    uint32_t flags = dfl & ~DH_DEFER;
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 4);
    const uint32_t n1 = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 4);
    flags |= fk_edge_flags(FT, D);
    const uint64_t *src = S.items + ibeg;
    bool view = true;
    if (tx) {
        // the transcoded view: epi_tx_doc's tests, item positions as code points, the document's bytes
        const uint4 V = S.vrec[d];
        const uint32_t c0 = V.z, c1 = V.w;
        const int64_t tb = (int64_t)(((uint64_t)(V.y & 0x7FFFFFFFu) << 32) | V.x);
        view = V.y != TX_NONE && !(dfl & DH_DEFER) &&
               !(FT.tx_unsafe_edge && (((flags & DH_NA0) && (flags & DH_EDGE0) && fk_txu_edge(FT, S.tarena + tb, c0)) ||
                                       ((flags & DH_NA1) && (flags & DH_EDGE1) && fk_txu_edge(FT, S.tarena + tb + c0, c1)))) &&
               !(FT.tx_unsafe_short && (((flags & DH_NA0) && fk_txu_short(FT, S.tarena + tb, c0)) ||
                                        ((flags & DH_NA1) && fk_txu_short(FT, S.tarena + tb + c0, c1))));
        if (view) {
            const uint64_t nb = tx_bytes(D.t1 - D.t0, D.t2 - D.t1);
            const uint16_t *ch0 = (const uint16_t *)(S.tarena + tb + nb);
            const uint16_t *ch1 = ch0 + ((flags & DH_NA0) ? tx_nchunks(D.t0, D.t1) : 0u);
            bool unsafe = false;
            for (uint32_t i = (uint32_t)lane; i < n0 + n1; i += WAVE) {
                uint64_t it = src[i];
                const bool t = i < n0;
                unsafe |= (FT.pat_info[it_pat(it)] & PI_TXUNSAFE) != 0;
                if (flags & (t ? DH_NA0 : DH_NA1))
                    it = it_with_pos(it, tx_pos(arena, t ? D.t0 : D.t1, t ? ch0 : ch1, it_pos(it)));
                items[t ? i : FK_BIG0 + (i - n0)] = it;
            }
            view = __ballot(unsafe) == 0ull;
            D.arena = S.tarena;
            D.t0 = tb;
            D.t1 = D.t0 + c0;
            D.t2 = D.t1 + c1;
            D.l1 = (int32_t)c0;
            D.l2 = (int32_t)(c0 + c1);
        }
        if (!view) {
            if (lane == 0) {
                S.dflags[d] = dfl | DH_RESOLVE;
                const uint32_t i = atomicAdd(S.res_cnt, 1u);
                if (i < S.defer_cap) S.res_list[i] = d;
            }
            wave_sync();
            return 4u;
        }
    } else {
        for (uint32_t k = (uint32_t)lane; k < n0; k += WAVE) items[k] = src[k];
        for (uint32_t k = (uint32_t)lane; k < n1; k += WAVE) items[FK_BIG0 + k] = src[n0 + k];
    }
    wave_sync();
    const bool done = fk_scan_epilogue<FK_BIG0>(FT, S, GS, D, items, n0, n1, flags, wave, O, TC);
    uint2 h;
    h.x = ibeg;
    if (!done) {
        h.y = DH_DEFER;
        if (lane == 0) {
            const uint32_t j = atomicAdd(S.defer_cnt, 1u);
            if (j < S.defer_cap) S.defer_list[j] = d;
            else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
            if (!tx) atomicAdd(&S.stats[5], 1ull);
            atomicAdd(&S.stats[13], 1ull);
        }
    } else {
        // (the header's counts saturate: informational only past the resolve kernel)
        h.y = min(n0, 1023u) | (min(n1, 127u) << DH_N1_SHIFT) | (flags & ~DH_DEFER) | (tx ? DH_TX : 0u);
        if (lane == 0 && !tx)
            S.vrec[d] = make_uint4((uint32_t)D.t0, (uint32_t)((uint64_t)D.t0 >> 32), (uint32_t)(D.t1 - D.t0), (uint32_t)(D.t2 - D.t1));
    }
    if (lane == 0) S.hdr[d] = h;
    wave_sync();
    return (done ? 0u : 1u) | (tx ? 2u : 0u) | ((tx && !done) ? 8u : 0u);
}

// the epilogue's per-document loads: lanes 0..2 the offsets, lane 3 the header, lane 4 the item counts,
// lane 5 the flags (y)
__device__ __forceinline__ void epi_meta(const FastScratch &S, const int64_t *__restrict__ off, int64_t d, int64_t &ov,
                                         uint2 &hv)
{
    const int lane = lane_id();
    ov = lane < 3 ? off[2 * d + lane] : 0;
    hv = lane == 3 ? S.hdr[d] : (lane == 4 ? S.ncnt[d] : (lane == 5 ? make_uint2(0u, S.dflags[d]) : make_uint2(0u, 0u)));
}

// the loads that depend on epi_meta's: lanes 0..3 the edge keys (first / last eight bytes of each field),
// lanes < n0 + n1 the document's first 64 items (all-ASCII documents the epilogue will finish only)
__device__ __forceinline__ void epi_prefetch(const uint8_t *__restrict__ arena, const FastScratch &S, int64_t ov,
                                             uint2 hv, uint64_t &ek, uint64_t &itp)
{
    const int lane = lane_id();
    const int64_t t0 = rdlane64(ov, 0), t1 = rdlane64(ov, 1), t2 = rdlane64(ov, 2);
    const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 5);
    if (fl & (DH_NA0 | DH_NA1 | DH_DEFER)) return;
    if (t1 - t0 > MAX_FIELD_BYTES || t2 - t1 > MAX_FIELD_BYTES) return;
    const int f = lane >> 1;
    const int64_t fb = f ? t1 : t0, fe = f ? t2 : t1;
    if (lane < 4 && fe - fb >= (int64_t)EDGE_MIN_M + 1) {
        const int64_t a = (lane & 1) ? fe - 8 : fb;
        ek = (uint64_t)ld_u32_unaligned(arena, a) | ((uint64_t)ld_u32_unaligned(arena, a + 4) << 32);
    }
    const uint32_t ibeg = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 3);
    const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 4) + (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 4);
    if ((uint32_t)lane < n) itp = S.items[ibeg + (uint32_t)lane];
}

// ---------------------------------------------------------------- kernel 3: per-document epilogue
__global__ __launch_bounds__(EK_BLOCK, EK_MINW) void kw_epi_kernel(FastTables FT, const uint8_t *__restrict__ arena,
                                                          const int64_t *__restrict__ off, int64_t n_docs,
                                                          FastScratch S, DevScratch GS)
{
    __shared__ uint64_t items_all[EK_WAVES * (FK_ITEMS0 + FK_ITEMS1)];
    __shared__ uint32_t blk_docs[EK_BIGQ];   // this workgroup's big documents (finished after its loop)
    __shared__ uint32_t blk_n;
    static_assert(EK_WAVES * (FK_ITEMS0 + FK_ITEMS1) >= FK_BIG0 + FK_BIG1, "a big document needs the block's LDS");
    if (threadIdx.x == 0) blk_n = 0;
    __syncthreads();
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t wave = (int64_t)blockIdx.x * EK_WAVES + wib;
    const int64_t n_waves = (int64_t)gridDim.x * EK_WAVES;
    uint64_t *items = items_all + wib * (FK_ITEMS0 + FK_ITEMS1);
    uint32_t ndefer = 0, ndef_items = 0, ntx = 0, nres = 0;
    OutCtx O;
    O.shared = nullptr;
    O.out = S.kout + (size_t)wave * S.out_cap;
    O.cap = S.out_cap;
    O.n = 0;
    TaskCounts TC = {0u, 0u, 0u, 0u};
    // Software pipeline over the wave's documents: the next document's offsets / header / counts / flags
    // are in flight while the current one is processed, and its edge keys and first 64 items are loaded
    // right after, so a document starts with only the edge-bitmap and name-table round trips ahead of it.
    int64_t ov = 0;
    uint2 hv = make_uint2(0u, 0u);
    uint64_t ek = 0, itp = 0;
    if (wave < n_docs) {
        epi_meta(S, off, wave, ov, hv);
        epi_prefetch(arena, S, ov, hv, ek, itp);
    }
    unsigned long long ekt[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    EK_T0(tk0);
    for (int64_t d = wave; d < n_docs; d += n_waves) {
        EK_T0(td0);
        const int64_t dn = d + n_waves;
        int64_t ovn = 0;
        uint2 hvn = make_uint2(0u, 0u);
        if (dn < n_docs) epi_meta(S, off, dn, ovn, hvn);
        FastDoc D;
        D.arena = arena;
        D.t0 = rdlane64(ov, 0);
        D.t1 = rdlane64(ov, 1);
        D.t2 = rdlane64(ov, 2);
        D.doc = (uint32_t)d;
        D.l1 = (int32_t)(D.t1 - D.t0);
        D.l2 = (int32_t)(D.t2 - D.t0);
        const uint32_t ibeg = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 3);
        uint32_t flags = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 5);
        if (flags & (DH_NA0 | DH_NA1)) {
            // a non-ASCII field: the transcoded view, or the resolve kernel
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 4);
            const uint32_t n1 = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 4);
            const uint32_t fl = flags | fk_edge_flags(FT, D);
            bool done = false;
            if (FK_TX && epi_tx_doc(FT, S, GS, D, S.vrec[d], ibeg, n0, n1, fl, items, wave, O, TC, &done)) {
                ++ntx;
                uint2 h;
                h.x = ibeg;
                if (!done) {
                    ++ndefer;
                    ++ndef_items;
                    h.y = DH_DEFER;
                    if (lane == 0) {
                        atomicAdd(&S.stats[13], 1ull);
                        const uint32_t i = atomicAdd(S.defer_cnt, 1u);
                        if (i < S.defer_cap) S.defer_list[i] = (uint32_t)d;
                        else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
                    }
                } else {
                    h.y = n0 | (n1 << DH_N1_SHIFT) | (fl & ~DH_DEFER) | DH_TX;   // (vrec: kw_tx_kernel's)
                }
                if (lane == 0) S.hdr[d] = h;
            } else {
                ++nres;
                if (lane == 0) {
                    S.dflags[d] = flags | DH_RESOLVE;
                    const uint32_t i = atomicAdd(S.res_cnt, 1u);
                    if (i < S.defer_cap) S.res_list[i] = (uint32_t)d;
                }
            }
            wave_sync();
        } else {
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)hv.x, 4);
            const uint32_t n1 = (uint32_t)__builtin_amdgcn_readlane((int)hv.y, 4);
            EK_TACC(ekt[5], td0);
            EK_T0(td1);
            flags |= fk_edge_flags_key(FT, D, ek);
            EK_TACC(ekt[6], td1);
            bool defer = (flags & DH_DEFER) != 0 || D.t1 - D.t0 > MAX_FIELD_BYTES || D.t2 - D.t1 > MAX_FIELD_BYTES;
            if (defer && lane == 0) atomicAdd(&S.stats[15], 1ull);   // (rare: counted where they happen)
            bool queued = false;
            if (!defer && (n0 > (uint32_t)FK_ITEMS0 || n1 > (uint32_t)FK_ITEMS1)) {
                // more items than this kernel's LDS holds: the big-document epilogue, beyond its caps the generic kernel
                uint32_t bi = 0xFFFFFFFFu;
                if (n0 <= (uint32_t)FK_BIG0 && n1 <= (uint32_t)FK_BIG1) {
                    if (lane == 0) bi = atomicAdd(&blk_n, 1u);
                    bi = (uint32_t)__builtin_amdgcn_readfirstlane((int)bi);
                }
                if (bi < S.bigq) {
                    if (lane == 0) blk_docs[bi] = (uint32_t)d;
                    queued = true;
                } else if (n0 <= (uint32_t)FK_BIG0 && n1 <= (uint32_t)FK_BIG0) {
                    // the workgroup's queue is full (or the title is past FK_BIG1): the resolve kernel's big documents
                    ++nres;
                    queued = true;
                    if (lane == 0) {
                        S.dflags[d] = flags | DH_RESOLVE;
                        const uint32_t i = atomicAdd(S.res_cnt, 1u);
                        if (i < S.defer_cap) S.res_list[i] = (uint32_t)d;
                    }
                } else {
                    defer = true;
                    ++ndef_items;
                    if (lane == 0) atomicAdd(&S.stats[14], 1ull);
                }
            }
            if (!queued) {
                flags &= ~DH_DEFER;
                if (!defer) {
                    // the first 64 items came with the prefetch (text items first, then the title's)
                    if ((uint32_t)lane < n0 + n1) items[(uint32_t)lane < n0 ? lane : FK_ITEMS0 + lane - (int)n0] = itp;
                    const uint64_t *src = S.items + ibeg;
                    for (uint32_t i = (uint32_t)lane + WAVE; i < n0; i += WAVE) items[i] = src[i];
                    for (uint32_t i = (uint32_t)lane; i < n1; i += WAVE)
                        if (n0 + i >= (uint32_t)WAVE) items[FK_ITEMS0 + i] = src[n0 + i];
                    wave_sync();
                    EK_T0(td2);
                    const bool done = fk_scan_epilogue(FT, S, GS, D, items, n0, n1, flags, wave, O, TC, ekt);
                    EK_TACC(ekt[7], td2);
                    if (!done) {
                        defer = true;
                        ++ndef_items;
                        if (lane == 0) atomicAdd(&S.stats[13], 1ull);
                    }
                }
                uint2 h;
                h.x = ibeg;
                if (defer) {
                    ++ndefer;
                    h.y = DH_DEFER;
                    if (lane == 0) {
                        const uint32_t i = atomicAdd(S.defer_cnt, 1u);
                        if (i < S.defer_cap) S.defer_list[i] = (uint32_t)d;
                        else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
                    }
                } else {
                    h.y = n0 | (n1 << DH_N1_SHIFT) | flags;
                    if (lane == 0) S.vrec[d] = make_uint4((uint32_t)D.t0, (uint32_t)((uint64_t)D.t0 >> 32), (uint32_t)(D.t1 - D.t0), (uint32_t)(D.t2 - D.t1));
                }
                if (lane == 0) S.hdr[d] = h;
                wave_sync();
            }
        }
        EK_T0(td3);
        ek = 0;
        itp = 0;
        if (dn < n_docs) epi_prefetch(arena, S, ovn, hvn, ek, itp);
        ov = ovn;
        hv = hvn;
        EK_TACC(ekt[8], td3);
        EK_TACC(ekt[9], td0);
    }
    EK_TACC(ekt[10], tk0);
    if (EK_TIMING && lane == 0)
        for (int i = 0; i < 11; ++i) atomicAdd(&S.stats[21 + i], ekt[i]);
    // the workgroup's big documents: wave 0 with the whole workgroup's LDS as one 4096 + 512-item buffer
    __syncthreads();
#if defined(EK_TIMING_SKIP_BIG)   // (timing variant only, results void: the big documents are not finished)
    const uint32_t nb = 0;
#else
    const uint32_t nb = min(blk_n, S.bigq);
#endif
    if (wib == 0 && nb) {
        for (uint32_t i = 0; i < nb; ++i) ndefer += epi_big_doc(FT, S, GS, arena, off, blk_docs[i], items_all, wave, O, TC) & 1u;
        if (lane == 0) atomicAdd(&S.stats[16], (unsigned long long)nb);
    }
    if (lane == 0) {
        S.kout_cnt[wave] = O.n;
        S.vcnt[wave] = TC.v;
        if (TC.e) atomicAdd(&S.stats[7], (unsigned long long)TC.e);
        S.scnt[wave] = TC.s;
        S.xcnt[wave] = TC.x;
        S.xmark[wave] = TC.x;   // (the regex tasks the epilogue queued: KW_RX_SPLIT's early phase)
        if (TC.v > S.vcap || TC.s > S.scap || TC.x > S.xcap) {
            atomicOr(&S.status[0], ST_TASK_OVERFLOW);
            atomicMax(&S.tmax[0], TC.v);
            atomicMax(&S.tmax[2], TC.s);
            atomicMax(&S.tmax[3], TC.x);
        }
        atomicAdd(&S.stats[4], (unsigned long long)ndefer);
        atomicAdd(&S.stats[5], (unsigned long long)ndef_items);
        if (ntx) atomicAdd(&S.stats[18], (unsigned long long)ntx);
        if (nres) atomicAdd(&S.stats[19], (unsigned long long)nres);
    }
}



// ---------------------------------------------------------------- kernel 3b: the epilogue over groups of documents
// The same decisions as kw_epi_kernel, but a wave takes a filter group (32 consecutive documents) at a time
// and works the items of its plain documents (all-ASCII, not deferred, <= 64 items per field) 64 at a time
// across documents: lane = item, a batch is a run of whole (document, field) segments, sorted by (segment,
// name, position), the name groups are (segment, name) runs.  Document-level work (edge prefilter, short-field
// tasks, headers, view records) is lane = document.  Edge windows of flagged documents and the other
// documents (non-ASCII, big, deferred) take the per-document code after the batches.
__device__ __forceinline__ uint32_t ep_n(const uint32_t (&v)[2], uint32_t f) { return f ? v[1] : v[0]; }

template <bool TXB>
__global__ __launch_bounds__(EK_BLOCK, EK_MINW) void kw_epi_flat_kernel(FastTables FT, const uint8_t *__restrict__ arena,
                                                               const int64_t *__restrict__ off, int64_t n_docs,
                                                               FastScratch S, DevScratch GS)
{
    __shared__ uint64_t items_all[EK_WAVES * (FK_ITEMS0 + FK_ITEMS1)];
    __shared__ uint32_t blk_docs[EK_BIGQ];
    __shared__ uint4 segtx_all[TXB ? EK_WAVES * WAVE : 1];   // TXB: the segments' arena start, chunk table
    __shared__ uint32_t blk_n;
    if (threadIdx.x == 0) blk_n = 0;
    __syncthreads();
    const int lane = lane_id();
    const int wib = threadIdx.x / WAVE;
    const int64_t wave = (int64_t)blockIdx.x * EK_WAVES + wib;
    const int64_t n_waves = (int64_t)gridDim.x * EK_WAVES;
    uint64_t *items = items_all + wib * (FK_ITEMS0 + FK_ITEMS1);
    uint4 *segtx = segtx_all + (TXB ? wib * WAVE : 0);
    uint32_t ndefer = 0, ndef_items = 0, ntx = 0, nres = 0;
    OutCtx O;
    O.shared = nullptr;
    O.out = S.kout + (size_t)wave * S.out_cap;
    O.cap = S.out_cap;
    O.n = 0;
    TaskCounts TC = {0u, 0u, 0u, 0u};
    uint4 *vq = S.vq + (size_t)wave * S.vcap;
    uint4 *sq = S.sq + (size_t)wave * S.scap, *xq = S.xq + (size_t)wave * S.xcap;
    const int64_t n_groups = (n_docs + FG_DOCS - 1) / FG_DOCS;
    for (int64_t g = wave; g < n_groups; g += n_waves) {
        const int64_t d0 = g * FG_DOCS;
        const int nd = (int)(n_docs - d0 < FG_DOCS ? n_docs - d0 : FG_DOCS);
        // ---- lane = document: offsets, header, counts, flags, the edge prefilter
        const bool act = lane < nd;
        const int64_t d = d0 + (act ? lane : 0);
        const int64_t t0 = act ? off[2 * d] : 0, t1 = act ? off[2 * d + 1] : 0, t2 = act ? off[2 * d + 2] : 0;
        const uint2 hd = act ? S.hdr[d] : make_uint2(0u, 0u);
        const uint2 nc = act ? S.ncnt[d] : make_uint2(0u, 0u);
        const uint32_t fl = act ? S.dflags[d] : 0u;
        uint32_t ef = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int f = k >> 1;
            const int64_t fb = f ? t1 : t0, fe = f ? t2 : t1;
            if (act && fe - fb >= (int64_t)EDGE_MIN_M + 1) {
                const int64_t a = (k & 1) ? fe - 8 : fb;
                const uint64_t key8 = (uint64_t)ld_u32_unaligned(arena, a) | ((uint64_t)ld_u32_unaligned(arena, a + 4) << 32);
                const uint32_t idx = fk_edge_index(key8);
                if ((((k & 1) ? FT.edge_suf : FT.edge_pre)[idx >> 5] >> (idx & 31u)) & 1u) ef |= f ? DH_EDGE1 : DH_EDGE0;
            }
        }
        const uint32_t flags = fl | ef;
        const int64_t l0 = t1 - t0, l1 = t2 - t1;
        // TXB: a document with a non-ASCII field joins the batches on its transcoded view (the transcoding
        // kernel's record V: the view's place, the fields' code point counts; its items' positions become code
        // points).  The host picks TXB only when no name is PI_TXUNSAFE (kw_epi_kernel's per-document tests)
        const bool na = (fl & (DH_NA0 | DH_NA1)) != 0;
        uint32_t c0 = (uint32_t)l0, c1 = (uint32_t)l1;   // the fields' code points
        bool txd = false;
        uint4 V = make_uint4(0u, TX_NONE, 0u, 0u);
        if (TXB && act && na) {
            V = S.vrec[d];
            txd = V.y != TX_NONE;
            if (txd) { c0 = V.z; c1 = V.w; }
        }
        const bool flat = act && !(fl & DH_DEFER) && (!na || txd) && l0 <= MAX_FIELD_BYTES &&
                          l1 <= MAX_FIELD_BYTES && nc.x <= (uint32_t)WAVE && nc.y <= (uint32_t)WAVE;
        const uint64_t flatm = __ballot(flat);
        const uint64_t txm = TXB ? __ballot(flat && txd) : 0ull;   // (wave-uniform: 0 for an all-ASCII group)
        if (txm) {   // segment 2 l + f's arena start and chunk table of code point counts (tarena offset; tx_pos)
            wave_sync();
            if (flat && txd) {
                const int64_t ch0 = (int64_t)(((uint64_t)(V.y & 0x7FFFFFFFu) << 32) | V.x) + (int64_t)tx_bytes(l0, l1);
                const int64_t ch1 = ch0 + 2 * (int64_t)((fl & DH_NA0) ? tx_nchunks(t0, t1) : 0u);
                segtx[2 * lane] = make_uint4((uint32_t)t0, (uint32_t)((uint64_t)t0 >> 32), (uint32_t)ch0,
                                             (uint32_t)((uint64_t)ch0 >> 32));
                segtx[2 * lane + 1] = make_uint4((uint32_t)t1, (uint32_t)((uint64_t)t1 >> 32), (uint32_t)ch1,
                                                 (uint32_t)((uint64_t)ch1 >> 32));
            }
            wave_sync();
        }
        // ---- lane = segment s = 2 * document + field of the plain documents: size, first item, batch offset
        const int sd = lane >> 1, sf = lane & 1;
        const uint32_t s_n0 = (uint32_t)__shfl((int)nc.x, sd, WAVE), s_n1 = (uint32_t)__shfl((int)nc.y, sd, WAVE);
        const uint32_t s_beg = (uint32_t)__shfl((int)hd.x, sd, WAVE);
        const bool s_flat = (flatm >> sd) & 1ull;
        const uint32_t sz = s_flat ? (sf ? s_n1 : s_n0) : 0u;
        const uint32_t st = s_beg + (sf ? s_n0 : 0u);
        int stot;
        const uint32_t soff = (uint32_t)wave_excl_scan_dpp((int)sz, &stot);
        const uint32_t s_l0 = (uint32_t)__shfl((int)c0, sd, WAVE), s_l1 = (uint32_t)__shfl((int)c1, sd, WAVE);
        const uint32_t s_len = sf ? s_l1 : s_l0;   // the segment's field length in code points
        // the segments of non-ASCII fields (transcoded documents)
        uint64_t snam = 0;
        if (txm) {
            const uint32_t s_fl = (uint32_t)__shfl((int)fl, sd, WAVE);
            snam = __ballot(s_flat && ((txm >> sd) & 1ull) && (s_fl & (sf ? DH_NA1 : DH_NA0)));
        }
        // ---- batches of whole segments, <= 64 items each
        for (uint32_t base = 0; base < (uint32_t)stot;) {
            // the segments that fit: soff + sz - base <= 64 (soff ascending)
            const uint64_t fit = __ballot(soff >= base && soff + sz - base <= (uint32_t)WAVE);
            const int last = 63 - __builtin_clzll(fit);
            const uint32_t bend = (uint32_t)__shfl((int)(soff + sz), last, WAVE);
            const uint32_t cnt = bend - base;
            // lane = item: its segment (the last one starting at or before it), the item
            int sg = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const int c = sg + step;
                const uint32_t oc = (uint32_t)__shfl((int)soff, c & 63, WAVE);
                if (c < WAVE && oc <= base + (uint32_t)lane) sg = c;
            }
            const bool valid = (uint32_t)lane < cnt;
            const uint32_t sgo = (uint32_t)__shfl((int)soff, sg, WAVE), sgs = (uint32_t)__shfl((int)st, sg, WAVE);
            uint64_t it0 = valid ? S.items[sgs + (base + (uint32_t)lane - sgo)] : 0ull;
            if (snam && valid && ((snam >> sg) & 1ull)) {   // (an item of a non-ASCII field: its position in code points)
                const uint4 e = segtx[sg];
                const int64_t fbs = (int64_t)(((uint64_t)e.y << 32) | e.x), chs = (int64_t)(((uint64_t)e.w << 32) | e.z);
                it0 = it_with_pos(it0, tx_pos(arena, fbs, (const uint16_t *)(S.tarena + chs), it_pos(it0)));
            }
            base = bend;
            // sort by (segment, name, position, kind); the use rides along
            uint32_t use = it_use(it0);
            const uint64_t key0 = valid ? (((uint64_t)sg << 58) | ((it0 >> 19) << 13)) : ~0ull;   // (it >> 19: name,
            const uint64_t key = wave_sort_reg_kv(key0, use);                                      //  position, kind)
            const uint32_t seg = (uint32_t)(key >> 58);
            const uint32_t pat = valid ? (uint32_t)((key >> 38) & 0xFFFFFu) : 0xFFFFFu;
            const uint32_t bpos = (uint32_t)((key >> 15) & IT_POS_MASK);
            const uint32_t kind = (uint32_t)((key >> 13) & 3u);
            const uint32_t f = seg & 1u;
            const uint32_t doc = (uint32_t)(d0 + (seg >> 1));
            const uint32_t nf = (uint32_t)__shfl((int)s_len, (int)seg & 63, WAVE);
            const uint32_t pi = valid ? FT.pat_info[pat] : 0u;
            const uint32_t rxk = valid ? FT.pat_rxk[pat] : 0u;
            const uint32_t rxl = valid ? FT.pat_rxl[pat] : 0u;
            const uint32_t uinfo = (valid && kind == FU_PIECE) ? FT.use_info1[use] : 0u;
            const uint32_t m = pi_m(pi);
            // (RXM items are exact regex matches in an ASCII field only; a transcoded field's regex names are searched)
            const bool rxi = rxk == RXK_REGEX && rxl != 0u && !((snam >> seg) & 1ull);
            const uint32_t mlen = rxi ? rxl : m;
            const bool fuzzy = (pi & PI_FUZZY) != 0;
            const uint64_t gkey = key >> 38;   // (segment, name)
            const uint64_t prev_g = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(gkey >> 32), 1, WAVE) << 32) |
                                    (uint32_t)__shfl_up((int)(uint32_t)gkey, 1, WAVE);
            const bool head = valid && (lane == 0 || prev_g != gkey);
            const uint64_t heads = __ballot(head);
            const uint64_t below = (lane == 63) ? ~0ull : ((2ull << lane) - 1);
            const int gs = 63 - __builtin_clzll((heads & below) | 1ull);
            const uint64_t after = heads & ~below;
            const int ge = after ? __builtin_ctzll(after) : (int)cnt;
            const uint64_t gmask = (ge >= 64 ? ~0ull : ((1ull << ge) - 1)) & ~((1ull << gs) - 1);
            const bool live = valid && !(fuzzy && m >= nf);
            const uint64_t fullm = __ballot(live && kind == FU_FULL);
            const bool decided = (fullm & gmask) != 0;
            // pieces of undecided fuzzy names -> verify tasks, one per (group, alignment base): a piece lane is
            // pushed unless the previous piece lane of its group had the same base
            const bool vpiece = live && fuzzy && !decided && kind == FU_PIECE;
            const uint32_t o = (uinfo >> 16) & 0xFFu, pl = uinfo >> 24;
            const int64_t wkey = vpiece ? piece_window_key(bpos, o, pl, m, nf) : -1;
            const uint64_t vm = __ballot(vpiece);
            const uint64_t pv = vm & ((1ull << lane) - 1);
            const int pvl = pv ? 63 - __builtin_clzll(pv) : lane;
            const int pgs = __shfl(gs, pvl, WAVE);
            const uint32_t pk_lo = (uint32_t)__shfl((int)(uint32_t)wkey, pvl, WAVE);
            const uint32_t pk_hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)wkey >> 32), pvl, WAVE);
            const int64_t pkey = (int64_t)(((uint64_t)pk_hi << 32) | pk_lo);
            const bool vpush = vpiece && !(pv && pgs == gs && pkey == wkey);
            const uint64_t vpm = __ballot(vpush);
            if (vpm) {
                const uint32_t vi = TC.v + mbcnt(vpm);
                if (vpush && vi < S.vcap) vq[vi] = make_uint4(doc, (pat << 1) | f, bpos, o | (pl << 8));
                TC.v += (uint32_t)__popcll(vpm);
            }
            // positions: uppercase names, exact occurrences of decided literal fuzzy names, RXM matches of decided
            // regex names (leftmost non-overlapping per group)
            const bool relevant = live && ((!fuzzy && kind == FU_UPPER) ||
                                           (fuzzy && decided && ((rxk == RXK_LITERAL && kind == FU_FULL) ||
                                                                 (rxi && kind == FU_RXM && use != IT_USE_MASK))));
            const uint64_t relm = __ballot(relevant);
            const uint64_t prevrel = relm & gmask & ((1ull << lane) - 1);
            const int pr = prevrel ? 63 - __builtin_clzll(prevrel) : -1;
            const uint32_t pcpos = (uint32_t)__shfl((int)bpos, pr < 0 ? lane : pr, WAVE);
            const bool overlap = relevant && pr >= 0 && bpos < pcpos + mlen;
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
                    const uint32_t stp = (uint32_t)__shfl((int)bpos, l, WAVE);
                    const uint32_t len = (uint32_t)__shfl((int)mlen, l, WAVE);
                    if (hh != cur_head) { cur_head = hh; keep |= 1ull << l; last_end = stp + len; continue; }
                    if (stp >= last_end) { keep |= 1ull << l; last_end = stp + len; }
                }
            }
            emit_hits(O, GS, (keep >> lane) & 1ull, doc, pat, bpos, f);
            const bool dec_head = head && live && fuzzy && decided;
            if (dec_head && m >= EDGE_MIN_M && m <= EDGE_MAX_M) (void)dset_insert(S, dset_key(doc, pat, f));
            emit_hits(O, GS, dec_head && rxi && (keep & gmask) == 0, doc, pat, KW_NOPOS, f);
            const bool xrx = dec_head && rxk == RXK_REGEX && !rxi;
            const uint64_t xm = __ballot(xrx);
            if (xm) {
                const uint32_t xi = TC.x + mbcnt(xm);
                if (xrx && xi < S.xcap) xq[xi] = make_uint4(doc, (pat << 1) | f, 0u, 0u);
                TC.x += (uint32_t)__popcll(xm);
            }
        }
        // ---- lane = document: short-field tasks, headers, view records of the plain documents.  A short field
        // of more than SHORT_EXACT_MAX bytes whose names at least as long are few (titles: <= 12 of the S&P500
        // KB's) first takes the short kernel's signature test here: without a candidate name it needs no task.
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            const int64_t lf = f ? (int64_t)c1 : (int64_t)c0;
            bool sh = flat && lf <= (int64_t)MAXM;
            if (EPI_SHORT_PREF && sh && lf > (int64_t)SHORT_EXACT_MAX) {
                const uint32_t n = (uint32_t)lf, cnt = (uint32_t)FT.f_count_ge[n];
                if (cnt <= (uint32_t)WAVE) {
                    // (a transcoded document's field: its view bytes; the reads past the field stay in tarena's
                    // document record or its 64-byte tail)
                    int64_t fb = f ? t1 : t0;
                    const uint8_t *fa = arena;
                    if (txd) {
                        const uint4 Vs = S.vrec[d];
                        fb = (int64_t)(((uint64_t)(Vs.y & 0x7FFFFFFFu) << 32) | Vs.x) + (f ? (int64_t)Vs.z : 0);
                        fa = S.tarena;
                    }
                    const int64_t a0 = fb & ~(int64_t)3;
                    const uint32_t sh0 = (uint32_t)(fb - a0);
                    // the field's <= 67 bytes as dwords loaded six at a time (three round trips, not one per dword;
                    // the arena is padded; more at once spills the epilogue's registers), then the names'
                    // signatures four at a time
                    uint64_t fsig = 0;
                    for (uint32_t w0 = 0; 4 * w0 < n + sh0; w0 += 6) {
                        uint32_t xw[6];
#pragma unroll
                        for (int w = 0; w < 6; ++w) xw[w] = *(const uint32_t *)(fa + a0 + 4 * (w0 + (uint32_t)w));
#pragma unroll
                        for (int w = 0; w < 6; ++w) {
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                const uint32_t p = 4 * (w0 + (uint32_t)w) + (uint32_t)k;
                                if (p >= sh0 && p < n + sh0) fsig |= 1ull << ((xw[w] >> (8 * k)) & 63u);
                            }
                        }
                    }
                    const uint32_t allow = (2 * n - 1) / 20;
                    bool cand = false;
                    for (uint32_t c = 0; c < cnt && !cand; ++c)
                        cand = (uint32_t)__popcll(fsig & ~FT.pat_sig[FT.f_first + c]) <= allow;
                    sh = cand;
                }
            }
            const uint64_t shm = __ballot(sh);
            if (SHORT_COUNT && lane == 0 && shm) atomicAdd(&S.stats[25 + f], (unsigned long long)__popcll(shm));
            if (shm) {
                const uint32_t si = TC.s + mbcnt(shm);
                if (sh && si < S.scap) sq[si] = make_uint4((uint32_t)d, (uint32_t)f, 0u, 0u);
                TC.s += (uint32_t)__popcll(shm);
            }
        }
        // edge windows of the flagged plain documents (after all their items: the decided set is complete)
        uint64_t edm = __ballot(flat && (ef & (DH_EDGE0 | DH_EDGE1)));
        while (edm) {
            const int l = __builtin_ctzll(edm);
            edm &= edm - 1;
            FastDoc D;
            if ((txm >> l) & 1ull) {   // (a transcoded document: its windows on the view)
                const uint4 Vl = S.vrec[d0 + l];
                D.arena = S.tarena;
                D.t0 = (int64_t)(((uint64_t)(Vl.y & 0x7FFFFFFFu) << 32) | Vl.x);
                D.t1 = D.t0 + Vl.z;
                D.t2 = D.t1 + Vl.w;
            } else {
                D.arena = arena;
                D.t0 = rdlane64(t0, l);
                D.t1 = rdlane64(t1, l);
                D.t2 = rdlane64(t2, l);
            }
            D.doc = (uint32_t)(d0 + l);
            D.l1 = (int32_t)(D.t1 - D.t0);
            D.l2 = (int32_t)(D.t2 - D.t0);
            fk_epi_edge(FT, S, GS, D, (uint32_t)__builtin_amdgcn_readlane((int)flags, l), O, TC, xq);
        }
        if (flat) {
            S.hdr[d] = make_uint2(hd.x, nc.x | (nc.y << DH_N1_SHIFT) | flags | (txd ? DH_TX : 0u));
            if (!txd)   // (a transcoded document's view record is the transcoding kernel's)
                S.vrec[d] = make_uint4((uint32_t)t0, (uint32_t)((uint64_t)t0 >> 32), (uint32_t)l0, (uint32_t)l1);
        }
        ntx += (uint32_t)__popcll(txm);
        // ---- the other documents, one at a time (kw_epi_kernel's per-document code)
        uint64_t slow = __ballot(act && !flat);
        while (slow) {
            const int l = __builtin_ctzll(slow);
            slow &= slow - 1;
            const int64_t dd = d0 + l;
            FastDoc D;
            D.arena = arena;
            D.t0 = rdlane64(t0, l);
            D.t1 = rdlane64(t1, l);
            D.t2 = rdlane64(t2, l);
            D.doc = (uint32_t)dd;
            D.l1 = (int32_t)(D.t1 - D.t0);
            D.l2 = (int32_t)(D.t2 - D.t0);
            const uint32_t ibeg = (uint32_t)__builtin_amdgcn_readlane((int)hd.x, l);
            const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)nc.x, l);
            const uint32_t n1 = (uint32_t)__builtin_amdgcn_readlane((int)nc.y, l);
            const uint32_t dfl = (uint32_t)__builtin_amdgcn_readlane((int)fl, l);
            const uint32_t dflags = (uint32_t)__builtin_amdgcn_readlane((int)flags, l);
            if (TXB && (dfl & (DH_NA0 | DH_NA1))) {   // (no view, or more than 64 items in a field)
                ++nres;
                if (lane == 0) {
                    S.dflags[dd] = dfl | DH_RESOLVE;
                    const uint32_t i = atomicAdd(S.res_cnt, 1u);
                    if (i < S.defer_cap) S.res_list[i] = (uint32_t)dd;
                }
                wave_sync();
                continue;
            }
            if (dfl & (DH_NA0 | DH_NA1)) {
                bool done = false;
                if (FK_TX && (n0 > (uint32_t)FK_ITEMS0 || n1 > (uint32_t)FK_ITEMS1) && n0 <= (uint32_t)FK_BIG0 &&
                    n1 <= (uint32_t)FK_BIG1 && !(dflags & DH_DEFER)) {
                    // more items than a wave holds: the workgroup's big documents, on its LDS after the loop
                    uint32_t bi = 0;
                    if (lane == 0) bi = atomicAdd(&blk_n, 1u);
                    bi = (uint32_t)__builtin_amdgcn_readfirstlane((int)bi);
                    if (bi < S.bigq) {
                        if (lane == 0) blk_docs[bi] = (uint32_t)dd | EK_TXBIG;
                        wave_sync();
                        continue;
                    }
                }
                if (FK_TX && epi_tx_doc(FT, S, GS, D, S.vrec[dd], ibeg, n0, n1, dflags, items, wave, O, TC, &done)) {
                    ++ntx;
                    uint2 h;
                    h.x = ibeg;
                    if (!done) {
                        ++ndefer;
                        ++ndef_items;
                        h.y = DH_DEFER;
                        if (lane == 0) {
                            atomicAdd(&S.stats[13], 1ull);
                            const uint32_t i = atomicAdd(S.defer_cnt, 1u);
                            if (i < S.defer_cap) S.defer_list[i] = (uint32_t)dd;
                            else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
                        }
                    } else {
                        h.y = n0 | (n1 << DH_N1_SHIFT) | (dflags & ~DH_DEFER) | DH_TX;   // (vrec: kw_tx_kernel's)
                    }
                    if (lane == 0) S.hdr[dd] = h;
                } else {
                    ++nres;
                    if (lane == 0) {
                        S.dflags[dd] = dfl | DH_RESOLVE;
                        const uint32_t i = atomicAdd(S.res_cnt, 1u);
                        if (i < S.defer_cap) S.res_list[i] = (uint32_t)dd;
                    }
                }
                wave_sync();
                continue;
            }
            bool defer = (dflags & DH_DEFER) != 0 || D.t1 - D.t0 > MAX_FIELD_BYTES || D.t2 - D.t1 > MAX_FIELD_BYTES;
            if (defer && lane == 0) atomicAdd(&S.stats[15], 1ull);
            if (!defer && (n0 > (uint32_t)FK_ITEMS0 || n1 > (uint32_t)FK_ITEMS1)) {
                if (n0 <= (uint32_t)FK_BIG0 && n1 <= (uint32_t)FK_BIG0) {
                    // the workgroup's big documents; with its queue full (or the title past FK_BIG1) the resolve
                    // kernel's big documents
                    uint32_t bi = 0xFFFFFFFFu;
                    if (lane == 0 && n1 <= (uint32_t)FK_BIG1) bi = atomicAdd(&blk_n, 1u);
                    bi = (uint32_t)__builtin_amdgcn_readfirstlane((int)bi);
                    if (lane == 0) {
                        if (bi < S.bigq) {
                            blk_docs[bi] = (uint32_t)dd;
                        } else {
                            S.dflags[dd] = dflags | DH_RESOLVE;
                            const uint32_t i = atomicAdd(S.res_cnt, 1u);
                            if (i < S.defer_cap) S.res_list[i] = (uint32_t)dd;
                        }
                    }
                    continue;
                }
                defer = true;
                ++ndef_items;
                if (lane == 0) atomicAdd(&S.stats[14], 1ull);
            }
            const uint32_t fl2 = dflags & ~DH_DEFER;
            if (!defer) {
                const uint64_t *src = S.items + ibeg;
                for (uint32_t i = (uint32_t)lane; i < n0; i += WAVE) items[i] = src[i];
                for (uint32_t i = (uint32_t)lane; i < n1; i += WAVE) items[FK_ITEMS0 + i] = src[n0 + i];
                wave_sync();
                if (!fk_scan_epilogue(FT, S, GS, D, items, n0, n1, fl2, wave, O, TC)) {
                    defer = true;
                    ++ndef_items;
                    if (lane == 0) atomicAdd(&S.stats[13], 1ull);
                }
            }
            uint2 h;
            h.x = ibeg;
            if (defer) {
                ++ndefer;
                h.y = DH_DEFER;
                if (lane == 0) {
                    const uint32_t i = atomicAdd(S.defer_cnt, 1u);
                    if (i < S.defer_cap) S.defer_list[i] = (uint32_t)dd;
                    else atomicOr(&S.status[0], ST_ITEM_OVERFLOW);
                }
            } else {
                h.y = n0 | (n1 << DH_N1_SHIFT) | fl2;
                if (lane == 0) S.vrec[dd] = make_uint4((uint32_t)D.t0, (uint32_t)((uint64_t)D.t0 >> 32), (uint32_t)(D.t1 - D.t0), (uint32_t)(D.t2 - D.t1));
            }
            if (lane == 0) S.hdr[dd] = h;
            wave_sync();
        }
    }
    // the workgroup's big documents: wave 0 with the whole workgroup's LDS as one 4096 + 512-item buffer
    __syncthreads();
#if defined(EK_TIMING_SKIP_BIG)   // (timing variant only, results void: the big documents are not finished)
    const uint32_t nb = 0;
#else
    const uint32_t nb = min(blk_n, S.bigq);
#endif
    if (wib == 0 && nb) {
        for (uint32_t i = 0; i < nb; ++i) {
            const uint32_t r = epi_big_doc(FT, S, GS, arena, off, blk_docs[i], items_all, wave, O, TC);
            ndefer += r & 1u;
            ndef_items += (r >> 3) & 1u;
            ntx += (r >> 1) & 1u;
            nres += (r >> 2) & 1u;
        }
        if (lane == 0) atomicAdd(&S.stats[16], (unsigned long long)nb);
    }
    if (lane == 0) {
        S.kout_cnt[wave] = O.n;
        S.vcnt[wave] = TC.v;
        if (TC.e) atomicAdd(&S.stats[7], (unsigned long long)TC.e);
        S.scnt[wave] = TC.s;
        S.xcnt[wave] = TC.x;
        S.xmark[wave] = TC.x;   // (the regex tasks the epilogue queued: KW_RX_SPLIT's early phase)
        if (TC.v > S.vcap || TC.s > S.scap || TC.x > S.xcap) {
            atomicOr(&S.status[0], ST_TASK_OVERFLOW);
            atomicMax(&S.tmax[0], TC.v);
            atomicMax(&S.tmax[2], TC.s);
            atomicMax(&S.tmax[3], TC.x);
        }
        atomicAdd(&S.stats[4], (unsigned long long)ndefer);
        atomicAdd(&S.stats[5], (unsigned long long)ndef_items);
        if (ntx) atomicAdd(&S.stats[18], (unsigned long long)ntx);
        if (nres) atomicAdd(&S.stats[19], (unsigned long long)nres);
    }
}

}  // namespace kw
