// libkwmatch: host side of the C-ABI declared in include/kwmatch.h.
//
// kw_compile turns the active names of the knowledge base into the device
// tables the scan kernel walks (anchor strings and their uses, the LDS filter,
// the global anchor hash table, bit-parallel match vectors, regex atom
// programs, the short-field substring table).  kw_scan launches the fused
// scan/resolve kernel plus a two-kernel compaction of the per-wave result
// regions.  Reference: match_keywords.py:148-192 (the loops this replaces).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "kwmatch_kernels.hpp"
#include "kwmatch_fast_kernel.hpp"
#include "kwmatch_split.hpp"
#include "kwenv.hpp"

using namespace kw;

// The regex tasks the epilogue queued run beside the verify / short kernels (instead of after them) for KBs of
// at most this many patterns: config 2 (3074) 4.85 -> 4.79 ms; config 4 (52k names, verify-heavy) 9.15 -> 9.37.
#ifndef RX_SPLIT_MAX_PAT
#define RX_SPLIT_MAX_PAT 16384
#endif

// Scratch sizes of one launch configuration (every field only grows over a handle's life).
struct ScratchCaps {
    int nk = 0, nr = 0, ng = 0;            // epilogue, resolve and generic waves (task waves = nk)
    int ns = 0;                            // filter regions (filter waves = probe waves)
    uint32_t item_cap = 0, out_cap = 0;    // per filter region items, per wave result records
    uint32_t cand_cap = 0;                 // per filter region candidates
    uint32_t gi_cap = ITEM_CAP, gc_cap = CP_CAP;   // generic kernel: items per field, code points per field
    int64_t hdr_cap = 0;                   // documents
    uint32_t defer_cap = 0, rx_cap = 0;
    uint32_t vcap = 0, ecap = 0, scap = 0, xcap = 0;   // per scan wave task regions
    uint64_t dsize = 0;                    // decided-set slots (power of two)
    uint64_t tx_cap = 0;                   // bytes of the transcoded view of non-ASCII documents
    bool covers(const ScratchCaps &o) const
    {
        return tx_cap >= o.tx_cap && nk >= o.nk && nr >= o.nr && ng >= o.ng && ns >= o.ns && cand_cap >= o.cand_cap &&
               item_cap >= o.item_cap && out_cap >= o.out_cap && gi_cap >= o.gi_cap && gc_cap >= o.gc_cap &&
               hdr_cap >= o.hdr_cap && defer_cap >= o.defer_cap && rx_cap >= o.rx_cap && vcap >= o.vcap &&
               ecap >= o.ecap && scap >= o.scap && xcap >= o.xcap && dsize >= o.dsize;
    }
    void grow(const ScratchCaps &o)
    {
        nk = std::max(nk, o.nk); nr = std::max(nr, o.nr); ng = std::max(ng, o.ng); ns = std::max(ns, o.ns);
        cand_cap = std::max(cand_cap, o.cand_cap);
        gi_cap = std::max(gi_cap, o.gi_cap); gc_cap = std::max(gc_cap, o.gc_cap);
        item_cap = std::max(item_cap, o.item_cap); out_cap = std::max(out_cap, o.out_cap);
        hdr_cap = std::max(hdr_cap, o.hdr_cap); defer_cap = std::max(defer_cap, o.defer_cap);
        rx_cap = std::max(rx_cap, o.rx_cap); vcap = std::max(vcap, o.vcap); ecap = std::max(ecap, o.ecap);
        scap = std::max(scap, o.scap); xcap = std::max(xcap, o.xcap); dsize = std::max(dsize, o.dsize);
        tx_cap = std::max(tx_cap, o.tx_cap);
    }
};

struct kw_handle {
    int device = 0;
    DevTables T{};
    void *d_tables = nullptr;
    size_t tables_bytes = 0;
    // scratch
    int n_waves = 0;
    uint32_t out_cap = 0;
    DevScratch S{};
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    void *d_small = nullptr;       // status, stats, out_cnt, offsets
    unsigned long long *d_offs = nullptr;
    unsigned long long *d_total = nullptr;   // in d_small: the scan's record count
    // kw_scan_host: library-owned device copies of a host arena / offsets, and the stream they use
    uint8_t *h_arena = nullptr;
    int64_t *h_off = nullptr;
    size_t h_arena_cap = 0, h_off_cap = 0;
    hipStream_t own = nullptr;
    kw_hit *d_hits = nullptr;
    size_t hits_cap = 0;
    // last scan
    const uint8_t *arena = nullptr;
    const int64_t *doc_off = nullptr;
    int64_t n_docs = 0;
    hipStream_t stream = nullptr;
    bool scanned = false;
    bool fetched = false;
    int64_t n_hits = 0;
    unsigned long long stats[KW_N_STATS] = {0};
    int rescans = 0;   // scans of the last kw_scan's batch redone after growing a buffer
    uint32_t rescan_causes = 0;   // the ST_* overflow bits that made them (= the KW_RESCAN_* bits)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    int cus = 256;
    int blocks_per_cu = 2;
    std::string err;
    int n_pat = 0;
    int launched_waves = 0;
    // fast path: scan waves (nk), resolve waves (nr), generic waves (ng)
    FastTables FT{};
    FastScratch FS{};
    int nk = 0, nr = 0, ng = 0;
    uint32_t defer_cap = 0, item_cap = 0, rx_cap = 0;
    bool item_clamped = false;          // this batch's rescans needed more probe items than 32-bit indexes reach
                                        // (FS.item_grow = 0 for its remaining rescans; reset by every kw_scan)
    ScratchCaps caps;
    uint32_t *out_cnt_all = nullptr;   // counts of every result region (scan, task, resolve, generic)
    kw_hit *out_all = nullptr;
    int64_t hdr_cap = 0;
    int resolve_blocks_per_cu = 1;
    int filter_blocks_per_cu = 1, probe_blocks_per_cu = 1, epi_blocks_per_cu = 1;
    int ns = 0;                        // filter regions of the last launch
    hipEvent_t evf = nullptr, evp = nullptr;   // after the filter / probe kernels
    hipStream_t side = nullptr;                // the resolve kernel's stream (beside epilogue + tasks)
    hipStream_t side2 = nullptr;               // the short-field task kernel's stream (beside verify)
    hipStream_t side3 = nullptr;               // the epilogue's regex tasks (beside verify / short; KW_RX_SPLIT)
    hipEvent_t evrx = nullptr;                 // after them (side3)
    hipEvent_t eve = nullptr, evq = nullptr;   // after the epilogue (main); after the short kernel (side2)
    hipEvent_t evs0 = nullptr, evs1 = nullptr, evt = nullptr;   // resolve start / end (side), tasks end
    int n_anchor_fast = 0;
    unsigned long long fstats[16] = {0};
    hipEvent_t evr = nullptr, evg = nullptr;
    unsigned long long tx_need = 0;    // transcoded-view bytes the last scan wanted (the next one's capacity)
    hipEvent_t evx = nullptr;          // after the transcoding kernel (side stream)
};

static thread_local std::string g_err;

#define HIPCHK(h, x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            (h)->err = std::string("HIP error ") + hipGetErrorString(e_) + " at " #x; \
            return KW_EHIP;                                                            \
        }                                                                              \
    } while (0)

// ------------------------------------------------------------------ host tables
namespace {

bool utf8_decode(const uint8_t *s, size_t n, std::vector<uint32_t> &out)
{
    out.clear();
    size_t i = 0;
    while (i < n) {
        uint32_t b = s[i];
        uint32_t len, cp;
        if (b < 0x80) { len = 1; cp = b; }
        else if ((b & 0xE0) == 0xC0) { len = 2; cp = b & 0x1F; }
        else if ((b & 0xF0) == 0xE0) { len = 3; cp = b & 0x0F; }
        else if ((b & 0xF8) == 0xF0) { len = 4; cp = b & 0x07; }
        else return false;
        if (i + len > n) return false;
        for (uint32_t k = 1; k < len; ++k) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        out.push_back(cp);
        i += len;
    }
    return true;
}

size_t utf8_offset(const std::vector<uint32_t> &cps, size_t upto)
{
    size_t b = 0;
    for (size_t i = 0; i < upto; ++i) b += cps[i] < 0x80 ? 1 : cps[i] < 0x800 ? 2 : cps[i] < 0x10000 ? 3 : 4;
    return b;
}

uint32_t kfull_h(uint32_t m)
{
    uint32_t k = 0;
    while (20u * (k + 1) < m) ++k;
    return k;
}

// largest indel distance any window of the partial_ratio family may have and
// still pass 20*d < m+|W|: full windows d = 2k, edge
// windows |W| = m-1 give floor((2m-2)/20).
uint32_t dmax_h(uint32_t m)
{
    uint32_t a = 2 * kfull_h(m);
    uint32_t b = m >= 1 ? (2 * m - 2) / 20 : 0;
    return a > b ? a : b;
}

// ------------------------------------------------------------------ fast-path tables
// 4-byte q-gram counts of the background sample (the corpus statistics every
// anchor choice is priced with).  Without a sample every count is 0 and a
// character-class heuristic breaks the ties.
struct QStats {
    std::unordered_map<uint32_t, uint32_t> c4;
    bool have = false;
    uint32_t count(const uint8_t *p) const
    {
        const uint32_t k = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        auto it = c4.find(k);
        uint32_t c = it == c4.end() ? 0u : it->second;
        // class heuristic: starting inside a lowercase word or on a space is common in prose
        const uint8_t b = p[0];
        const uint32_t h = (b >= 'a' && b <= 'z') ? 4u : (b == ' ' ? 2u : 0u);
        return have ? 4 * c + h : h;
    }
};

struct FastBuild {
    std::vector<uint32_t> s1, p2, l2, t3, b2, edge_pre, edge_suf;
    int has_short = 0;
    int has_t3 = 0;
    uint32_t gate[6] = {0, 0, 0, 0, 0, 0};   // stage-1 pair box (FastTables::gate)
    std::vector<uint64_t> ht_key, as_head, sig, bsig;
    std::vector<uint32_t> ht_begin, ht_cnt, kl, as_len, as_use_begin, as_use_cnt, use_pat, use_info0, use_info1,
        rxk, boff;
    uint32_t ht_mask = 0;
    std::unordered_map<uint64_t, std::vector<uint32_t>> edge;   // one-deletion variants
    std::vector<uint64_t> edge_key;
    std::vector<uint32_t> edge_begin, edge_cnt, edge_ent;
    uint32_t edge_mask = 0;
    std::vector<uint32_t> ht4, arec, urec, urec2;   // merged probe records (4 x u32 each)
    std::vector<int32_t> rxf_idx;
    std::vector<uint64_t> rxf_pm, rxf_any, rxf_ext_mask;
    std::vector<uint32_t> rxf_len, rxf_ext_off, rxf_ext_cp;
    std::vector<uint8_t> rx_bytes;                  // RXM program strings (after the names in the device bytes)
    std::vector<uint32_t> use_rxs, rxl;             // per use: RXM string offset (~0: none); per pattern: RXM length
    std::vector<uint64_t> use_wild;                 // per use: wildcard positions of an RXM string
};

// rarest 4-byte window inside bytes [lo, hi) (hi - lo >= 4); returns its start
size_t rarest4(const QStats &Q, const uint8_t *s, size_t lo, size_t hi, size_t max_start)
{
    size_t best = lo;
    uint32_t bc = 0xFFFFFFFFu;
    for (size_t a = lo; a + 4 <= hi && a <= max_start; ++a) {
        uint32_t c = Q.count(s + a);
        if (c < bc) { bc = c; best = a; }
    }
    return best;
}

int build_fast(FastBuild &B, const QStats &Q, int n_pat, const uint8_t *pat_bytes, const int64_t *pat_off,
               const std::vector<std::vector<uint32_t>> &cps, const std::vector<std::vector<uint32_t>> &tcps,
               const std::vector<uint32_t> &pat_info,
               const std::vector<int4> &atoms, const std::vector<uint32_t> &rxo, std::string &err)
{
    struct Use { uint32_t pat, i0, i1; uint32_t rxs = 0xFFFFFFFFu; uint64_t wild = 0; };   // rxs: RXM string offset
    std::unordered_map<std::string, uint32_t> aid;
    std::vector<std::string> astr;
    std::vector<std::vector<Use>> auses;
    auto add = [&](const std::string &a, Use u) {
        auto it = aid.find(a);
        uint32_t id;
        if (it == aid.end()) { id = (uint32_t)astr.size(); aid.emplace(a, id); astr.push_back(a); auses.emplace_back(); }
        else id = it->second;
        auses[id].push_back(u);
    };
    B.rxk.assign(std::max(n_pat, 1), RXK_LITERAL);
    B.rxf_idx.assign(std::max(n_pat, 1), -1);
    B.edge_pre.assign(FK_EDGE_WORDS, 0);
    B.edge_suf.assign(FK_EDGE_WORDS, 0);
    B.boff.assign(std::max(n_pat, 1), 0);
    B.rxl.assign(std::max(n_pat, 1), 0);
    struct RxmTodo { uint32_t pat, L; uint64_t wild; std::string rs; };
    std::vector<RxmTodo> rxm_todo;   // quantifier-free ASCII regex programs: RXM uses once every anchor is known
    B.sig.assign(std::max(n_pat, 1), 0);
    B.bsig.assign(2 * (size_t)std::max(n_pat, 1), 0);
    for (int i = 0; i < n_pat; ++i) {
        const uint8_t *s = pat_bytes + pat_off[i];
        const size_t bl = (size_t)(pat_off[i + 1] - pat_off[i]);
        B.boff[i] = (uint32_t)pat_off[i];
        const uint32_t m = (uint32_t)cps[i].size();
        const bool fuzzy = pat_info[i] & PI_FUZZY;
        for (uint32_t c : cps[i]) B.sig[i] |= 1ull << (c & 63);
        for (uint32_t c : tcps[i]) B.sig[i] |= 1ull << (c & 63);   // (the transcoded view's bytes too)
        for (size_t j = 0; j + 1 < tcps[i].size(); ++j) {
            const uint32_t h = fk_bg_bit(tcps[i][j], tcps[i][j + 1]);
            B.bsig[2 * (size_t)i + (h >> 6)] |= 1ull << (h & 63);
        }
        // whole-name use (U or FULL): anchor at the rarest 4-byte window (offset <= 255)
        auto span_use = [&](uint32_t kind, size_t sb, size_t se, uint32_t pcp, uint32_t pcl) {
            const size_t len = se - sb;
            size_t a = 0, al = len;
            if (len >= 4) {
                a = rarest4(Q, s + sb, 0, len, 255) ;
                al = std::min<size_t>(8, len - a);
            }
            Use u;
            u.pat = (uint32_t)i;
            u.i0 = kind | ((uint32_t)a << 8) | ((uint32_t)sb << 16);
            u.i1 = (uint32_t)len | (pcp << 16) | (pcl << 24);
            add(std::string((const char *)s + sb + a, al), u);
        };
        if (!fuzzy) { span_use(FU_UPPER, 0, bl, 0, 0); continue; }
        if (m == 0) continue;
        span_use(FU_FULL, 0, bl, 0, 0);
        // positions: literal search, or the regex engine after the decision
        if (rxo[i + 1] > rxo[i]) {
            B.rxk[i] = RXK_REGEX;
            // quantifier-free programs of <= 64 atoms take the shift-and search
            bool fixed = rxo[i + 1] - rxo[i] <= 64;
            for (uint32_t a = rxo[i]; a < rxo[i + 1] && fixed; ++a) fixed = atoms[a].z == 1 && atoms[a].w == 1;
            if (fixed) {
                const uint32_t r = (uint32_t)B.rxf_len.size();
                B.rxf_idx[i] = (int32_t)r;
                B.rxf_len.push_back(rxo[i + 1] - rxo[i]);
                uint64_t any = 0;
                std::vector<std::pair<uint32_t, uint64_t>> ext;
                B.rxf_pm.resize((size_t)(r + 1) * 128, 0);
                for (uint32_t a = rxo[i]; a < rxo[i + 1]; ++a) {
                    const uint64_t bit = 1ull << (a - rxo[i]);
                    if (atoms[a].x == KW_RX_ANY) { any |= bit; continue; }
                    const uint32_t c = (uint32_t)atoms[a].y;
                    if (c < 128) { B.rxf_pm[(size_t)r * 128 + c] |= bit; continue; }
                    size_t k = 0;
                    while (k < ext.size() && ext[k].first != c) ++k;
                    if (k == ext.size()) ext.emplace_back(c, 0);
                    ext[k].second |= bit;
                }
                for (uint32_t c = 0; c < 128; ++c)
                    if (c != '\n') B.rxf_pm[(size_t)r * 128 + c] |= any;   // '.' matches anything but '\n'
                B.rxf_any.push_back(any);
                B.rxf_ext_off.push_back((uint32_t)B.rxf_ext_cp.size());
                for (auto &e : ext) { B.rxf_ext_cp.push_back(e.first); B.rxf_ext_mask.push_back(e.second); }
                // an RXM use: the program as a byte string with '.' wildcards (ASCII atoms only), anchored at
                // its rarest 4-byte window of literals; the probe's RXM items are then exactly the program's
                // matches in an ASCII field (re.finditer positions without a search over the field)
                const uint32_t L = rxo[i + 1] - rxo[i];
                bool ascii_prog = true;
                std::string rs(L, '\0');
                uint64_t wild = 0;
                for (uint32_t a = rxo[i]; a < rxo[i + 1]; ++a) {
                    const uint32_t k = a - rxo[i];
                    if (atoms[a].x == KW_RX_ANY) { wild |= 1ull << k; continue; }
                    if ((uint32_t)atoms[a].y >= 128u || atoms[a].y == 0) ascii_prog = false;
                    rs[k] = (char)atoms[a].y;
                }
                if (ascii_prog) rxm_todo.push_back({(uint32_t)i, L, wild, rs});
            }
        }
        // m <= 20: interior windows must be exact (FULL); the one-deletion edge
        // windows (11 <= m <= 20) go to the edge table instead of pieces
        if (kfull_h(m) == 0) {
            if (m >= EDGE_MIN_M && m <= EDGE_MAX_M) {
                for (uint32_t del = 0; del < m; ++del) {
                    if (del > 0 && cps[i][del] == cps[i][del - 1]) continue;   // same variant as del-1
                    // keyed by the code points (resolve kernel) and, for non-ASCII names, by the transcoded
                    // view's bytes (epilogue); every lookup compares the candidate exactly
                    for (int view = 0; view < 2; ++view) {
                        const auto &cv = view ? tcps[i] : cps[i];
                        if (view && cv == cps[i]) break;
                        uint64_t hh = 0;
                        for (uint32_t j = 0; j < m; ++j)
                            if (j != del) hh = hh * SUB_B + cv[j];
                        const uint64_t key = (hh + (uint64_t)(m - 1) * 0x9E3779B97F4A7C15ull) | 1ull;
                        auto &ev = B.edge[key];
                        if (ev.empty() || ev.back() != (((uint32_t)i << 5) | del)) ev.push_back(((uint32_t)i << 5) | del);
                    }
                    // prefilter keys: first / last eight UTF-8 bytes of the variant (>= 10 code points)
                    std::string v;
                    v.append((const char *)s, utf8_offset(cps[i], del));
                    v.append((const char *)s + utf8_offset(cps[i], del + 1), bl - utf8_offset(cps[i], del + 1));
                    const uint8_t *vp = (const uint8_t *)v.data();
                    uint64_t kp = 0, ks = 0;
                    const uint8_t *ve = vp + v.size() - 8;
                    for (int k = 0; k < 8; ++k) {
                        kp |= (uint64_t)vp[k] << (8 * k);
                        ks |= (uint64_t)ve[k] << (8 * k);
                    }
                    B.edge_pre[fk_edge_index(kp) >> 5] |= 1u << (fk_edge_index(kp) & 31);
                    B.edge_suf[fk_edge_index(ks) >> 5] |= 1u << (fk_edge_index(ks) & 31);
                }
            }
            continue;
        }
        // pigeonhole pieces: K = dmax+1 pieces, cuts chosen to minimise the
        // largest "rarest 4-gram" count over the pieces (each piece is anchored
        // at its own rarest 4-gram)
        const uint32_t dm = dmax_h(m);
        if (dm == 0) continue;
        const uint32_t K = dm + 1;
        std::vector<size_t> boffs(m + 1);
        for (uint32_t c = 0; c <= m; ++c) boffs[c] = utf8_offset(cps[i], c);
        const uint32_t minlen = 4;
        if (m < K * minlen) { err = "kw_compile: name too short for its pieces"; return KW_EUNSUPPORTED; }
        // cost[a][b] for piece cps [a, b)
        std::vector<uint32_t> cost((size_t)(m + 1) * (m + 1), 0xFFFFFFFFu);
        for (uint32_t a = 0; a < m; ++a) {
            uint32_t best = 0xFFFFFFFFu;
            for (uint32_t b = a + 1; b <= m; ++b) {
                // add the 4-byte windows that end inside cp b-1
                size_t lo_b = boffs[a];
                for (size_t w = (boffs[b - 1] >= 3 ? boffs[b - 1] - 3 : 0); w + 4 <= boffs[b]; ++w)
                    if (w >= lo_b) best = std::min(best, Q.count(s + w));
                if (boffs[b] - boffs[a] >= 4) cost[(size_t)a * (m + 1) + b] = best;
            }
        }
        const uint32_t INF = 0xFFFFFFFFu;
        // dp[k][a]: best (max cost) splitting cps [a, m) into k pieces
        std::vector<uint32_t> dp((size_t)(K + 1) * (m + 1), INF), nxt((size_t)(K + 1) * (m + 1), 0);
        for (uint32_t a = 0; a + minlen <= m; ++a) dp[(size_t)1 * (m + 1) + a] = cost[(size_t)a * (m + 1) + m];
        for (uint32_t k = 2; k <= K; ++k)
            for (uint32_t a = 0; a + k * minlen <= m; ++a)
                for (uint32_t b = a + minlen; b + (k - 1) * minlen <= m; ++b) {
                    const uint32_t c1 = cost[(size_t)a * (m + 1) + b], c2 = dp[(size_t)(k - 1) * (m + 1) + b];
                    if (c1 == INF || c2 == INF) continue;
                    const uint32_t v = std::max(c1, c2);
                    if (v < dp[(size_t)k * (m + 1) + a]) { dp[(size_t)k * (m + 1) + a] = v; nxt[(size_t)k * (m + 1) + a] = b; }
                }
        if (dp[(size_t)K * (m + 1)] == INF) { err = "kw_compile: no piece split"; return KW_EUNSUPPORTED; }
        uint32_t a = 0;
        for (uint32_t k = K; k >= 1; --k) {
            const uint32_t b = (k == 1) ? m : nxt[(size_t)k * (m + 1) + a];
            span_use(FU_PIECE, boffs[a], boffs[b], a, b - a);
            a = b;
        }
    }
    // ---- RXM uses: anchored at a window of literals whose first four bytes already key another anchor (the
    // filters pass nothing new; the probe checks one more use there), the rarest such window
    {
        std::unordered_map<uint32_t, int> pre4;
        for (const auto &st : astr)
            if (st.size() >= 4) pre4[*(const uint32_t *)st.data()] = 1;
        for (const auto &t : rxm_todo) {
            size_t best = SIZE_MAX;
            uint32_t bc = 0xFFFFFFFFu;
            for (size_t w = 0; w + 4 <= t.L && w <= 255; ++w) {
                if ((t.wild >> w) & 0xFull) continue;
                if (!pre4.count(*(const uint32_t *)(t.rs.data() + w))) continue;
                const uint32_t c = Q.count((const uint8_t *)t.rs.data() + w);
                if (c < bc) { bc = c; best = w; }
            }
            if (best == SIZE_MAX) continue;   // (its positions come from the regex tasks' search)
            size_t al = 4;
            while (al < 8 && best + al < t.L && !((t.wild >> (best + al)) & 1ull)) ++al;
            Use u;
            u.pat = t.pat;
            u.i0 = FU_RXM | ((uint32_t)best << 8);
            u.i1 = t.L;
            u.rxs = (uint32_t)B.rx_bytes.size();
            u.wild = t.wild;
            B.rx_bytes.insert(B.rx_bytes.end(), t.rs.begin(), t.rs.end());
            B.rxl[t.pat] = t.L;
            add(t.rs.substr(best, al), u);
        }
    }
    // ---- anchors, uses
    const uint32_t na = (uint32_t)astr.size();
    for (uint32_t a = 0; a < na; ++a) {
        const std::string &st = astr[a];
        uint64_t hd = 0;
        for (size_t k = 0; k < st.size() && k < 8; ++k) hd |= (uint64_t)(uint8_t)st[k] << (8 * k);
        B.as_head.push_back(hd);
        B.as_len.push_back((uint32_t)st.size());
        B.as_use_begin.push_back((uint32_t)B.use_pat.size());
        B.as_use_cnt.push_back((uint32_t)auses[a].size());
        for (auto &u : auses[a]) {
            B.use_pat.push_back(u.pat);
            B.use_info0.push_back(u.i0);
            B.use_info1.push_back(u.i1);
            B.use_rxs.push_back(u.rxs);
            B.use_wild.push_back(u.wild);
        }
    }
    if (B.use_pat.size() > IT_USE_MASK) { err = "kw_compile: more than 2^19 anchor uses"; return KW_EUNSUPPORTED; }
    // ---- LDS filters (stage 1: 4-gram table + exact pair table; stage 2: l2 / t3 / b2), global hash table
    B.s1.assign(FK_S1_WORDS, 0);
    B.p2.assign(FK_P2_WORDS, 0);
    B.l2.assign(FK_L2_WORDS, 0);
    B.t3.assign(FK_T3_WORDS, 0);
    B.b2.assign(FK_B2_WORDS, 0);
    std::unordered_map<uint64_t, std::vector<uint32_t>> keys;
    uint32_t s1_ext = 0;                         // 4-grams the fuzzy 3-byte anchors added to the stage-1 table
    uint32_t box[4] = {255u, 0u, 255u, 0u};      // first byte lo / hi, second byte lo / hi of the boxed anchors
    for (uint32_t a = 0; a < na; ++a) {
        const std::string &st = astr[a];
        const uint8_t *p = (const uint8_t *)st.data();
        if (st.size() >= 4) {
            const uint32_t k4 = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
            const uint32_t h1 = fk_s1_hash(k4);
            B.s1[fk_s1_word(h1)] |= 1u << (h1 & 31);
            B.l2[fk_l2_index(k4) >> 5] |= 1u << (fk_l2_index(k4) & 31);
            keys[(4ull << 32) | k4].push_back(a);
        } else if (st.size() >= 2) {
            const uint32_t k2 = (uint32_t)p[0] | ((uint32_t)p[1] << 8);
            B.p2[fk_b2_index(k2) >> 5] |= 1u << (fk_b2_index(k2) & 31);
            // stage 1: a fuzzy 3-byte anchor (a whole name, found anywhere) as the 256 4-grams that start with
            // it while their number is small; every other short anchor (the uppercase names' whole 2-3 bytes)
            // through the pair box
            bool upper_only = true;
            for (const auto &u : auses[a]) upper_only = upper_only && (u.i0 & 0xFFu) == FU_UPPER;
            if (st.size() == 3 && !upper_only && s1_ext < FK_S1_EXT_MAX) {
                for (uint32_t x = 0; x < 256; ++x) {
                    const uint32_t k4 = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | (x << 24);
                    const uint32_t h1 = fk_s1_hash(k4);
                    B.s1[fk_s1_word(h1)] |= 1u << (h1 & 31);
                }
                s1_ext += 256;
            } else {
                box[0] = std::min<uint32_t>(box[0], p[0]);
                box[1] = std::max<uint32_t>(box[1], p[0]);
                box[2] = std::min<uint32_t>(box[2], p[1]);
                box[3] = std::max<uint32_t>(box[3], p[1]);
                B.has_short = 1;
            }
            if (st.size() == 3) {
                const uint32_t k3 = k2 | ((uint32_t)p[2] << 16);
                B.t3[fk_t3_index(k3) >> 5] |= 1u << (fk_t3_index(k3) & 31);
                B.has_t3 = 1;
                keys[(3ull << 32) | k3].push_back(a);
            } else {
                B.b2[fk_b2h_index(k2) >> 5] |= 1u << (fk_b2h_index(k2) & 31);
                keys[(2ull << 32) | k2].push_back(a);
            }
        } else {
            err = "kw_compile: one-byte anchor";
            return KW_EUNSUPPORTED;
        }
    }
    // the box as SWAR range constants per byte: bytes < 0x80 in [lo, hi] by two additions, bytes >= 0x80 all
    // in (one flag) when the range reaches them
    if (B.has_short) {
        for (int r = 0; r < 2; ++r) {
            const uint32_t lo = box[2 * r], hi = box[2 * r + 1];
            const uint32_t alo = std::min(lo, 0x80u), ahi = std::min(hi, 0x7Fu);
            const uint32_t A = alo <= ahi ? 0x80u - alo : 0u, Bc = alo <= ahi ? 0x7Fu - ahi : 0u;
            B.gate[3 * r] = A * 0x01010101u;
            B.gate[3 * r + 1] = Bc * 0x01010101u;
            B.gate[3 * r + 2] = hi >= 0x80u ? 0x80808080u : 0u;
        }
    }
    // open addressing with linear probing: a candidate whose key is absent (most stage-2 survivors of the
    // shorter key lengths) walks to an empty slot, one dependent load per slot; KW_HT_SCALE = slots per key
    // (4: config 2 4.64-4.67 -> 4.60-4.62 ms, probe 1.11 -> 1.08; config 4 probe 1.78 -> 1.74; 8 is no better for
    // config 2 and doubles the table's L2 footprint; r05_ht_scale_ab.txt)
    uint32_t hs = 1024, hscale = 4;
    if (const char *e = kw_env("KW_HT_SCALE")) hscale = (uint32_t)std::max(1, atoi(e));
    while (hs < (size_t)hscale * keys.size()) hs <<= 1;
    B.ht_mask = hs - 1;
    B.ht_key.assign(hs, ~0ull);
    B.ht_begin.assign(hs, 0);
    B.ht_cnt.assign(hs, 0);
    for (auto &kv : keys) {
        uint32_t slot = fk_ht_slot(kv.first, B.ht_mask);
        while (B.ht_key[slot] != ~0ull) slot = (slot + 1) & B.ht_mask;
        B.ht_key[slot] = kv.first;
        B.ht_begin[slot] = (uint32_t)B.kl.size();
        B.ht_cnt[slot] = (uint32_t)kv.second.size();
        B.kl.insert(B.kl.end(), kv.second.begin(), kv.second.end());
    }
    if (B.kl.empty()) B.kl.push_back(0);
    // merged records for the scan's probe: slot {key lo, key hi, first anchor record, count} ->
    // anchor record {head lo, head hi, first use, uses << 8 | len} -> use {info0, info1, pattern, byte offset of the span}
    B.ht4.assign((size_t)hs * 4, 0);
    for (uint32_t sl = 0; sl < hs; ++sl) {
        B.ht4[4 * sl] = (uint32_t)B.ht_key[sl];
        B.ht4[4 * sl + 1] = (uint32_t)(B.ht_key[sl] >> 32);
        B.ht4[4 * sl + 2] = B.ht_begin[sl];
        B.ht4[4 * sl + 3] = B.ht_cnt[sl];
    }
    for (uint32_t a : B.kl) {
        if (B.as_len.empty()) break;
        if (B.as_use_cnt[a] >= (1u << 24)) { err = "kw_compile: anchor with more than 2^24 uses"; return KW_EUNSUPPORTED; }
        B.arec.push_back((uint32_t)B.as_head[a]);
        B.arec.push_back((uint32_t)(B.as_head[a] >> 32));
        B.arec.push_back(B.as_use_begin[a]);
        B.arec.push_back((B.as_use_cnt[a] << 8) | B.as_len[a]);
    }
    const uint32_t rx_base = (uint32_t)(n_pat ? pat_off[n_pat] : 0) + 16;   // RXM strings follow the names (+16 pad)
    for (size_t u = 0; u < B.use_pat.size(); ++u) {
        const bool rxm = B.use_rxs[u] != 0xFFFFFFFFu;
        const uint32_t sb = rxm ? rx_base + B.use_rxs[u] : B.boff[B.use_pat[u]] + (B.use_info0[u] >> 16);
        const uint32_t sl = B.use_info1[u] & 0xFFFF;
        const uint8_t *sp = rxm ? B.rx_bytes.data() + B.use_rxs[u] : pat_bytes + sb;
        B.urec.push_back(B.use_info0[u]);
        B.urec.push_back(B.use_info1[u]);
        B.urec.push_back(B.use_pat[u]);
        B.urec.push_back(sb);
        // first and last (up to) 8 bytes of the span: spans of <= 16 bytes need no other compare
        uint64_t hd = 0, tl = 0;
        const uint32_t hl = sl < 8 ? sl : 8;
        for (uint32_t k = 0; k < hl; ++k) hd |= (uint64_t)sp[k] << (8 * k);
        for (uint32_t k = 0; k < hl; ++k) tl |= (uint64_t)sp[sl - hl + k] << (8 * k);
        B.urec2.push_back((uint32_t)hd);
        B.urec2.push_back((uint32_t)(hd >> 32));
        B.urec2.push_back((uint32_t)tl);
        B.urec2.push_back((uint32_t)(tl >> 32));
    }
    if (B.urec2.empty()) B.urec2.assign(4, 0);
    if (B.arec.empty()) B.arec.assign(4, 0);
    if (B.urec.empty()) B.urec.assign(4, 0);
    {
        uint32_t es = 256;
        while (es < 2 * B.edge.size()) es <<= 1;
        B.edge_mask = es - 1;
        B.edge_key.assign(es, 0);
        B.edge_begin.assign(es, 0);
        B.edge_cnt.assign(es, 0);
        for (auto &kv : B.edge) {
            uint32_t slot = (uint32_t)(kv.first >> 32) & B.edge_mask;
            while (B.edge_key[slot] != 0) slot = (slot + 1) & B.edge_mask;
            B.edge_key[slot] = kv.first;
            B.edge_begin[slot] = (uint32_t)B.edge_ent.size();
            B.edge_cnt[slot] = (uint32_t)kv.second.size();
            B.edge_ent.insert(B.edge_ent.end(), kv.second.begin(), kv.second.end());
        }
        if (B.edge_ent.empty()) B.edge_ent.push_back(0);
    }
    B.rxf_ext_off.push_back((uint32_t)B.rxf_ext_cp.size());
    if (B.rxf_len.empty()) { B.rxf_len.push_back(1); B.rxf_any.push_back(0); B.rxf_pm.resize(128, 0); }
    if (B.rxf_ext_cp.empty()) { B.rxf_ext_cp.push_back(0); B.rxf_ext_mask.push_back(0); }
    if (B.as_head.empty()) { B.as_head.push_back(0); B.as_len.push_back(0); B.as_use_begin.push_back(0); B.as_use_cnt.push_back(0); }
    if (B.use_pat.empty()) { B.use_pat.push_back(0); B.use_info0.push_back(0); B.use_info1.push_back(0); }
    if (B.use_wild.empty()) { B.use_wild.push_back(0); B.use_rxs.push_back(0xFFFFFFFFu); }
    return KW_OK;
}

bool is_word_h(const uint32_t *bits, uint32_t c)
{
    if (c >= 0x110000u) return false;
    return (bits[c >> 5] >> (c & 31)) & 1u;
}

template <class T>
size_t push_array(std::vector<uint8_t> &blob, const std::vector<T> &v)
{
    size_t off = (blob.size() + 255) & ~size_t(255);
    blob.resize(off + v.size() * sizeof(T) + 16);
    if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

}  // namespace

extern "C" int kw_compile(const uint8_t *pat_bytes, const int64_t *pat_off, const uint8_t *pat_class, int32_t n_pat,
                          const int32_t *rx_atoms, const int64_t *rx_off, const uint32_t *word_bitmap,
                          const uint8_t *bg, int64_t bg_len, int32_t device, kw_handle **out)
{
    if (!out) return KW_EINVAL;
    *out = nullptr;
    kw_handle *h = new kw_handle();
    auto fail = [&](int code, const std::string &msg) {
        g_err = msg;
        h->err = msg;
        *out = h;   // caller can read kw_last_error, then kw_destroy
        return code;
    };
    if (n_pat < 0 || (n_pat > 0 && (!pat_bytes || !pat_off || !pat_class)) || !word_bitmap)
        return fail(KW_EINVAL, "kw_compile: null argument");
    if (n_pat >= (1 << 20)) return fail(KW_EUNSUPPORTED, "kw_compile: more than 2^20 patterns");
    h->device = device;
    h->n_pat = n_pat;

    // ---- patterns
    std::vector<std::vector<uint32_t>> cps(n_pat);
    std::vector<uint32_t> pat_info(n_pat), pat_cp_off(n_pat + 1), pat_cps;
    int f_first = n_pat, empty_pat = -1;
    int prev_m = 1 << 30;
    for (int i = 0; i < n_pat; ++i) {
        const uint8_t *s = pat_bytes + pat_off[i];
        size_t bl = (size_t)(pat_off[i + 1] - pat_off[i]);
        if (!utf8_decode(s, bl, cps[i])) return fail(KW_EINVAL, "kw_compile: pattern " + std::to_string(i) + " is not valid UTF-8");
        uint32_t m = (uint32_t)cps[i].size();
        const bool fuzzy = pat_class[i] == KW_CLASS_FUZZY;
        if (!fuzzy && pat_class[i] != KW_CLASS_UPPER) return fail(KW_EINVAL, "kw_compile: bad class of pattern " + std::to_string(i));
        if (fuzzy) {
            if (f_first == n_pat) f_first = i;
            if ((int)m > prev_m) return fail(KW_EINVAL, "kw_compile: fuzzy patterns must be sorted by length, longest first");
            prev_m = (int)m;
            if (m > (uint32_t)MAXM)
                return fail(KW_EUNSUPPORTED,
                            "kw_compile: fuzzy name '" + std::string((const char *)s, bl) + "' (pattern " + std::to_string(i) +
                                ") is longer than 64 code points: rapidfuzz's partial_ratio switches to a matching-blocks "
                                "heuristic for needles over 64 whose score is not the window-family maximum restated "
                                "here, and rapidfuzz is absent from this image, so no result for it could be checked");
            if (bl == 1) return fail(KW_EUNSUPPORTED, "kw_compile: one-byte fuzzy names are not supported");
            if (m == 0) empty_pat = i;
        } else {
            if (f_first != n_pat) return fail(KW_EINVAL, "kw_compile: uppercase patterns must precede fuzzy ones");
            if (m < 2) return fail(KW_EINVAL, "kw_compile: uppercase names have at least 2 code points");
            if (m > 255) return fail(KW_EUNSUPPORTED, "kw_compile: uppercase name longer than 255 code points");
        }
        if (bl > 65535) return fail(KW_EUNSUPPORTED, "kw_compile: name longer than 65535 bytes");
        uint32_t pi = (fuzzy ? PI_FUZZY : 0u) | (m << 8) | ((uint32_t)bl << 16) | (bl == m ? PI_ASCII : 0u);
        if (!fuzzy) {
            if (is_word_h(word_bitmap, cps[i].front())) pi |= PI_WORD_FIRST;
            if (is_word_h(word_bitmap, cps[i].back())) pi |= PI_WORD_LAST;
        }
        pat_info[i] = pi;
        pat_cp_off[i] = (uint32_t)pat_cps.size();
        pat_cps.insert(pat_cps.end(), cps[i].begin(), cps[i].end());
    }
    pat_cp_off[n_pat] = (uint32_t)pat_cps.size();

    // ---- regex programs
    std::vector<int4> atoms;
    std::vector<uint32_t> rxo(n_pat + 1, 0);
    for (int i = 0; i < n_pat; ++i) {
        rxo[i] = (uint32_t)atoms.size();
        const bool fuzzy = pat_info[i] & PI_FUZZY;
        int64_t a0 = rx_off ? rx_off[i] : 0, a1 = rx_off ? rx_off[i + 1] : 0;
        if (!fuzzy || a1 <= a0 || !rx_atoms) {
            if (fuzzy) pat_info[i] |= PI_LITERAL;
            continue;
        }
        int nq = 0, minsum = 0;
        for (int64_t a = a0; a < a1; ++a) {
            int4 t;
            t.x = rx_atoms[4 * a]; t.y = rx_atoms[4 * a + 1]; t.z = rx_atoms[4 * a + 2]; t.w = rx_atoms[4 * a + 3];
            if ((t.x != KW_RX_LIT && t.x != KW_RX_ANY) || t.z < 0 || (t.w >= 0 && t.w < t.z))
                return fail(KW_EUNSUPPORTED, "kw_compile: bad regex atom in pattern " + std::to_string(i));
            if (!(t.z == 1 && t.w == 1)) ++nq;
            minsum += t.z;
            atoms.push_back(t);
        }
        if (nq > RX_MAX_QUANT) return fail(KW_EUNSUPPORTED, "kw_compile: too many quantified atoms in pattern " + std::to_string(i));
        if (minsum == 0) return fail(KW_EUNSUPPORTED, "kw_compile: regex that can match the empty string in pattern " + std::to_string(i));
    }
    rxo[n_pat] = (uint32_t)atoms.size();
    if (atoms.empty()) atoms.push_back(int4{0, 0, 1, 1});

    // ---- anchor strings and their uses
    std::unordered_map<std::string, uint32_t> as_id;
    std::vector<std::string> as_str;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> as_uses;   // (pat, info)
    auto add_use = [&](const std::string &a, uint32_t pat, uint32_t info) {
        auto it = as_id.find(a);
        uint32_t id;
        if (it == as_id.end()) {
            id = (uint32_t)as_str.size();
            as_id.emplace(a, id);
            as_str.push_back(a);
            as_uses.emplace_back();
        } else {
            id = it->second;
        }
        as_uses[id].emplace_back(pat, info);
    };
    for (int i = 0; i < n_pat; ++i) {
        const std::string full((const char *)pat_bytes + pat_off[i], (size_t)(pat_off[i + 1] - pat_off[i]));
        const uint32_t m = (uint32_t)cps[i].size();
        if (!(pat_info[i] & PI_FUZZY)) {
            add_use(full, (uint32_t)i, USE_UPPER | (m << 16));
            continue;
        }
        if (m == 0) continue;
        add_use(full, (uint32_t)i, USE_FULL | (m << 16));
        uint32_t dm = dmax_h(m);
        if (dm == 0) continue;
        uint32_t K = dm + 1;
        for (uint32_t k = 0; k < K; ++k) {
            uint32_t b = (k * m) / K, e = ((k + 1) * m) / K;
            size_t bb = utf8_offset(cps[i], b), be = utf8_offset(cps[i], e);
            std::string piece = full.substr(bb, be - bb);
            if (piece.size() < 2) return fail(KW_EUNSUPPORTED, "kw_compile: piece shorter than 2 bytes");
            add_use(piece, (uint32_t)i, USE_PIECE | (b << 8) | ((e - b) << 16));
        }
    }
    const uint32_t n_as = (uint32_t)as_str.size();
    std::vector<uint64_t> as_head(n_as);
    std::vector<uint32_t> as_off(n_as), as_len(n_as), as_use_begin(n_as), as_use_cnt(n_as), use_pat, use_info;
    std::vector<uint8_t> as_bytes;
    for (uint32_t a = 0; a < n_as; ++a) {
        const std::string &s = as_str[a];
        uint64_t hd = 0;
        for (size_t k = 0; k < s.size() && k < 8; ++k) hd |= (uint64_t)(uint8_t)s[k] << (8 * k);
        as_head[a] = hd;
        as_off[a] = (uint32_t)as_bytes.size();
        as_len[a] = (uint32_t)s.size();
        as_bytes.insert(as_bytes.end(), s.begin(), s.end());
        as_use_begin[a] = (uint32_t)use_pat.size();
        as_use_cnt[a] = (uint32_t)as_uses[a].size();
        for (auto &u : as_uses[a]) { use_pat.push_back(u.first); use_info.push_back(u.second); }
    }
    if (use_pat.size() > IT_USE_MASK) return fail(KW_EUNSUPPORTED, "kw_compile: more than 2^19 anchor uses");

    // ---- 3-byte keys: LDS filter bits + global hash table key -> anchor list
    std::map<uint32_t, std::vector<uint32_t>> key_anchors;
    for (uint32_t a = 0; a < n_as; ++a) {
        const std::string &s = as_str[a];
        uint32_t b0 = (uint8_t)s[0], b1 = (uint8_t)s[1];
        if (s.size() >= 3) {
            key_anchors[b0 | (b1 << 8) | ((uint32_t)(uint8_t)s[2] << 16)].push_back(a);
        } else {
            for (uint32_t x = 0; x < 256; ++x) key_anchors[b0 | (b1 << 8) | (x << 16)].push_back(a);
        }
    }
    std::vector<uint32_t> filt(FILT_WORDS, 0);
    uint32_t ht_size = 1024;
    while (ht_size < 2 * key_anchors.size()) ht_size <<= 1;
    int ht_log = 0;
    while ((1u << ht_log) < ht_size) ++ht_log;
    std::vector<uint32_t> ht_key(ht_size, 0xFFFFFFFFu), ht_begin(ht_size, 0), ht_cnt(ht_size, 0), kl_anchor;
    for (auto &kv : key_anchors) {
        uint32_t key = kv.first;
        uint32_t hb = (key * HASH_MUL) >> (32 - FILT_BITS);
        filt[hb >> 5] |= 1u << (hb & 31);
        uint32_t slot = (key * HASH_MUL) >> (32 - ht_log);
        while (ht_key[slot] != 0xFFFFFFFFu) slot = (slot + 1) & (ht_size - 1);
        ht_key[slot] = key;
        ht_begin[slot] = (uint32_t)kl_anchor.size();
        ht_cnt[slot] = (uint32_t)kv.second.size();
        kl_anchor.insert(kl_anchor.end(), kv.second.begin(), kv.second.end());
    }
    if (kl_anchor.empty()) kl_anchor.push_back(0);

    // ---- bit-parallel match vectors (needle = name)
    // ---- the epilogue's transcoded view of non-ASCII documents: the non-ASCII code points of the fuzzy names,
    // most frequent first, get the one-byte markers 0x81..0xFF; a name with a code point beyond them, or with
    // quantified regex atoms and a non-ASCII code point, is PI_TXUNSAFE (its documents go to the resolve kernel)
    std::vector<uint32_t> tx_key(256, 0xFFFFFFFFu), tx_val(256, 0x80u), tx_inv(128, 0xFFFFFFFFu);
    std::vector<std::vector<uint32_t>> tcps(n_pat);
    std::vector<uint32_t> pat_tcps;
    std::vector<uint8_t> pat_tbytes;
    int tx_unsafe_short = 0, tx_unsafe_edge = 0;
    std::vector<uint32_t> txu_pat;   // the PI_TXUNSAFE names (the epilogue's short-field test)
    {
        std::map<uint32_t, uint64_t> freq;
        for (int i = f_first; i < n_pat; ++i)
            for (uint32_t c : cps[i])
                if (c >= 0x80) ++freq[c];
        std::vector<std::pair<uint64_t, uint32_t>> order;
        for (auto &kv : freq) order.emplace_back(kv.second, kv.first);
        std::sort(order.begin(), order.end(), [](const auto &a, const auto &b) {
            return a.first != b.first ? a.first > b.first : a.second < b.second;
        });
        size_t nmark = 127;
        if (const char *e = kw_env("KW_TEST_TX_MARKERS")) nmark = std::min<size_t>(127, (size_t)std::max(0, atoi(e)));
        std::unordered_map<uint32_t, uint32_t> mk;
        for (size_t k = 0; k < order.size() && k < nmark; ++k) {
            const uint32_t cp = order[k].second, v = 0x81u + (uint32_t)k;
            mk[cp] = v;
            tx_inv[v - 0x80u] = cp;
            uint32_t slot = (cp * 0x9E3779B1u) >> 24;
            while (tx_key[slot] != 0xFFFFFFFFu) slot = (slot + 1) & 255u;
            tx_key[slot] = cp;
            tx_val[slot] = v;
        }
        for (int i = 0; i < n_pat; ++i) {
            bool unmapped = false;
            tcps[i].reserve(cps[i].size());
            for (uint32_t c : cps[i]) {
                if (c < 0x80) { tcps[i].push_back(c); continue; }
                auto it = mk.find(c);
                unmapped |= it == mk.end();
                tcps[i].push_back(it == mk.end() ? 0x80u : it->second);
            }
            pat_tcps.insert(pat_tcps.end(), tcps[i].begin(), tcps[i].end());
            if (!(pat_info[i] & PI_FUZZY)) continue;
            bool quantified = false;
            for (uint32_t a = rxo[i]; a < rxo[i + 1]; ++a) quantified |= !(atoms[a].z == 1 && atoms[a].w == 1);
            quantified |= rxo[i + 1] - rxo[i] > 64;
            const bool nonascii = !(pat_info[i] & PI_ASCII);
            if (unmapped || (nonascii && quantified)) {
                pat_info[i] |= PI_TXUNSAFE;
                tx_unsafe_short = 1;
                txu_pat.push_back((uint32_t)i);
                const uint32_t m = (uint32_t)cps[i].size();
                if (m >= EDGE_MIN_M && m <= EDGE_MAX_M) tx_unsafe_edge = 1;
            }
        }
        if (pat_tcps.empty()) pat_tcps.push_back(0);
        pat_tbytes.assign(pat_tcps.begin(), pat_tcps.end());   // (every value < 256)
        pat_tbytes.resize(pat_tbytes.size() + 72, 0);          // (unaligned 4-byte reads past a name)
    }

    std::vector<uint64_t> pm_ascii((size_t)std::max(n_pat, 1) * 128, 0);
    std::vector<uint32_t> pm_ext_off(n_pat + 1, 0), pm_ext_cp;
    std::vector<uint64_t> pm_ext_mask;
    for (int i = 0; i < n_pat; ++i) {
        pm_ext_off[i] = (uint32_t)pm_ext_cp.size();
        if (!(pat_info[i] & PI_FUZZY)) continue;
        const auto &c = cps[i];
        size_t ext0 = pm_ext_cp.size();
        for (size_t j = 0; j < c.size(); ++j) {
            if (c[j] < 128) { pm_ascii[(size_t)i * 128 + c[j]] |= 1ull << j; continue; }
            size_t k = ext0;
            while (k < pm_ext_cp.size() && pm_ext_cp[k] != c[j]) ++k;
            if (k == pm_ext_cp.size()) { pm_ext_cp.push_back(c[j]); pm_ext_mask.push_back(0); }
            pm_ext_mask[k] |= 1ull << j;
        }
    }
    pm_ext_off[n_pat] = (uint32_t)pm_ext_cp.size();
    if (pm_ext_cp.empty()) { pm_ext_cp.push_back(0); pm_ext_mask.push_back(0); }

    // ---- short fields: substrings (<= SHORT_EXACT_MAX code points) of fuzzy names
    std::unordered_map<uint64_t, std::vector<uint32_t>> subs;
    for (int i = f_first; i < n_pat; ++i) {
        const auto &c = cps[i];
        // keyed by code points and, for non-ASCII names, by the transcoded view's bytes (exact compare follows)
        for (int view = 0; view < 2; ++view) {
            const auto &cv = view ? tcps[i] : c;
            if (view && cv == c) break;
            for (size_t s0 = 0; s0 < cv.size(); ++s0) {
                uint64_t hh = 0;
                for (size_t l = 1; l <= (size_t)SHORT_EXACT_MAX && s0 + l <= cv.size(); ++l) {
                    hh = hh * SUB_B + cv[s0 + l - 1];
                    uint64_t key = (hh + (uint64_t)l * 0x9E3779B97F4A7C15ull) | 1ull;
                    // entry: pattern | first offset of the substring << 20 (one compare verifies the hash)
                    auto &v = subs[key];
                    if (v.empty() || (v.back() & 0xFFFFFu) != (uint32_t)i) v.push_back((uint32_t)i | ((uint32_t)s0 << 20));
                }
            }
        }
    }
    uint32_t sub_size = 1024;
    while (sub_size < 2 * subs.size()) sub_size <<= 1;
    std::vector<uint64_t> sub_key(sub_size, 0);
    std::vector<uint32_t> sub_begin(sub_size, 0), sub_cnt(sub_size, 0), sub_pat;
    for (auto &kv : subs) {
        uint32_t slot = (uint32_t)(kv.first >> 32) & (sub_size - 1);
        while (sub_key[slot] != 0) slot = (slot + 1) & (sub_size - 1);
        sub_key[slot] = kv.first;
        sub_begin[slot] = (uint32_t)sub_pat.size();
        sub_cnt[slot] = (uint32_t)kv.second.size();
        sub_pat.insert(sub_pat.end(), kv.second.begin(), kv.second.end());
    }
    if (sub_pat.empty()) sub_pat.push_back(0);

    std::vector<int32_t> f_count_ge(MAXM + 2, 0);
    for (int n = 0; n <= MAXM + 1; ++n) {
        int c = 0;
        for (int i = f_first; i < n_pat; ++i) c += ((int)cps[i].size() >= n);
        f_count_ge[n] = c;
    }
    std::vector<uint32_t> wb(word_bitmap, word_bitmap + 0x110000 / 32);
    if (pat_info.empty()) pat_info.push_back(0);
    if (pat_cps.empty()) pat_cps.push_back(0);
    if (use_pat.empty()) { use_pat.push_back(0); use_info.push_back(0); }
    if (as_head.empty()) { as_head.push_back(0); as_off.push_back(0); as_len.push_back(0); as_use_begin.push_back(0); as_use_cnt.push_back(0); }
    if (as_bytes.empty()) as_bytes.push_back(0);

    // ---- fast-path tables (anchors priced with the background sample's q-grams)
    QStats Q;
    if (bg && bg_len >= 4) {
        Q.have = true;
        Q.c4.reserve((size_t)std::min<int64_t>(bg_len, 1 << 22));
        for (int64_t i = 0; i + 4 <= bg_len; ++i) {
            const uint32_t k = (uint32_t)bg[i] | ((uint32_t)bg[i + 1] << 8) | ((uint32_t)bg[i + 2] << 16) |
                               ((uint32_t)bg[i + 3] << 24);
            ++Q.c4[k];
        }
    }
    FastBuild FB;
    {
        std::string ferr;
        int frc = build_fast(FB, Q, n_pat, pat_bytes, pat_off, cps, tcps, pat_info, atoms, rxo, ferr);
        if (frc) return fail(frc, ferr);
    }
    if (const char *dump = kw_env("KW_DUMP_ANCHORS")) {
        // developer aid: one line per anchor use "hex(anchor) pattern kind" (anchor tuning)
        if (FILE *f = fopen(dump, "w")) {
            for (size_t a = 0; a < FB.as_len.size(); ++a)
                for (uint32_t u = FB.as_use_begin[a]; u < FB.as_use_begin[a] + FB.as_use_cnt[a]; ++u) {
                    for (uint32_t k = 0; k < std::min<uint32_t>(FB.as_len[a], 8); ++k)
                        fprintf(f, "%02x", (unsigned)((FB.as_head[a] >> (8 * k)) & 0xFF));
                    fprintf(f, " %u %u\n", FB.use_pat[u], FB.use_info0[u] & 0xFF);
                }
            fclose(f);
        }
    }
    std::vector<uint8_t> all_bytes(pat_bytes, pat_bytes + (n_pat ? pat_off[n_pat] : 0));
    all_bytes.resize(all_bytes.size() + 16, 0);
    all_bytes.insert(all_bytes.end(), FB.rx_bytes.begin(), FB.rx_bytes.end());   // RXM strings (build_fast's rx_base)
    all_bytes.resize(all_bytes.size() + 16, 0);

    // ---- one device blob
    std::vector<uint8_t> blob;
    size_t o_filt = push_array(blob, filt), o_htk = push_array(blob, ht_key), o_htb = push_array(blob, ht_begin),
           o_htc = push_array(blob, ht_cnt), o_kl = push_array(blob, kl_anchor), o_ash = push_array(blob, as_head),
           o_aso = push_array(blob, as_off), o_asl = push_array(blob, as_len), o_asub = push_array(blob, as_use_begin),
           o_asuc = push_array(blob, as_use_cnt), o_asb = push_array(blob, as_bytes), o_up = push_array(blob, use_pat),
           o_ui = push_array(blob, use_info), o_pi = push_array(blob, pat_info), o_pco = push_array(blob, pat_cp_off),
           o_pc = push_array(blob, pat_cps), o_pma = push_array(blob, pm_ascii), o_peo = push_array(blob, pm_ext_off),
           o_pec = push_array(blob, pm_ext_cp), o_pem = push_array(blob, pm_ext_mask), o_rxo = push_array(blob, rxo),
           o_rxa = push_array(blob, atoms), o_wb = push_array(blob, wb), o_fc = push_array(blob, f_count_ge),
           o_sk = push_array(blob, sub_key), o_sb = push_array(blob, sub_begin), o_sc = push_array(blob, sub_cnt),
           o_sp = push_array(blob, sub_pat);
    size_t f_s1 = push_array(blob, FB.s1), f_p2 = push_array(blob, FB.p2), f_b2 = push_array(blob, FB.b2), f_l2 = push_array(blob, FB.l2),
           f_t3 = push_array(blob, FB.t3), f_epre = push_array(blob, FB.edge_pre), f_esuf = push_array(blob, FB.edge_suf), f_htk = push_array(blob, FB.ht_key),
           f_htb = push_array(blob, FB.ht_begin), f_htc = push_array(blob, FB.ht_cnt), f_kl = push_array(blob, FB.kl),
           f_ash = push_array(blob, FB.as_head), f_asl = push_array(blob, FB.as_len),
           f_asub = push_array(blob, FB.as_use_begin), f_asuc = push_array(blob, FB.as_use_cnt),
           f_up = push_array(blob, FB.use_pat), f_ui0 = push_array(blob, FB.use_info0),
           f_ui1 = push_array(blob, FB.use_info1), f_rxk = push_array(blob, FB.rxk), f_boff = push_array(blob, FB.boff),
           f_pb = push_array(blob, all_bytes), f_sig = push_array(blob, FB.sig), f_bsig = push_array(blob, FB.bsig),
           f_ek = push_array(blob, FB.edge_key), f_eb = push_array(blob, FB.edge_begin),
           f_ec = push_array(blob, FB.edge_cnt), f_ee = push_array(blob, FB.edge_ent),
           f_rxi = push_array(blob, FB.rxf_idx), f_rxp = push_array(blob, FB.rxf_pm), f_rxa = push_array(blob, FB.rxf_any),
           f_rxl = push_array(blob, FB.rxf_len), f_rxeo = push_array(blob, FB.rxf_ext_off),
           f_rxec = push_array(blob, FB.rxf_ext_cp), f_rxem = push_array(blob, FB.rxf_ext_mask),
           f_ht4 = push_array(blob, FB.ht4), f_arec = push_array(blob, FB.arec), f_urec = push_array(blob, FB.urec),
           f_urec2 = push_array(blob, FB.urec2), f_tcps = push_array(blob, pat_tcps), f_txk = push_array(blob, tx_key),
           f_txv = push_array(blob, tx_val), f_txi = push_array(blob, tx_inv), f_tb = push_array(blob, pat_tbytes),
           f_uw = push_array(blob, FB.use_wild), f_prxl = push_array(blob, FB.rxl), f_txu = push_array(blob, txu_pat);

    HIPCHK(h, hipSetDevice(device));
    HIPCHK(h, hipMalloc(&h->d_tables, blob.size()));
    HIPCHK(h, hipMemcpy(h->d_tables, blob.data(), blob.size(), hipMemcpyHostToDevice));
    h->tables_bytes = blob.size();
    uint8_t *B = (uint8_t *)h->d_tables;
    DevTables &T = h->T;
    T.filt = (const uint32_t *)(B + o_filt);
    T.ht_key = (const uint32_t *)(B + o_htk);
    T.ht_begin = (const uint32_t *)(B + o_htb);
    T.ht_cnt = (const uint32_t *)(B + o_htc);
    T.ht_mask = ht_size - 1;
    T.ht_shift = 32 - ht_log;
    T.kl_anchor = (const uint32_t *)(B + o_kl);
    T.as_head = (const uint64_t *)(B + o_ash);
    T.as_off = (const uint32_t *)(B + o_aso);
    T.as_len = (const uint32_t *)(B + o_asl);
    T.as_use_begin = (const uint32_t *)(B + o_asub);
    T.as_use_cnt = (const uint32_t *)(B + o_asuc);
    T.as_bytes = (const uint8_t *)(B + o_asb);
    T.use_pat = (const uint32_t *)(B + o_up);
    T.use_info = (const uint32_t *)(B + o_ui);
    T.pat_info = (const uint32_t *)(B + o_pi);
    T.pat_cp_off = (const uint32_t *)(B + o_pco);
    T.pat_cps = (const uint32_t *)(B + o_pc);
    T.pm_ascii = (const uint64_t *)(B + o_pma);
    T.pm_ext_off = (const uint32_t *)(B + o_peo);
    T.pm_ext_cp = (const uint32_t *)(B + o_pec);
    T.pm_ext_mask = (const uint64_t *)(B + o_pem);
    T.rx_off = (const uint32_t *)(B + o_rxo);
    T.rx_atoms = (const int4 *)(B + o_rxa);
    T.word_bits = (const uint32_t *)(B + o_wb);
    T.f_count_ge = (const int32_t *)(B + o_fc);
    T.sub_key = (const uint64_t *)(B + o_sk);
    T.sub_begin = (const uint32_t *)(B + o_sb);
    T.sub_cnt = (const uint32_t *)(B + o_sc);
    T.sub_pat = (const uint32_t *)(B + o_sp);
    T.sub_mask = sub_size - 1;
    T.n_pat = n_pat;
    T.f_first = f_first;
    T.empty_pat = empty_pat;

    FastTables &F = h->FT;
    F.s1 = (const uint32_t *)(B + f_s1);
    F.p2 = (const uint32_t *)(B + f_p2);
    F.b2 = (const uint32_t *)(B + f_b2);
    F.l2 = (const uint32_t *)(B + f_l2);
    F.t3 = (const uint32_t *)(B + f_t3);
    F.edge_pre = (const uint32_t *)(B + f_epre);
    F.edge_suf = (const uint32_t *)(B + f_esuf);
    F.has_t3 = FB.has_t3;
    F.has_short = FB.has_short;
    for (int r = 0; r < 6; ++r) F.gate[r] = FB.gate[r];
    F.ht_key = (const uint64_t *)(B + f_htk);
    F.ht_begin = (const uint32_t *)(B + f_htb);
    F.ht_cnt = (const uint32_t *)(B + f_htc);
    F.ht_mask = FB.ht_mask;
    F.kl = (const uint32_t *)(B + f_kl);
    F.as_head = (const uint64_t *)(B + f_ash);
    F.as_len = (const uint32_t *)(B + f_asl);
    F.as_use_begin = (const uint32_t *)(B + f_asub);
    F.as_use_cnt = (const uint32_t *)(B + f_asuc);
    F.use_pat = (const uint32_t *)(B + f_up);
    F.use_info0 = (const uint32_t *)(B + f_ui0);
    F.use_info1 = (const uint32_t *)(B + f_ui1);
    F.pat_info = T.pat_info;
    F.pat_rxk = (const uint32_t *)(B + f_rxk);
    F.pat_boff = (const uint32_t *)(B + f_boff);
    F.pat_bytes = (const uint8_t *)(B + f_pb);
    F.pat_cp_off = T.pat_cp_off;
    F.pat_cps = T.pat_cps;
    F.pat_sig = (const uint64_t *)(B + f_sig);
    F.pat_bsig = (const uint64_t *)(B + f_bsig);
    F.f_count_ge = T.f_count_ge;
    F.sub_key = T.sub_key;
    F.sub_begin = T.sub_begin;
    F.sub_cnt = T.sub_cnt;
    F.sub_pat = T.sub_pat;
    F.sub_mask = T.sub_mask;
    F.edge_key = (const uint64_t *)(B + f_ek);
    F.edge_begin = (const uint32_t *)(B + f_eb);
    F.edge_cnt = (const uint32_t *)(B + f_ec);
    F.edge_ent = (const uint32_t *)(B + f_ee);
    F.edge_mask = FB.edge_mask;
    F.word_bits = T.word_bits;
    F.ht4 = (const uint4 *)(B + f_ht4);
    F.arec = (const uint4 *)(B + f_arec);
    F.urec = (const uint4 *)(B + f_urec);
    F.urec2 = (const uint4 *)(B + f_urec2);
    F.rxf_idx = (const int32_t *)(B + f_rxi);
    F.rxf_pm = (const uint64_t *)(B + f_rxp);
    F.rxf_any = (const uint64_t *)(B + f_rxa);
    F.rxf_len = (const uint32_t *)(B + f_rxl);
    F.rxf_ext_off = (const uint32_t *)(B + f_rxeo);
    F.rxf_ext_cp = (const uint32_t *)(B + f_rxec);
    F.rxf_ext_mask = (const uint64_t *)(B + f_rxem);
    F.f_first = f_first;
    F.empty_pat = empty_pat;
    F.pat_tcps = (const uint32_t *)(B + f_tcps);
    F.pat_tbytes = (const uint8_t *)(B + f_tb);
    F.tx_key = (const uint32_t *)(B + f_txk);
    F.tx_val = (const uint32_t *)(B + f_txv);
    F.tx_inv = (const uint32_t *)(B + f_txi);
    F.tx_unsafe_short = tx_unsafe_short;
    F.txu_pat = (const uint32_t *)(B + f_txu);
    F.n_txu = (uint32_t)txu_pat.size();
    F.use_wild = (const uint64_t *)(B + f_uw);
    F.pat_rxl = (const uint32_t *)(B + f_prxl);
    F.tx_unsafe_edge = tx_unsafe_edge;
    h->n_anchor_fast = (int)FB.as_len.size();

    hipDeviceProp_t prop;
    HIPCHK(h, hipGetDeviceProperties(&prop, device));
    h->cus = prop.multiProcessorCount;
    int bpc = 0;
    HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void *)kw_scan_kernel, BLOCK, kScanLds));
    h->blocks_per_cu = bpc > 0 ? bpc : 1;
    bpc = 0;
    HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void *)kw_resolve_kernel, RK_BLOCK, 0));
    h->resolve_blocks_per_cu = bpc > 0 ? bpc : 1;
    bpc = 0;
    HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void *)kw_filter_kernel, FS_BLOCK, 0));
    h->filter_blocks_per_cu = bpc > 0 ? bpc : 1;
    bpc = 0;
    HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void *)kw_probe_kernel, PK_BLOCK, 0));
    h->probe_blocks_per_cu = bpc > 0 ? bpc : 1;
    bpc = 0;
    HIPCHK(h, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, (const void *)kw_epi_kernel, EK_BLOCK, 0));
    h->epi_blocks_per_cu = bpc > 0 ? bpc : 1;
    {
        // KW_SIDE_PRIO=0..3 (bit 0: the side stream, transcoding beside the probe; bit 1: side2, the short
        // fields beside verify) at the greatest priority.  Default 2 (config 2:
        // 4.64-4.67 vs 4.68-4.69 ms; config 4 unchanged)
        const char *e = kw_env("KW_SIDE_PRIO");
        int sp = e ? atoi(e) : 2, lo = 0, hi = 0;
        HIPCHK(h, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(h, hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, (sp & 1) ? hi : lo));
        HIPCHK(h, hipStreamCreateWithPriority(&h->side2, hipStreamNonBlocking, (sp & 2) ? hi : lo));
        HIPCHK(h, hipStreamCreateWithPriority(&h->side3, hipStreamNonBlocking, (sp & 4) ? hi : lo));
    }
    HIPCHK(h, hipEventCreateWithFlags(&h->eve, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&h->evq, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&h->evrx, hipEventDisableTiming));
    HIPCHK(h, hipEventCreateWithFlags(&h->evx, hipEventDisableTiming));
    HIPCHK(h, hipEventCreate(&h->evs0));
    HIPCHK(h, hipEventCreate(&h->evs1));
    HIPCHK(h, hipEventCreate(&h->evt));
    HIPCHK(h, hipEventCreate(&h->evf));
    HIPCHK(h, hipEventCreate(&h->evp));
    HIPCHK(h, hipEventCreate(&h->ev0));
    HIPCHK(h, hipEventCreate(&h->ev1));
    HIPCHK(h, hipEventCreate(&h->evg));
    HIPCHK(h, hipEventCreate(&h->evr));
    HIPCHK(h, hipEventCreate(&h->ev2));
    *out = h;
    return KW_OK;
}

// (re)allocate scratch.  Result regions, in order: scan waves [0, nk), task waves [nk, 2 nk),
// resolve waves [2 nk, 2 nk + nr), generic waves after them (one count array, one gather).
static int ensure_scratch(kw_handle *h, const ScratchCaps &want)
{
    if (h->d_scratch && h->caps.covers(want)) return KW_OK;
    ScratchCaps c = h->caps;
    c.grow(want);
    if (h->d_scratch) { (void)hipFree(h->d_scratch); h->d_scratch = nullptr; }
    if (h->d_small) { (void)hipFree(h->d_small); h->d_small = nullptr; }
    if (h->d_hits) { (void)hipFree(h->d_hits); h->d_hits = nullptr; }
    const size_t per_items = (size_t)2 * c.gi_cap * sizeof(uint64_t);
    const size_t per_cps = (size_t)c.gc_cap * sizeof(uint32_t);
    const size_t per_blk = (size_t)(c.gc_cap / 16 + 2) * sizeof(uint32_t);
    const size_t per_fblk = (size_t)(CP_CAP / 16 + 2) * sizeof(uint32_t);
    const size_t per_fcps = (size_t)FK_CP_CAP * sizeof(uint32_t);
    const size_t per_out = (size_t)c.out_cap * sizeof(kw_hit);
    const size_t nw = (size_t)2 * c.nk + c.nr + c.ng;
    const size_t per_tasks = (size_t)(c.vcap + c.ecap + c.scap + c.xcap) * 16;
    size_t total = (size_t)c.ng * (per_items + per_cps + per_blk) + (size_t)c.nr * (per_fcps + per_fblk) +
                   nw * per_out + (size_t)c.ns * c.item_cap * 8 + (size_t)c.hdr_cap * 8 + (size_t)c.defer_cap * 8 +
                   (size_t)c.ns * c.cand_cap * 4 + (size_t)c.ns * 4 + (size_t)c.hdr_cap * 12 + 4 * 256 +
                   (size_t)c.nr * c.rx_cap * 16 + (size_t)c.nk * per_tasks + (size_t)c.nk * 16 + c.dsize * 8 +
                   (size_t)c.tx_cap + 64 + (size_t)c.hdr_cap * 16 + (size_t)c.defer_cap * 4 + 35 * 256;
    HIPCHK(h, hipMalloc(&h->d_scratch, total));
    uint8_t *p = (uint8_t *)h->d_scratch;
    auto carve = [&](size_t bytes) { uint8_t *r = p; p += (bytes + 255) & ~(size_t)255; return r; };
    h->S.items = (uint64_t *)carve((size_t)c.ng * per_items);
    h->S.cps = (uint32_t *)carve((size_t)c.ng * per_cps);
    h->S.blkcnt = (uint32_t *)carve((size_t)c.ng * per_blk);
    h->FS.cps = (uint32_t *)carve((size_t)c.nr * per_fcps);
    h->FS.cpbase = (uint32_t *)carve((size_t)c.nr * per_fblk);
    h->S.item_cap = c.gi_cap;
    h->S.cp_cap = c.gc_cap;
    kw_hit *outs = (kw_hit *)carve(nw * per_out);
    h->FS.items = (uint64_t *)carve((size_t)c.ns * c.item_cap * 8);
    h->FS.cand = (uint32_t *)carve((size_t)c.ns * c.cand_cap * 4);
    h->FS.cand_cap = c.cand_cap;
    h->FS.ccnt = (uint32_t *)carve((size_t)c.ns * 4);
    h->FS.ncnt = (uint2 *)carve((size_t)c.hdr_cap * 8);
    h->FS.dflags = (uint32_t *)carve((size_t)c.hdr_cap * 4);
    h->FS.hdr = (uint2 *)carve((size_t)c.hdr_cap * 8);
    h->FS.defer_list = (uint32_t *)carve((size_t)c.defer_cap * 4);
    h->FS.big_list = (uint32_t *)carve((size_t)c.defer_cap * 4);
    h->FS.res_list = (uint32_t *)carve((size_t)c.defer_cap * 4);
    h->FS.rx_tasks = (uint4 *)carve((size_t)c.nr * c.rx_cap * 16);
    h->FS.rx_cap = c.rx_cap;
    h->FS.vq = (uint4 *)carve((size_t)c.nk * c.vcap * 16);
    h->FS.eq = (uint4 *)carve((size_t)c.nk * c.ecap * 16);
    h->FS.sq = (uint4 *)carve((size_t)c.nk * c.scap * 16);
    h->FS.xq = (uint4 *)carve((size_t)c.nk * c.xcap * 16);
    h->FS.vcap = c.vcap;
    h->FS.ecap = c.ecap;
    h->FS.scap = c.scap;
    h->FS.xcap = c.xcap;
    uint32_t *tcnt = (uint32_t *)carve((size_t)c.nk * 20);
    h->FS.vcnt = tcnt;
    h->FS.ecnt = tcnt + c.nk;
    h->FS.scnt = tcnt + 2 * (size_t)c.nk;
    h->FS.xcnt = tcnt + 3 * (size_t)c.nk;
    h->FS.xmark = tcnt + 4 * (size_t)c.nk;
    h->FS.dset = (unsigned long long *)carve(c.dsize * 8);
    h->FS.dmask = c.dsize - 1;
    h->FS.vrec = (uint4 *)carve((size_t)c.hdr_cap * 16);
    h->FS.tarena = (uint8_t *)carve((size_t)c.tx_cap + 64);
    h->FS.tx_cap = c.tx_cap;
    size_t small = 1024 + nw * 4 + 256 + (nw + 1) * 8 + 256;
    HIPCHK(h, hipMalloc(&h->d_small, small));
    uint8_t *q = (uint8_t *)h->d_small;
    h->S.status = (uint32_t *)q;                        // 4 x u32
    h->FS.status = h->S.status;
    h->FS.defer_cnt = (uint32_t *)(q + 16);
    h->FS.big_cnt = (uint32_t *)(q + 20);               // 2 x u32: all-ASCII, non-ASCII big documents
    h->FS.tmax = (uint32_t *)(q + 32);                  // 4 x u32
    h->FS.cmax = (uint32_t *)(q + 48);                  // 2 x u32
    h->S.gmax = (uint32_t *)(q + 56);                   // 2 x u32
    h->S.stats = (unsigned long long *)(q + 64);        // 3 x u64 (generic)
    h->FS.stats = (unsigned long long *)(q + 128);      // 32 x u64 (fast path; 21.. developer counters)
    h->FS.tx_used = (unsigned long long *)(q + 384);    // transcoded-view bytes handed out
    h->FS.res_cnt = (uint32_t *)(q + 392);              // documents left to the resolve kernel
    h->d_total = (unsigned long long *)(q + 400);       // hit records of the scan (kw_offsets_kernel)
    h->FS.gnext = (uint32_t *)(q + 408);                // 2 x u32: the filter's next work unit / the probe's next region
    uint32_t *cnts = (uint32_t *)(q + 1024);
    h->out_cnt_all = cnts;
    h->FS.kout_cnt = cnts;
    h->FS.tout_cnt = cnts + c.nk;
    h->FS.out_cnt = cnts + 2 * (size_t)c.nk;
    h->S.out_cnt = cnts + 2 * (size_t)c.nk + c.nr;
    h->d_offs = (unsigned long long *)(q + 1024 + ((nw * 4 + 255) & ~(size_t)255));
    h->out_all = outs;
    h->FS.kout = outs;
    h->FS.tout = outs + (size_t)c.nk * c.out_cap;
    h->FS.out = outs + (size_t)2 * c.nk * c.out_cap;
    h->S.out = outs + ((size_t)2 * c.nk + c.nr) * c.out_cap;
    h->S.out_cap = c.out_cap;
    h->FS.out_cap = c.out_cap;
    h->FS.item_cap = c.item_cap;
    h->FS.defer_cap = c.defer_cap;
    h->caps = c;
    h->nk = c.nk;
    h->nr = c.nr;
    h->ng = c.ng;
    h->item_cap = c.item_cap;
    h->out_cap = c.out_cap;
    h->hdr_cap = c.hdr_cap;
    h->defer_cap = c.defer_cap;
    h->rx_cap = c.rx_cap;
    h->hits_cap = nw * c.out_cap;
    HIPCHK(h, hipMalloc(&h->d_hits, h->hits_cap * sizeof(kw_hit) + 16));
    h->scratch_bytes = total;
    return KW_OK;
}

// regions x item_cap of the probe's item arrays must index with 32 bits (hdr.x; KW_TEST_ITEM_LIMIT lowers it)
static uint64_t item_index_limit()
{
    if (const char *e = kw_env("KW_TEST_ITEM_LIMIT")) return std::max<uint64_t>(1, (uint64_t)atoll(e));
    return 0xFFFFFFFFull;
}

static int launch_scan(kw_handle *h)
{
    hipStream_t st = h->stream;
    // KW_SERIAL=1 (profiling aid): every kernel on the main stream, so kernel traces show isolated durations
    static const bool serial = kw_env("KW_SERIAL") != nullptr;
    hipStream_t side = serial ? st : h->side, side2 = serial ? st : h->side2, side3 = serial ? st : h->side3;
    const int64_t n_docs = h->n_docs;
    // split scan: filter regions (one wave each, resident at once), probe waves = filter regions,
    // epilogue waves = task regions
    int nsb = (int)std::min<int64_t>((n_docs + FS_WAVES - 1) / FS_WAVES, (int64_t)h->cus * h->filter_blocks_per_cu);
    if (nsb < 1) nsb = 1;
    int neb = (int)std::min<int64_t>((n_docs + EK_WAVES - 1) / EK_WAVES, (int64_t)h->cus * h->epi_blocks_per_cu);
    if (neb < 1) neb = 1;
    // candidate regions: the filter's work units of K consecutive 32-document groups, about four per filter wave
    // (claimed dynamically by the filter waves; one probe wave each)
    const int64_t n_groups_all = (n_docs + FG_DOCS - 1) / FG_DOCS;
    int64_t kchunk = std::max<int64_t>(1, n_groups_all / ((int64_t)nsb * FS_WAVES * 4));
    if (const char *e = kw_env("KW_CHUNK_GROUPS")) kchunk = std::max(1, atoi(e));
    const bool dyn_groups = kw_env("KW_STATIC_GROUPS") == nullptr;   // (A/B: grid-stride, one chunk per wave)
    if (!dyn_groups && !kw_env("KW_CHUNK_GROUPS")) kchunk = (n_groups_all + (int64_t)nsb * FS_WAVES - 1) / ((int64_t)nsb * FS_WAVES);
    const int n_regions = (int)std::max<int64_t>(1, (n_groups_all + kchunk - 1) / kchunk);
    const int n_epi = neb * EK_WAVES;
    int rmul = 2;   // resolve blocks per resident slot: later blocks balance the uneven documents (measured: 2-3 % faster than 1)
    if (const char *e = kw_env("KW_RESOLVE_MUL")) rmul = std::max(1, atoi(e));
    int nrb = (int)std::min<int64_t>((n_docs + (int64_t)RK_WAVES * WAVE - 1) / ((int64_t)RK_WAVES * WAVE),
                                     (int64_t)h->cus * h->resolve_blocks_per_cu * rmul);
    if (const char *e = kw_env("KW_RESOLVE_BLOCKS")) nrb = std::min(nrb, std::max(1, atoi(e)));
    if (nrb < 1) nrb = 1;
    // generic kernel: 4 blocks per CU (one resident, 1 wave / SIMD at 256 VGPRs): the deferred documents'
    // costs vary by orders of magnitude, later blocks take the work of the slow ones
    int gmul = 4;
    if (const char *e = kw_env("KW_GENERIC_BLOCKS_PER_CU")) gmul = std::max(1, atoi(e));
    int ngb = std::max(1, (int)std::min<int64_t>((int64_t)h->cus * gmul, (n_docs + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK));
    {   // a generic wave's scratch grows with the largest deferred field: fewer waves then, within a budget
        const size_t per_wave = (size_t)2 * h->caps.gi_cap * 8 + (size_t)h->caps.gc_cap * 4 +
                                (size_t)(h->caps.gc_cap / 16 + 2) * 4;
        const size_t budget = (size_t)4 << 30;
        ngb = std::max(1, std::min(ngb, (int)std::max<size_t>(1, budget / per_wave / WAVES_PER_BLOCK)));
    }
    ScratchCaps w;
    w.nk = n_epi;
    w.ns = n_regions;
    w.nr = nrb * RK_WAVES;
    w.ng = ngb * WAVES_PER_BLOCK;
    const int64_t docs_per_k = (n_docs + w.nk - 1) / w.nk;
    const int64_t docs_per_s = (n_docs + w.ns - 1) / w.ns;
    // (regions of a few groups: a 1024 floor; a region that needs more grows every region and rescans)
    w.item_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1024, docs_per_s * 32), (int64_t)1 << 26);
    w.cand_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(1024, docs_per_s * 40), (int64_t)1 << 26);
    if (const char *e = kw_env("KW_TEST_CAND_CAP")) w.cand_cap = (uint32_t)std::max(1, atoi(e));
    if (const char *e = kw_env("KW_TEST_ITEM_CAP")) w.item_cap = (uint32_t)std::max(1, atoi(e));
    w.item_cap = (uint32_t)std::min<uint64_t>(w.item_cap, item_index_limit() / (uint64_t)n_regions);
    const int64_t docs_per_r = (n_docs + w.nr - 1) / w.nr;
    w.out_cap = (uint32_t)std::min<int64_t>(std::max<int64_t>(4096, std::max(docs_per_r, docs_per_k) * 48),
                                            (int64_t)1 << 26);
    w.rx_cap = (uint32_t)std::min<int64_t>(docs_per_r * 2 + 64, (int64_t)1 << 20);
    if (const char *e = kw_env("KW_TEST_RX_CAP")) w.rx_cap = (uint32_t)std::max(1, atoi(e));   // tests: force the rescan
    w.hdr_cap = std::max<int64_t>(n_docs, 1);
    w.defer_cap = (uint32_t)std::max<int64_t>(n_docs, 1);
    w.vcap = (uint32_t)std::min<int64_t>(docs_per_k * 8 + 256, (int64_t)1 << 24);
    w.ecap = (uint32_t)std::min<int64_t>(docs_per_k * 2 + 16, (int64_t)1 << 24);
    w.scap = w.ecap;
    w.xcap = (uint32_t)std::min<int64_t>(docs_per_k * 4 + 64, (int64_t)1 << 24);
    if (const char *e = kw_env("KW_TEST_TASK_CAP")) w.vcap = w.ecap = w.scap = w.xcap = (uint32_t)std::max(1, atoi(e));
    w.dsize = 4096;
    while (w.dsize < (uint64_t)std::max<int64_t>(n_docs, 1) * 16) w.dsize <<= 1;
    if (const char *e = kw_env("KW_TEST_DSET_SIZE")) w.dsize = std::max<uint64_t>(2, (uint64_t)atoll(e));
    // transcoded view: 768 B per document (~25 % of 2 KB articles non-ASCII), or what the last scan wanted
    w.tx_cap = std::max<uint64_t>((uint64_t)64 << 20, (uint64_t)std::max<int64_t>(n_docs, 1) * 768);
    w.tx_cap = std::max<uint64_t>(w.tx_cap, h->tx_need);
    if (const char *e = kw_env("KW_TEST_TX_CAP")) w.tx_cap = (uint64_t)std::max<long long>(16, atoll(e));
    int rc = ensure_scratch(h, w);
    if (rc) return rc;
    {   // the probe's item index (hdr.x) is 32-bit: regions x item_cap stays below 2^32; a larger need than the
        // clamped capacity defers the overflowing batches' documents to the generic kernel instead of growing
        const uint64_t icap = std::min<uint64_t>(h->caps.item_cap, item_index_limit() / (uint64_t)n_regions);
        h->FS.item_cap = (uint32_t)icap;
        h->FS.item_grow = icap == h->caps.item_cap && !h->item_clamped ? 1u : 0u;
    }
    h->FS.bigq = EK_BIGQ;   // (KW_TEST_BIGQ lowers it: tests send the big documents to the resolve kernel)
    if (const char *e = kw_env("KW_TEST_BIGQ")) h->FS.bigq = (uint32_t)std::min(std::max(0, atoi(e)), EK_BIGQ);
    h->FS.dyn = dyn_groups ? 1 : 0;
    h->FS.chunk_groups = kchunk;
    const int nk = h->nk;   // the allocation may be larger than this launch needs: every region is cleared
    HIPCHK(h, hipMemsetAsync(h->S.status, 0, 416, st));   // status .. stats, tx_used, res_cnt, total, gnext
    HIPCHK(h, hipMemsetAsync(h->out_cnt_all, 0, ((size_t)2 * nk + h->nr + h->ng) * 4, st));
    HIPCHK(h, hipMemsetAsync(h->FS.vcnt, 0, (size_t)nk * 20, st));   // vcnt, ecnt, scnt, xcnt, xmark
    HIPCHK(h, hipMemsetAsync(h->FS.dset, 0, (h->FS.dmask + 1) * 8, st));
    if (n_docs > 0) {
        HIPCHK(h, hipMemsetAsync(h->FS.ncnt, 0, (size_t)n_docs * 8, st));
        HIPCHK(h, hipMemsetAsync(h->FS.dflags, 0, (size_t)n_docs * 4, st));
    }
    HIPCHK(h, hipEventRecord(h->ev0, st));
    if (n_docs > 0)
        hipLaunchKernelGGL(kw_filter_kernel, dim3(nsb), dim3(FS_BLOCK), 0, st, h->FT, h->arena, h->doc_off, n_docs,
                           h->FS);
    HIPCHK(h, hipEventRecord(h->evf, st));
    // the transcoded view of the documents with a non-ASCII field (the filter flagged them) on the side
    // stream, beside the probe; the epilogue waits for it
    static const int tx_bpc = kw_env("KW_TX_BLOCKS_PER_CU") ? std::max(1, atoi(kw_env("KW_TX_BLOCKS_PER_CU"))) : 8;
    HIPCHK(h, hipStreamWaitEvent(side, h->evf, 0));
    if (n_docs > 0)
        hipLaunchKernelGGL(kw_tx_kernel, dim3(std::max(1, (int)std::min<int64_t>((n_docs + TX_BLOCK - 1) / TX_BLOCK, (int64_t)h->cus * tx_bpc))),
                           dim3(TX_BLOCK), 0, side, h->FT, h->arena, h->doc_off, n_docs, h->FS);
    HIPCHK(h, hipEventRecord(h->evx, side));
    // probe waves: the filter's wave count (each claims regions until none are left); KW_PROBE_WAVES (dev) sets it
    static const int probe_waves = kw_env("KW_PROBE_WAVES") ? std::max(1, atoi(kw_env("KW_PROBE_WAVES"))) : 0;
    if (n_docs > 0)
        hipLaunchKernelGGL(kw_probe_kernel, dim3((std::min(n_regions, probe_waves ? probe_waves : nsb * FS_WAVES) + PK_WAVES - 1) / PK_WAVES),
                           dim3(PK_BLOCK), 0, st, h->FT,
                           h->T, h->arena, h->doc_off, n_regions, h->FS);
    HIPCHK(h, hipEventRecord(h->evp, st));
    HIPCHK(h, hipStreamWaitEvent(st, h->evx, 0));
    if (n_docs > 0) {
        // the group epilogue (lane = item across 32 documents); KW_EPI_FLAT=0: one wave per document
        static const bool flat = !kw_env("KW_EPI_FLAT") || atoi(kw_env("KW_EPI_FLAT")) != 0;
        // its transcoded documents in the batches too when no name is PI_TXUNSAFE (KW_TEST_EPI_TXB=0, read per
        // scan: one at a time, as with such names)
        const bool txb = EF_TX_FLAT && (!kw_env("KW_TEST_EPI_TXB") || atoi(kw_env("KW_TEST_EPI_TXB")) != 0);
        if (flat && txb && h->FT.n_txu == 0)
            hipLaunchKernelGGL(kw_epi_flat_kernel<true>, dim3(neb), dim3(EK_BLOCK), 0, st, h->FT, h->arena,
                               h->doc_off, n_docs, h->FS, h->S);
        else if (flat)
            hipLaunchKernelGGL(kw_epi_flat_kernel<false>, dim3(neb), dim3(EK_BLOCK), 0, st, h->FT, h->arena,
                               h->doc_off, n_docs, h->FS, h->S);
        else
            hipLaunchKernelGGL(kw_epi_kernel, dim3(neb), dim3(EK_BLOCK), 0, st, h->FT, h->arena, h->doc_off, n_docs,
                               h->FS, h->S);
        HIPCHK(h, hipGetLastError());
    }
    h->ns = n_regions;
    HIPCHK(h, hipEventRecord(h->ev1, st));
    // the non-ASCII documents the epilogue's transcoded view left (DH_RESOLVE): the resolve kernel on the side
    // stream, beside the task kernels (disjoint documents, disjoint result regions); joined before the generic kernel
    HIPCHK(h, hipStreamWaitEvent(side, h->ev1, 0));
    HIPCHK(h, hipEventRecord(h->evs0, side));
    if (n_docs > 0) {
        hipLaunchKernelGGL(kw_resolve_kernel, dim3(nrb), dim3(RK_BLOCK), 0, side, h->FT, h->T, h->arena, h->doc_off,
                           n_docs, h->FS, h->S);
        // its documents with more items than its LDS holds: one wave each, wave w in resolve wave w's regions
        hipLaunchKernelGGL(kw_resolve_big_kernel, dim3(std::min(nrb * RK_WAVES, h->cus * 4)), dim3(WAVE), 0, side,
                           h->FT, h->T, h->arena, h->doc_off, h->FS, h->S);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipEventRecord(h->evs1, side));
    if (n_docs > 0) {
        // flat resolve tasks: verify -> short -> regex (regex decisions of the first two queue up);
        // G[k] waves share each epilogue wave's task region
        int G[4] = {1, 4, 4, 4};   // measured on MI355X (config 2, 2 runs each): 4.98 vs 5.00-5.01 ms for {1, 4, 2, 4} and {1, 4, 8, 4}, 5.00 {2, 4, 4, 4}, 5.17 {1, 4, 6, 6}, 5.34 {1, 4, 4, 8}
        if (const char *e = kw_env("KW_TASK_G")) sscanf(e, "%d,%d,%d,%d", &G[0], &G[1], &G[2], &G[3]);
        auto task = [&](auto kern, int g, hipStream_t s) {
            g = std::max(1, std::min(g, 16));
            const int nb = (n_epi * g + RK_WAVES - 1) / RK_WAVES;
            hipLaunchKernelGGL(kern, dim3(nb), dim3(RK_BLOCK), 0, s, h->FT, h->T, h->arena, h->doc_off,
                               n_epi, g, h->FS, h->S);
        };
        // the early regex tasks at 2 waves per region (config 2: 4.68 ms vs 4.78 at G[3] = 4, 4.70 at 1)
        const int g_early = kw_env("KW_RX_EARLY_G") ? atoi(kw_env("KW_RX_EARLY_G")) : 2;
        auto rx_task = [&](int phase, hipStream_t s) {
            const int g = std::max(1, std::min(phase == 1 && g_early > 0 ? g_early : G[3], 16));
            const int nb = (n_epi * g + RK_WAVES - 1) / RK_WAVES;
            hipLaunchKernelGGL(kw_rx_task_kernel, dim3(nb), dim3(RK_BLOCK), 0, s, h->FT, h->T, h->arena, h->doc_off,
                               n_epi, g, h->FS, h->S, phase);
        };
        // verify and short-field tasks are independent (both only append decisions): side by side; the
        // regex tasks they queued run after both.  The regex tasks the epilogue queued (its waves write their
        // count into xmark too) run beside them on side3 (KW_RX_SPLIT=0: all regex tasks after verify and short)
        const int rx_split_env = kw_env("KW_RX_SPLIT") ? atoi(kw_env("KW_RX_SPLIT")) : -1;   // (read per scan: tests)
        const bool rx_split = rx_split_env >= 0 ? rx_split_env != 0 : h->n_pat <= RX_SPLIT_MAX_PAT;
        HIPCHK(h, hipEventRecord(h->eve, st));
        if (rx_split) {
            HIPCHK(h, hipStreamWaitEvent(side3, h->eve, 0));
            rx_task(1, side3);
            HIPCHK(h, hipEventRecord(h->evrx, side3));
        }
        HIPCHK(h, hipStreamWaitEvent(side2, h->eve, 0));
        task(kw_short_kernel, G[2], side2);
        HIPCHK(h, hipEventRecord(h->evq, side2));
        task(kw_verify_kernel, G[0], st);
        HIPCHK(h, hipStreamWaitEvent(st, h->evq, 0));
        rx_task(rx_split ? 2 : 0, st);
        if (rx_split) HIPCHK(h, hipStreamWaitEvent(st, h->evrx, 0));
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipEventRecord(h->evt, st));
    // the generic kernel redoes every document the fast path deferred (the filter, probe, epilogue and resolve
    // kernels list them; the task kernels never do): on the side stream right after the resolve kernels,
    // beside the task kernels (its documents have no tasks; its result regions are its own).  It waited for the
    // tasks before: config 4 at 10M articles defers 943 documents, 9 ms of generic kernel after 23 ms of tasks
    HIPCHK(h, hipEventRecord(h->evr, side));
    if (n_docs > 0) {
        hipLaunchKernelGGL(kw_scan_kernel, dim3(ngb), dim3(BLOCK), kScanLds, side, h->T, h->arena, h->doc_off, n_docs,
                           h->S, (const uint32_t *)h->FS.defer_list, (const uint32_t *)h->FS.defer_cnt,
                           h->FS.defer_cap);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipEventRecord(h->evg, side));
    HIPCHK(h, hipStreamWaitEvent(st, h->evg, 0));
    const int nw = 2 * nk + h->nr + h->ng;
    if (n_docs > 0) {
        hipLaunchKernelGGL(kw_offsets_kernel, dim3(1), dim3(1024), 0, st, h->out_cnt_all, nw, h->out_cap, h->d_offs,
                           h->d_total);
        hipLaunchKernelGGL(kw_gather_kernel, dim3(nw), dim3(256), 0, st, h->out_all, h->out_cap, h->out_cnt_all,
                           h->d_offs, h->d_hits);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipEventRecord(h->ev2, st));
    h->launched_waves = nw;
    return KW_OK;
}

extern "C" int kw_scan(kw_handle *h, const uint8_t *d_arena, const int64_t *d_doc_off, int64_t n_docs, void *stream)
{
    if (!h) return KW_EINVAL;
    if (n_docs < 0 || (n_docs > 0 && (!d_arena || !d_doc_off))) { h->err = "kw_scan: bad arguments"; return KW_EINVAL; }
    if (((uintptr_t)d_arena & 15) != 0) { h->err = "kw_scan: arena must be 16-byte aligned"; return KW_EINVAL; }
    HIPCHK(h, hipSetDevice(h->device));
    h->arena = d_arena;
    h->doc_off = d_doc_off;
    h->n_docs = n_docs;
    h->stream = (hipStream_t)stream;
    h->scanned = true;
    h->fetched = false;
    h->rescans = 0;
    h->rescan_causes = 0;
    h->item_clamped = false;   // (per batch: a later batch with fewer regions may grow its item regions again)
    return launch_scan(h);
}

extern "C" int kw_scan_host(kw_handle *h, const uint8_t *arena, int64_t arena_bytes, const int64_t *doc_off,
                            int64_t n_docs)
{
    if (!h) return KW_EINVAL;
    if (n_docs < 0 || arena_bytes < 0 || (n_docs > 0 && (!arena || !doc_off))) {
        h->err = "kw_scan_host: bad arguments";
        return KW_EINVAL;
    }
    HIPCHK(h, hipSetDevice(h->device));
    if (!h->own) HIPCHK(h, hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking));
    const size_t ab = (size_t)arena_bytes + 64, ob = (size_t)(2 * n_docs + 1) * sizeof(int64_t);
    if (ab > h->h_arena_cap) {
        if (h->h_arena) HIPCHK(h, hipFree(h->h_arena));
        h->h_arena = nullptr;
        h->h_arena_cap = ab + ab / 4;
        HIPCHK(h, hipMalloc((void **)&h->h_arena, h->h_arena_cap));
    }
    if (ob > h->h_off_cap) {
        if (h->h_off) HIPCHK(h, hipFree(h->h_off));
        h->h_off = nullptr;
        h->h_off_cap = ob + ob / 4;
        HIPCHK(h, hipMalloc((void **)&h->h_off, h->h_off_cap));
    }
    if (arena_bytes > 0) HIPCHK(h, hipMemcpyAsync(h->h_arena, arena, (size_t)arena_bytes, hipMemcpyHostToDevice, h->own));
    HIPCHK(h, hipMemsetAsync(h->h_arena + arena_bytes, 0, 64, h->own));   // the tiles' read-past pad
    if (n_docs > 0) HIPCHK(h, hipMemcpyAsync(h->h_off, doc_off, ob, hipMemcpyHostToDevice, h->own));
    return kw_scan(h, h->h_arena, h->h_off, n_docs, h->own);
}

extern "C" int kw_hits_host(kw_handle *h, kw_hit *dst, int64_t cap, int64_t *n_hits)
{
    if (!h || !n_hits) return KW_EINVAL;
    const kw_hit *d = nullptr;
    int rc = kw_hits(h, n_hits, &d);
    if (rc) return rc;
    if (*n_hits > cap) { h->err = "kw_hits_host: destination too small"; return KW_EINVAL; }
    if (*n_hits > 0) HIPCHK(h, hipMemcpy(dst, d, (size_t)*n_hits * sizeof(kw_hit), hipMemcpyDeviceToHost));
    return KW_OK;
}

extern "C" int kw_device_count(int32_t *n)
{
    if (!n) return KW_EINVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return KW_OK;
}

extern "C" int kw_device_init(int32_t device)
{
    if (hipSetDevice(device) != hipSuccess) return KW_EHIP;
    return hipFree(nullptr) == hipSuccess ? KW_OK : KW_EHIP;   // creates the device context
}

static int finish(kw_handle *h)
{
    if (!h->scanned) { h->err = "kw_hits: no scan"; return KW_ESTATE; }
    if (h->fetched) return KW_OK;
    for (int attempt = 0; attempt < 6; ++attempt) {
        HIPCHK(h, hipStreamSynchronize(h->stream));
        // the scan's small results in one copy: status (0), generic stats (64), fast-path stats (128),
        // transcoded-view bytes (384), record count (400)
        unsigned long long small[51];
        HIPCHK(h, hipMemcpy(small, h->S.status, sizeof(small), hipMemcpyDeviceToHost));
        if (kw_env("KW_DEBUG_TASKS") && h->nk > 0) {   // (developer aid) the task regions' queue lengths
            std::vector<uint32_t> tc((size_t)4 * h->nk);
            HIPCHK(h, hipMemcpy(tc.data(), h->FS.vcnt, tc.size() * 4, hipMemcpyDeviceToHost));
            for (int q = 0; q < 4; ++q) {
                uint64_t sum = 0;
                uint32_t mx = 0;
                for (int t = 0; t < h->nk; ++t) { sum += tc[(size_t)q * h->nk + t]; mx = std::max(mx, tc[(size_t)q * h->nk + t]); }
                fprintf(stderr, "kw tasks %c: %d regions, total %llu, mean %.1f, max %u\n", "vesx"[q], h->nk,
                        (unsigned long long)sum, (double)sum / h->nk, mx);
            }
        }
        uint32_t status[4];
        memcpy(status, small, sizeof(status));
        if (h->n_docs == 0) { h->n_hits = 0; h->fetched = true; return KW_OK; }
        if (status[0] & ST_FIELD_TOO_LONG) {
            char buf[256];
            snprintf(buf, sizeof(buf), "kw_scan: a field longer than %lld bytes (positions are 23-bit in the "
                     "device item records; the reference has no such limit)", (long long)MAX_FIELD_BYTES);
            h->err = buf;
            return KW_EOVERFLOW;
        }
        if (status[0] & (ST_ITEM_OVERFLOW | ST_CP_OVERFLOW)) {
            // a deferred field needs more anchor items or code points than the generic kernel's buffers hold:
            // grow them to the need (fewer generic waves, within the scratch budget) and scan again
            uint32_t gm[2];
            HIPCHK(h, hipMemcpy(gm, h->S.gmax, sizeof(gm), hipMemcpyDeviceToHost));
            ScratchCaps w = h->caps;
            if (status[0] & ST_ITEM_OVERFLOW) {
                uint32_t c = w.gi_cap;
                while (c < gm[0] && c < (1u << 30)) c <<= 1;
                if (c < gm[0]) { h->err = "kw_scan: a field with more than 2^30 anchor occurrences"; return KW_EOVERFLOW; }
                w.gi_cap = c;
            }
            if (status[0] & ST_CP_OVERFLOW) w.gc_cap = std::max(w.gc_cap, gm[1] + 64);
            const size_t per_wave = (size_t)2 * w.gi_cap * 8 + (size_t)w.gc_cap * 4 + (size_t)(w.gc_cap / 16 + 2) * 4;
            const size_t budget = (size_t)4 << 30;
            w.ng = (int)std::min<size_t>((size_t)w.ng, std::max<size_t>(WAVES_PER_BLOCK, budget / per_wave / WAVES_PER_BLOCK * WAVES_PER_BLOCK));
            h->caps.ng = w.ng;   // the generic wave count may shrink
            int rc = ensure_scratch(h, w);
            if (rc) return rc;
            ++h->rescans;
            h->rescan_causes |= status[0] & ~ST_FIELD_TOO_LONG;
            rc = launch_scan(h);
            if (rc) return rc;
            continue;
        }
        if (status[0] & (ST_OUT_OVERFLOW | ST_RX_OVERFLOW | ST_TASK_OVERFLOW | ST_DSET_FULL | ST_CAND_OVERFLOW)) {
            // grow what overflowed (result regions to the largest count seen, queues to the largest need) and rescan
            ScratchCaps w = h->caps;
            if (status[0] & ST_OUT_OVERFLOW) {
                std::vector<uint32_t> cnt(h->launched_waves);
                HIPCHK(h, hipMemcpy(cnt.data(), h->out_cnt_all, cnt.size() * 4, hipMemcpyDeviceToHost));
                uint32_t mx = 0;
                for (uint32_t c : cnt) mx = std::max(mx, c);
                w.out_cap = std::max(w.out_cap, mx + 1024);
            }
            if (status[0] & ST_RX_OVERFLOW) w.rx_cap = std::max(status[2], w.rx_cap * 2);
            if (status[0] & ST_TASK_OVERFLOW) {
                uint32_t tm[4];
                HIPCHK(h, hipMemcpy(tm, h->FS.tmax, sizeof(tm), hipMemcpyDeviceToHost));
                w.vcap = std::max(w.vcap, tm[0]);
                w.ecap = std::max(w.ecap, tm[1]);
                w.scap = std::max(w.scap, tm[2]);
                w.xcap = std::max(w.xcap, tm[3]);
            }
            if (status[0] & ST_DSET_FULL) w.dsize *= 4;
            if (status[0] & ST_CAND_OVERFLOW) {
                uint32_t cm[2];
                HIPCHK(h, hipMemcpy(cm, h->FS.cmax, sizeof(cm), hipMemcpyDeviceToHost));
                w.cand_cap = std::max(w.cand_cap, cm[0] + cm[0] / 8 + 64);
                const uint64_t lim = item_index_limit() / (uint64_t)std::max(1, h->ns);
                const uint64_t want = (uint64_t)cm[1] + cm[1] / 8 + 64;
                if (want > lim) h->item_clamped = true;   // this batch: defer, never grow past the index limit
                w.item_cap = std::max<uint32_t>(w.item_cap, (uint32_t)std::min<uint64_t>(want, lim));
            }
            int rc = ensure_scratch(h, w);
            if (rc) return rc;
            ++h->rescans;
            h->rescan_causes |= status[0] & ~ST_FIELD_TOO_LONG;
            rc = launch_scan(h);
            if (rc) return rc;
            continue;
        }
        const unsigned long long tot = small[50];
        const unsigned long long *gst = small + 8, *fst = small + 16;
        h->stats[0] = fst[0] + gst[0];
        h->stats[1] = fst[1] + gst[1];
        h->stats[2] = fst[2] + gst[2];
        h->stats[3] = fst[3];
        for (int i = 4; i < KW_N_STATS; ++i) h->stats[i] = fst[i];
        h->stats[17] = (unsigned long long)h->rescans;
        h->stats[20] = (unsigned long long)h->rescan_causes;
        {   // the transcoded view: documents it took / left to the resolve kernel; the next scan's capacity
            const unsigned long long used = small[48];
            if (used > h->caps.tx_cap && !kw_env("KW_TEST_TX_CAP")) h->tx_need = used + used / 8;
        }
        if (kw_env("KW_DUMP_TIMING")) {   // FK_TIMING builds: resolve-kernel cycles summed over waves
            fprintf(stderr, "KW_TIMING resolve decode %llu edge %llu items %llu short %llu regex %llu all %llu\n", fst[21],
                    fst[22], fst[23], fst[24], fst[25], fst[26]);
            fprintf(stderr, "KW_TASKS verify %llu edge %llu short %llu regex %llu edge_docs %llu\n", fst[27], fst[28], fst[29],
                    fst[30], fst[31]);
        }
        h->n_hits = (int64_t)tot;
        h->fetched = true;
        return KW_OK;
    }
    h->err = "kw_hits: result buffer kept overflowing";
    return KW_EOVERFLOW;
}

extern "C" int kw_hits(kw_handle *h, int64_t *n_hits, const kw_hit **d_hits)
{
    if (!h || !n_hits || !d_hits) return KW_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    int rc = finish(h);
    if (rc) return rc;
    *n_hits = h->n_hits;
    *d_hits = h->d_hits;
    return KW_OK;
}

extern "C" int kw_hits_copy(kw_handle *h, kw_hit *d_dst, int64_t cap, int64_t *n_hits, void *stream)
{
    if (!h || !n_hits) return KW_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    int rc = finish(h);
    if (rc) return rc;
    *n_hits = h->n_hits;
    if (h->n_hits > cap) { h->err = "kw_hits_copy: destination too small"; return KW_EINVAL; }
    if (h->n_hits > 0)
        HIPCHK(h, hipMemcpyAsync(d_dst, h->d_hits, (size_t)h->n_hits * sizeof(kw_hit), hipMemcpyDeviceToDevice,
                                 (hipStream_t)stream));
    return KW_OK;
}

extern "C" int kw_stats(kw_handle *h, int64_t *stats, int32_t n_stats)
{
    if (!h || !stats) return KW_EINVAL;
    int rc = finish(h);
    if (rc) return rc;
    for (int i = 0; i < n_stats && i < KW_N_STATS; ++i) stats[i] = (int64_t)h->stats[i];
    return KW_OK;
}

extern "C" int kw_last_kernel_ms(kw_handle *h, float *fast_ms, float *generic_ms, float *total_ms)
{
    if (!h) return KW_EINVAL;
    int rc = finish(h);
    if (rc) return rc;
    if (fast_ms) HIPCHK(h, hipEventElapsedTime(fast_ms, h->ev0, h->evr));
    if (generic_ms) HIPCHK(h, hipEventElapsedTime(generic_ms, h->evr, h->evg));
    if (total_ms) HIPCHK(h, hipEventElapsedTime(total_ms, h->ev0, h->ev2));
    return KW_OK;
}

extern "C" int kw_last_kernel_times(kw_handle *h, float *ms, int32_t n)
{
    if (!h || !ms) return KW_EINVAL;
    int rc = finish(h);
    if (rc) return rc;
    hipEvent_t ev[6] = {h->ev0, h->ev1, h->evr, h->evg, h->ev2, h->ev2};
    for (int i = 0; i < n && i < 4; ++i) HIPCHK(h, hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]));
    if (n > 4) HIPCHK(h, hipEventElapsedTime(&ms[4], h->ev0, h->ev2));
    hipEvent_t sp[4] = {h->ev0, h->evf, h->evp, h->ev1};
    for (int i = 0; i + 5 < n && i < 3; ++i) HIPCHK(h, hipEventElapsedTime(&ms[5 + i], sp[i], sp[i + 1]));
    if (n > 8) HIPCHK(h, hipEventElapsedTime(&ms[8], h->evs0, h->evs1));
    if (n > 9) HIPCHK(h, hipEventElapsedTime(&ms[9], h->ev1, h->evt));
    return KW_OK;
}

extern "C" int kw_doc_routes(kw_handle *h, uint8_t *routes, int64_t n)
{
    if (!h || (n > 0 && !routes)) return KW_EINVAL;
    HIPCHK(h, hipSetDevice(h->device));
    int rc = finish(h);
    if (rc) return rc;
    if (n != h->n_docs) { h->err = "kw_doc_routes: n differs from the scanned document count"; return KW_EINVAL; }
    std::vector<uint2> hdr((size_t)n);
    std::vector<uint32_t> dfl((size_t)n);
    if (n > 0) {
        HIPCHK(h, hipMemcpy(hdr.data(), h->FS.hdr, (size_t)n * sizeof(uint2), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(dfl.data(), h->FS.dflags, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    for (int64_t d = 0; d < n; ++d) {
        const uint32_t y = hdr[d].y;
        // (dflags: DH_RESOLVE also marks the all-ASCII big documents an epilogue workgroup had no room for)
        routes[d] = (y & DH_DEFER)                                       ? KW_ROUTE_GENERIC
                    : (y & DH_TX)                                        ? KW_ROUTE_TRANSCODE
                    : ((y & (DH_NA0 | DH_NA1)) || (dfl[d] & DH_RESOLVE)) ? KW_ROUTE_RESOLVE
                                                                         : KW_ROUTE_SCAN;
    }
    return KW_OK;
}

extern "C" const char *kw_last_error(kw_handle *h)
{
    if (!h) return g_err.c_str();
    return h->err.c_str();
}

extern "C" int kw_destroy(kw_handle *h)
{
    if (!h) return KW_OK;
    (void)hipSetDevice(h->device);
    if (h->d_tables) (void)hipFree(h->d_tables);
    if (h->d_scratch) (void)hipFree(h->d_scratch);
    if (h->d_small) (void)hipFree(h->d_small);
    if (h->d_hits) (void)hipFree(h->d_hits);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->ev2) (void)hipEventDestroy(h->ev2);
    if (h->evg) (void)hipEventDestroy(h->evg);
    if (h->evr) (void)hipEventDestroy(h->evr);
    if (h->evf) (void)hipEventDestroy(h->evf);
    if (h->evs0) (void)hipEventDestroy(h->evs0);
    if (h->evs1) (void)hipEventDestroy(h->evs1);
    if (h->evt) (void)hipEventDestroy(h->evt);
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->side2) (void)hipStreamDestroy(h->side2);
    if (h->side3) (void)hipStreamDestroy(h->side3);
    if (h->own) (void)hipStreamDestroy(h->own);
    if (h->h_arena) (void)hipFree(h->h_arena);
    if (h->h_off) (void)hipFree(h->h_off);
    if (h->eve) (void)hipEventDestroy(h->eve);
    if (h->evq) (void)hipEventDestroy(h->evq);
    if (h->evrx) (void)hipEventDestroy(h->evrx);
    if (h->evx) (void)hipEventDestroy(h->evx);
    if (h->evp) (void)hipEventDestroy(h->evp);
    delete h;
    return KW_OK;
}
