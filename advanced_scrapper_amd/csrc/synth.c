/*
 * Seeded synthetic financial-news corpus generator (host C, OpenMP).
 *
 * Bench/test data only: it produces the article arena that BASELINE.json's
 * configs name ("~2 KB synthetic financial-news articles").
 * It is not part of the matching path and never runs on the device.
 *
 * Every document is a pure function of (seed, global doc index), so a shard
 * generated on rank r is byte-identical to the same documents generated as
 * part of the full corpus.  Only IEEE double arithmetic (no libm) is used so
 * the bytes do not depend on the host's libm.
 *
 * Per document:
 *   - article text: lognormal length, median 2048 B, clipped to [256, 16384]
 *     (stops at the first sentence end past the target);
 *   - title: 40-120 B, title-cased words;
 *   - injected KB names at Poisson(lambda=3): 70% exact, 10% uppercase names
 *     glued to word chars / punctuation / Unicode (\b cases), 10% near-misses
 *     (1..ceil(2m/20)-1 indels for m >= 21), 5% truncated at the text start or
 *     end (edge windows), 5% case-flipped;
 *   - 1% NaN titles, 0.1% NaN texts (flag bits; the arena holds "nan", the
 *     a6 rule of match_keywords.py:150-151), 2% of documents with non-ASCII.
 *
 * Arena layout: for doc d, text = [off[2d], off[2d+1]), title =
 * [off[2d+1], off[2d+2]); flags[d] bit0 = NaN text, bit1 = NaN title.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t s; } rng_t;

static inline uint64_t rnext(rng_t *r)
{
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline double runif(rng_t *r) { return (double)(rnext(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint32_t rint_(rng_t *r, uint32_t n) { return (uint32_t)((rnext(r) >> 32) * (uint64_t)n >> 32); }

/* 2^x for |x| < 8 without libm: integer part by doubling, fraction by a
   degree-7 Taylor polynomial of exp(f*ln2) (plenty for a length draw) */
static double pow2(double x)
{
    int ip = (int)x;
    if (x < 0 && (double)ip != x) ip -= 1;
    double f = x - ip;
    double t = f * 0.6931471805599453, term = 1.0, s = 1.0;
    for (int k = 1; k <= 7; ++k) { term *= t / k; s += term; }
    while (ip > 0) { s *= 2.0; --ip; }
    while (ip < 0) { s *= 0.5; ++ip; }
    return s;
}

static int poisson3(rng_t *r)
{
    /* Knuth, lambda = 3: L = e^-3 */
    const double L = 0.049787068367863944;
    int k = 0;
    double p = 1.0;
    do { ++k; p *= runif(r); } while (p > L);
    return k - 1;
}

typedef struct {
    const uint8_t *vocab; const int64_t *vocab_off; int n_vocab;
    const uint8_t *acr; const int64_t *acr_off; int n_acr;
    const uint8_t *uni; const int64_t *uni_off; int n_uni;
    const uint8_t *names; const int64_t *name_off; const uint8_t *name_kind; int n_names;
    const int32_t *u_idx; int n_u;   /* indices of kind-0 (uppercase) names */
    const int32_t *f_idx; int n_f;   /* indices of kind-1 (fuzzy-class) names */
} synth_ctx;

/* growable writer that can also run in count-only mode (buf == NULL) */
typedef struct { uint8_t *buf; int64_t n; uint8_t lastc; } wr_t;
static inline void put(wr_t *w, const uint8_t *s, int64_t len)
{
    if (len <= 0) return;
    if (w->buf) memcpy(w->buf + w->n, s, (size_t)len);
    w->n += len;
    w->lastc = s[len - 1];
}
static inline void putc_(wr_t *w, uint8_t c) { if (w->buf) w->buf[w->n] = c; w->n++; w->lastc = c; }
static inline uint8_t last(const wr_t *w, int64_t base) { return (w->n > base) ? w->lastc : 0; }

static void put_word(wr_t *w, const synth_ctx *c, rng_t *r, int cap)
{
    uint32_t k = rint_(r, (uint32_t)c->n_vocab);
    const uint8_t *s = c->vocab + c->vocab_off[k];
    int64_t len = c->vocab_off[k + 1] - c->vocab_off[k];
    if (cap && len > 0 && s[0] >= 'a' && s[0] <= 'z') {
        putc_(w, (uint8_t)(s[0] - 32));
        put(w, s + 1, len - 1);
    } else {
        put(w, s, len);
    }
}

static void put_number(wr_t *w, rng_t *r)
{
    char tmp[32];
    int n = 0;
    uint32_t kind = rint_(r, 4);
    uint32_t a = rint_(r, 1000), b = rint_(r, 10);
    if (kind == 0) { tmp[n++] = '$'; }
    /* a.b */
    char d[8]; int nd = 0;
    if (a == 0) d[nd++] = '0';
    while (a) { d[nd++] = (char)('0' + a % 10); a /= 10; }
    while (nd) tmp[n++] = d[--nd];
    tmp[n++] = '.';
    tmp[n++] = (char)('0' + b);
    if (kind == 1) tmp[n++] = '%';
    else if (kind == 0) { const char *bn = " billion"; while (*bn) tmp[n++] = *bn++; }
    put(w, (const uint8_t *)tmp, n);
}

/* write a (possibly perturbed) name; returns nothing */
static void put_name(wr_t *w, const synth_ctx *c, rng_t *r, int32_t idx, int mode)
{
    const uint8_t *s = c->names + c->name_off[idx];
    int64_t len = c->name_off[idx + 1] - c->name_off[idx];
    uint8_t tmp[512];
    if (len > 400) len = 400;
    if (mode == 0) { put(w, s, len); return; }
    if (mode == 3) {          /* case flip, ASCII letters only */
        for (int64_t i = 0; i < len; ++i) {
            uint8_t ch = s[i];
            if (ch >= 'a' && ch <= 'z') ch = (uint8_t)(ch - 32);
            else if (ch >= 'A' && ch <= 'Z') ch = (uint8_t)(ch + 32);
            tmp[i] = ch;
        }
        put(w, tmp, len);
        return;
    }
    if (mode == 2) {          /* near miss: k indels on ASCII positions */
        int64_t m = len;
        int kmax = (int)((2 * m + 19) / 20) - 1;
        if (kmax < 1) kmax = 1;
        int k = 1 + (int)rint_(r, (uint32_t)kmax);
        int64_t n = len;
        memcpy(tmp, s, (size_t)len);
        for (int e = 0; e < k && n > 2; ++e) {
            int64_t p = 1 + (int64_t)rint_(r, (uint32_t)(n - 2));
            if (tmp[p] >= 0x80) continue;   /* keep UTF-8 valid */
            if (rint_(r, 2) == 0) {          /* delete */
                memmove(tmp + p, tmp + p + 1, (size_t)(n - p - 1));
                --n;
            } else {                          /* insert a lowercase letter */
                memmove(tmp + p + 1, tmp + p, (size_t)(n - p));
                tmp[p] = (uint8_t)('a' + rint_(r, 26));
                ++n;
            }
        }
        put(w, tmp, n);
        return;
    }
}

static int32_t pick_name(const synth_ctx *c, rng_t *r, int want_u)
{
    if (want_u && c->n_u) return c->u_idx[rint_(r, (uint32_t)c->n_u)];
    if (!want_u && c->n_f) return c->f_idx[rint_(r, (uint32_t)c->n_f)];
    return (int32_t)rint_(r, (uint32_t)c->n_names);
}

/* a glue char for the \b cases */
static void put_glue(wr_t *w, rng_t *r)
{
    static const char *g[] = {"x", "_", "7", ".", ",", "-", "(", ")", "$", "+",
                              "\xc3\xa9", "\xe2\x80\x99", "\xe4\xb8\xad", "\xc3\x89", "s", "'"};
    const char *s = g[rint_(r, 16)];
    put(w, (const uint8_t *)s, (int64_t)strlen(s));
}

static void gen_text(wr_t *w, const synth_ctx *c, rng_t *r, int64_t target, int nonascii)
{
    int64_t base = w->n;
    int n_inject = poisson3(r);
    double words_est = (double)target / 6.5;
    double p_inj = words_est > 1 ? (double)n_inject / words_est : 0.5;
    int edge_start = 0, edge_end = 0;
    /* 5% of injections are edge truncations: decide up front */
    if (runif(r) < 1.0 - pow2(-0.0740 * n_inject)) {
        if (rint_(r, 2)) edge_start = 1; else edge_end = 1;
    }
    if (edge_start) {
        int32_t idx = pick_name(c, r, 0);
        const uint8_t *s = c->names + c->name_off[idx];
        int64_t len = c->name_off[idx + 1] - c->name_off[idx];
        int64_t drop = 1 + rint_(r, 2);
        while (drop < len && (s[drop] & 0xC0) == 0x80) ++drop;
        if (len > drop) { put(w, s + drop, len - drop); putc_(w, ' '); }
    }
    int sent_words = 0, sent_len = 6 + (int)rint_(r, 20);
    int first = (w->n == base);
    while (w->n - base < target) {
        if (!first) putc_(w, ' ');
        int cap = (sent_words == 0);
        double u = runif(r);
        if (u < p_inj) {
            double v = runif(r);
            if (v < 0.74) {                     /* exact */
                put_name(w, c, r, pick_name(c, r, rint_(r, 4) == 0), 0);
            } else if (v < 0.85) {              /* uppercase name glued */
                int32_t idx = pick_name(c, r, 1);
                int side = (int)rint_(r, 3);
                if (side != 1) put_glue(w, r);
                put_name(w, c, r, idx, 0);
                if (side != 0) put_glue(w, r);
            } else if (v < 0.95) {              /* near miss */
                put_name(w, c, r, pick_name(c, r, 0), 2);
            } else {                             /* case flipped */
                put_name(w, c, r, pick_name(c, r, rint_(r, 2)), 3);
            }
        } else if (u < p_inj + 0.04) {
            put_number(w, r);
        } else if (u < p_inj + 0.06 && c->n_acr) {
            uint32_t k = rint_(r, (uint32_t)c->n_acr);
            put(w, c->acr + c->acr_off[k], c->acr_off[k + 1] - c->acr_off[k]);
        } else if (nonascii && u < p_inj + 0.12 && c->n_uni) {
            uint32_t k = rint_(r, (uint32_t)c->n_uni);
            put(w, c->uni + c->uni_off[k], c->uni_off[k + 1] - c->uni_off[k]);
        } else {
            put_word(w, c, r, cap);
        }
        first = 0;
        if (++sent_words >= sent_len) {
            uint32_t p = rint_(r, 10);
            putc_(w, p < 8 ? '.' : (p == 8 ? '?' : ';'));
            sent_words = 0;
            sent_len = 6 + (int)rint_(r, 20);
            if (rint_(r, 12) == 0) { putc_(w, '\n'); putc_(w, '\n'); first = 1; }
        } else if (rint_(r, 14) == 0) {
            putc_(w, ',');
        }
    }
    if (last(w, base) != '.') putc_(w, '.');
    if (edge_end) {
        int32_t idx = pick_name(c, r, 0);
        const uint8_t *s = c->names + c->name_off[idx];
        int64_t len = c->name_off[idx + 1] - c->name_off[idx];
        int64_t drop = 1 + rint_(r, 2);
        int64_t keep = len - drop;
        while (keep > 0 && (s[keep] & 0xC0) == 0x80) --keep;
        if (keep > 0) { putc_(w, ' '); put(w, s, keep); }
    }
}

static void gen_title(wr_t *w, const synth_ctx *c, rng_t *r)
{
    int64_t base = w->n;
    int64_t target = 40 + rint_(r, 81);
    int inject = rint_(r, 10) < 3;
    int inj_at = inject ? (int)rint_(r, 6) : -1;
    int k = 0;
    while (w->n - base < target) {
        if (w->n > base) putc_(w, ' ');
        if (k == inj_at) put_name(w, c, r, pick_name(c, r, rint_(r, 3) == 0), 0);
        else put_word(w, c, r, 1);
        ++k;
    }
}

static int64_t gen_doc(uint8_t *out, const synth_ctx *c, uint64_t seed, int64_t gidx, int64_t *text_len,
                       uint8_t *flag)
{
    rng_t r = {seed * 0x100000001B3ull ^ (uint64_t)gidx * 0x9E3779B97F4A7C15ull};
    rnext(&r);
    wr_t w = {out, 0, 0};
    /* Irwin-Hall normal, sigma 0.55 in log2 units */
    double z = 0;
    for (int i = 0; i < 12; ++i) z += runif(&r);
    z -= 6.0;
    double len = 2048.0 * pow2(0.55 * z);
    if (len < 256) len = 256;
    if (len > 16000) len = 16000;
    int nonascii = rint_(&r, 50) == 0;
    uint8_t fl = 0;
    if (rint_(&r, 1000) == 0) fl |= 1;
    if (rint_(&r, 100) == 0) fl |= 2;
    if (fl & 1) put(&w, (const uint8_t *)"nan", 3);
    else gen_text(&w, c, &r, (int64_t)len, nonascii);
    *text_len = w.n;
    if (fl & 2) put(&w, (const uint8_t *)"nan", 3);
    else gen_title(&w, c, &r);
    *flag = fl;
    return w.n;
}

/* Pass 1: per-doc byte lengths (text, title) -> lens[2n]. */
void synth_lengths(const synth_ctx *c, uint64_t seed, int64_t doc_base, int64_t n_docs, int64_t *lens)
{
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < n_docs; ++i) {
        int64_t tl;
        uint8_t fl;
        int64_t tot = gen_doc(NULL, c, seed, doc_base + i, &tl, &fl);
        lens[2 * i] = tl;
        lens[2 * i + 1] = tot - tl;
    }
}

/* Pass 2: write into arena at off[2i] (off from the prefix sum of lens). */
void synth_fill(const synth_ctx *c, uint64_t seed, int64_t doc_base, int64_t n_docs, const int64_t *off,
                uint8_t *arena, uint8_t *flags)
{
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < n_docs; ++i) {
        int64_t tl;
        gen_doc(arena + off[2 * i], c, seed, doc_base + i, &tl, &flags[i]);
    }
}

int synth_ctx_size(void) { return (int)sizeof(synth_ctx); }

/* ------------------------------------------------------------------------
 * Synthetic CDX link rows (config 5): the `original` URL
 * column of an Internet-Archive CDX listing of finance.yahoo.com/news/ URLs.
 * Row r is a pure function of (seed, r).  About 30 % of rows repeat an earlier
 * article (uniform article ids over 1.31 n), and the spellings exercise every
 * rule of yahoo_links_selenium.py:63-79: http vs https, ':80' ports, query
 * strings / fragments after '.html', 'www.' hosts, rows without '.html',
 * 'news/%' and "news/'" paths, '<x>html' regex matches, non-ASCII slugs.
 * ------------------------------------------------------------------------ */
static const char *URL_WORDS[] = {
    "stocks", "market", "rally", "fed", "rates", "earnings", "beat", "miss", "oil", "gold", "bitcoin", "tesla",
    "apple", "nvidia", "amazon", "google", "microsoft", "bank", "jobs", "report", "inflation", "cpi", "dollar",
    "yields", "bonds", "tech", "shares", "surge", "drop", "record", "high", "low", "week", "ahead", "what",
    "know", "why", "how", "analyst", "upgrade", "downgrade", "deal", "merger", "ipo", "crypto", "china", "trade",
    "tariffs", "retail", "sales", "housing", "consumer", "outlook", "guidance", "q1", "q2", "q3", "q4"};
#define N_URL_WORDS ((int)(sizeof(URL_WORDS) / sizeof(URL_WORDS[0])))

static int64_t gen_url(uint8_t *out, uint64_t seed, int64_t row, int64_t n_articles, int64_t *ts)
{
    rng_t r = {seed * 0x9E3779B97F4A7C15ull ^ (uint64_t)row * 0xD1B54A32D192ED03ull};
    rnext(&r);
    const uint64_t art = (uint64_t)((rnext(&r) >> 11) % (uint64_t)(n_articles > 0 ? n_articles : 1));
    rng_t a = {seed ^ art * 0x94D049BB133111EBull};
    rnext(&a);
    wr_t w = {out, 0, 0};
    const uint32_t v = rint_(&r, 1000);
    /* scheme and host */
    const char *scheme = (v < 200) ? "http://" : "https://";
    put(&w, (const uint8_t *)scheme, (int64_t)strlen(scheme));
    if (v >= 950 && v < 1000) put(&w, (const uint8_t *)"www.", 4);
    put(&w, (const uint8_t *)"finance.yahoo.com", 17);
    if (rint_(&r, 20) == 0) put(&w, (const uint8_t *)":80", 3);
    put(&w, (const uint8_t *)"/news/", 6);
    const uint32_t odd = rint_(&r, 200);
    if (odd == 0) put(&w, (const uint8_t *)"%20", 3);
    else if (odd == 1) put(&w, (const uint8_t *)"'", 1);
    /* slug of the article */
    const int nw = 3 + (int)rint_(&a, 8);
    for (int i = 0; i < nw; ++i) {
        const char *s = URL_WORDS[rint_(&a, N_URL_WORDS)];
        if (i) putc_(&w, '-');
        put(&w, (const uint8_t *)s, (int64_t)strlen(s));
    }
    if (rint_(&a, 100) == 0) put(&w, (const uint8_t *)"-caf\xc3\xa9", 6);
    char id[24];
    int nd = 0;
    uint64_t x = 100000000ull + (art % 900000000ull);
    while (x) { id[nd++] = (char)('0' + x % 10); x /= 10; }
    putc_(&w, '-');
    while (nd) putc_(&w, (uint8_t)id[--nd]);
    /* ending */
    const uint32_t e = rint_(&r, 100);
    if (e < 5) {
        put(&w, (const uint8_t *)".htm", 4);                   /* no '.html': dropped */
    } else if (e < 6) {
        put(&w, (const uint8_t *)"xhtml", 5);                  /* regex '.html' matches 'xhtml' */
    } else {
        put(&w, (const uint8_t *)".html", 5);
        if (e >= 80 && e < 95) put(&w, (const uint8_t *)"?.tsrc=rss", 10);
        else if (e >= 95 && e < 98) put(&w, (const uint8_t *)"#comments", 9);
        else if (e >= 98) put(&w, (const uint8_t *)".html", 5);
    }
    if (ts) {
        /* 14-digit CDX timestamp YYYYMMDDhhmmss (2017..2025) */
        const uint64_t t = rnext(&r);
        const int64_t Y = 2017 + (int64_t)(t % 9), M = 1 + (int64_t)((t >> 8) % 12), D = 1 + (int64_t)((t >> 16) % 28);
        const int64_t h = (int64_t)((t >> 24) % 24), mi = (int64_t)((t >> 32) % 60), s = (int64_t)((t >> 40) % 60);
        *ts = ((((Y * 100 + M) * 100 + D) * 100 + h) * 100 + mi) * 100 + s;
    }
    return w.n;
}

void synth_url_lengths(uint64_t seed, int64_t row_base, int64_t n_rows, int64_t n_articles, int64_t *lens)
{
#pragma omp parallel for schedule(static, 4096)
    for (int64_t i = 0; i < n_rows; ++i) lens[i] = gen_url(NULL, seed, row_base + i, n_articles, NULL);
}

void synth_url_fill(uint64_t seed, int64_t row_base, int64_t n_rows, int64_t n_articles, const int64_t *off,
                    uint8_t *arena, int64_t *ts)
{
#pragma omp parallel for schedule(static, 4096)
    for (int64_t i = 0; i < n_rows; ++i) gen_url(arena + off[i], seed, row_base + i, n_articles, ts ? ts + i : NULL);
}
