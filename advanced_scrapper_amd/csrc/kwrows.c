/* Host assembly of the output rows' ticker_matches cells from the device hit records.
 *
 * Replaces, for the drop-in's write path, the Python loop of matcher.assemble_ticker_matches +
 * json.dumps (match_keywords.py:159-187 build ticker_matches; :137-138 serialise matched_names['text']
 * and ['title']).  Input: the hit records sorted by (doc, field, pattern, pos); per document the
 * article date as integer epoch microseconds (kb.epoch_us) and whether it exists; the KB occurrence
 * table in CSR form (ticker, traversal rank, period bounds as epoch-µs, open bounds = INT64_MIN/MAX);
 * the JSON text of every pattern name (json.dumps(name), ensure_ascii, quotes included).
 *
 * Rules (the same as assemble_ticker_matches): a (field, pattern) group of a document matches ticker t
 * iff one of the pattern's occurrences for t is in period (lo <= date <= hi); its dict position inside
 * t's text/title dict is the rank of the first such occurrence; tickers are emitted in KB order, names in
 * rank order, positions ascending ([] when the match has no position).  A ticker with nothing in period
 * emits no row.  Output per row: doc, ticker, and two JSON strings written exactly as json.dumps does
 * with its default separators (", " and ": ").
 *
 * Returns the number of rows, -1 when a capacity is too small (the caller grows the buffers and calls
 * again), -2 when an in-period match is a name whose regex does not compile (the caller reruns the Python
 * path, which raises re.error as the reference does).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef struct { uint32_t doc, pattern, pos, field; } kw_hit_rec;
typedef struct { int32_t ti, field, rank, pat; int64_t hs, he; } entry_t;

static int cmp_entry(const void *a, const void *b) {
    const entry_t *x = (const entry_t *)a, *y = (const entry_t *)b;
    if (x->ti != y->ti) return x->ti < y->ti ? -1 : 1;
    if (x->field != y->field) return x->field < y->field ? -1 : 1;
    return (x->rank > y->rank) - (x->rank < y->rank);
}

typedef struct { char *p; int64_t n, cap; int over; } sink_t;

static void put(sink_t *s, const char *src, int64_t len) {
    if (s->n + len > s->cap) { s->over = 1; return; }
    memcpy(s->p + s->n, src, (size_t)len);
    s->n += len;
}

static void put_u32(sink_t *s, uint32_t v) {
    char buf[12];
    int k = 12;
    do { buf[--k] = (char)('0' + v % 10); v /= 10; } while (v);
    put(s, buf + k, 12 - k);
}

/* one JSON object {"name": [p, ...], ...} of the entries [e0, e1) of one field */
static void put_dict(sink_t *s, const entry_t *e0, const entry_t *e1, const kw_hit_rec *h, const char *keys,
                     const int64_t *key_off) {
    put(s, "{", 1);
    for (const entry_t *e = e0; e < e1; ++e) {
        if (e != e0) put(s, ", ", 2);
        put(s, keys + key_off[e->pat], key_off[e->pat + 1] - key_off[e->pat]);
        put(s, ": [", 3);
        int first = 1;
        for (int64_t i = e->hs; i < e->he; ++i) {
            if (h[i].pos == 0xFFFFFFFFu) continue;
            if (!first) put(s, ", ", 2);
            put_u32(s, h[i].pos);
            first = 0;
        }
        put(s, "]", 1);
    }
    put(s, "}", 1);
}

static int64_t max_rows_guess(int64_t n_hits) { return n_hits + 1024; }

int64_t kwrows_assemble(const kw_hit_rec *h, int64_t n_hits, const int64_t *date_us, const uint8_t *date_ok,
                        int64_t n_docs, const int64_t *occ_off, const int32_t *occ_ti, const int32_t *occ_rank,
                        const int64_t *occ_lo, const int64_t *occ_hi, const uint8_t *invalid_rx,
                        const char *keys, const int64_t *key_off, int32_t n_tickers, int32_t *row_doc,
                        int32_t *row_ti, int64_t row_cap, char *out, int64_t *out_off, int64_t out_cap) {
    int64_t *seen = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_tickers > 0 ? n_tickers : 1));
    int64_t ecap = 1024, ne = 0, rows = 0, group = 0, rc = 0;
    entry_t *ent = (entry_t *)malloc(sizeof(entry_t) * (size_t)ecap);
    if (!seen || !ent) { free(seen); free(ent); return -3; }   /* allocation failure */
    for (int32_t t = 0; t < n_tickers; ++t) seen[t] = -1;
    sink_t s = {out, 0, out_cap, 0};
    out_off[0] = 0;
    int64_t i = 0;
    while (i < n_hits && rc == 0) {
        const uint32_t d = h[i].doc;
        int64_t j = i;
        while (j < n_hits && h[j].doc == d) ++j;
        if ((int64_t)d >= n_docs || !date_ok[d]) { i = j; continue; }
        const int64_t a = date_us[d];
        ne = 0;
        for (int64_t g = i; g < j;) {   /* (field, pattern) groups */
            int64_t ge = g;
            while (ge < j && h[ge].field == h[g].field && h[ge].pattern == h[g].pattern) ++ge;
            const uint32_t p = h[g].pattern;
            ++group;
            for (int64_t o = occ_off[p]; o < occ_off[p + 1]; ++o) {
                const int32_t t = occ_ti[o];
                if (seen[t] == group || a < occ_lo[o] || a > occ_hi[o]) continue;
                seen[t] = group;
                if (invalid_rx[p]) { rc = -2; break; }
                if (ne == ecap) {
                    ecap *= 2;
                    entry_t *ne_ = (entry_t *)realloc(ent, sizeof(entry_t) * (size_t)ecap);
                    if (!ne_) { rc = -3; break; }
                    ent = ne_;
                }
                ent[ne++] = (entry_t){t, (int32_t)h[g].field, occ_rank[o], (int32_t)p, g, ge};
            }
            if (rc) break;
            g = ge;
        }
        if (rc) break;
        qsort(ent, (size_t)ne, sizeof(entry_t), cmp_entry);
        for (int64_t e = 0; e < ne;) {
            int64_t ee = e, mid;
            while (ee < ne && ent[ee].ti == ent[e].ti) ++ee;
            mid = e;
            while (mid < ee && ent[mid].field == 0) ++mid;
            if (rows == row_cap) { rc = -1; break; }
            row_doc[rows] = (int32_t)d;
            row_ti[rows] = ent[e].ti;
            put_dict(&s, ent + e, ent + mid, h, keys, key_off);
            out_off[2 * rows + 1] = s.n;
            put_dict(&s, ent + mid, ent + ee, h, keys, key_off);
            out_off[2 * rows + 2] = s.n;
            ++rows;
            e = ee;
        }
        if (s.over) rc = -1;
        i = j;
    }
    free(seen);
    free(ent);
    return rc ? rc : rows;
}

/*
 * kwrows_assemble over nthreads threads: the sorted hit records are cut at document boundaries into one slice
 * per thread, each slice is assembled into the thread's own buffers (kwrows_assemble on the slice), and the
 * slices are concatenated in document order -- the same rows, JSON text and offsets as one kwrows_assemble
 * call.  need[0..1] gets the rows and JSON bytes of the whole result; returns the rows, -1 when row_cap or
 * out_cap is smaller than need (nothing written; call again with need), -2 / -3 as kwrows_assemble (the
 * first slice's error in document order).
 */
int64_t kwrows_assemble_mt(const kw_hit_rec *h, int64_t n_hits, const int64_t *date_us, const uint8_t *date_ok,
                           int64_t n_docs, const int64_t *occ_off, const int32_t *occ_ti, const int32_t *occ_rank,
                           const int64_t *occ_lo, const int64_t *occ_hi, const uint8_t *invalid_rx,
                           const char *keys, const int64_t *key_off, int32_t n_tickers, int32_t *row_doc,
                           int32_t *row_ti, int64_t row_cap, char *out, int64_t *out_off, int64_t out_cap,
                           int64_t *need, int32_t nthreads)
{
    int64_t nt = nthreads > 1 ? nthreads : 1;
    if (nt > n_hits / 4096 + 1) nt = n_hits / 4096 + 1;
    int64_t *cut = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nt + 1));
    int64_t *rows = (int64_t *)calloc((size_t)nt, sizeof(int64_t));
    int32_t **rd = (int32_t **)calloc((size_t)nt, sizeof(int32_t *));
    int32_t **rt = (int32_t **)calloc((size_t)nt, sizeof(int32_t *));
    char **ob = (char **)calloc((size_t)nt, sizeof(char *));
    int64_t **oo = (int64_t **)calloc((size_t)nt, sizeof(int64_t *));
    if (!cut || !rows || !rd || !rt || !ob || !oo) { free(cut); free(rows); free(rd); free(rt); free(ob); free(oo); return -3; }
    cut[0] = 0;
    for (int64_t t = 1; t < nt; ++t) {   /* slice starts at document boundaries */
        int64_t c = n_hits * t / nt;
        if (c < cut[t - 1]) c = cut[t - 1];
        while (c > cut[t - 1] && c < n_hits && h[c].doc == h[c - 1].doc) ++c;
        cut[t] = c;
    }
    cut[nt] = n_hits;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t a = cut[t], b = cut[t + 1];
        if (b <= a) { rows[t] = 0; continue; }
        int64_t rc_ = max_rows_guess(b - a), oc = 64 * (b - a) + 4096;
        for (;;) {
            rd[t] = (int32_t *)realloc(rd[t], sizeof(int32_t) * (size_t)rc_);
            rt[t] = (int32_t *)realloc(rt[t], sizeof(int32_t) * (size_t)rc_);
            ob[t] = (char *)realloc(ob[t], (size_t)oc);
            oo[t] = (int64_t *)realloc(oo[t], sizeof(int64_t) * (size_t)(2 * rc_ + 1));
            if (!rd[t] || !rt[t] || !ob[t] || !oo[t]) { rows[t] = -3; break; }
            const int64_t r = kwrows_assemble(h + a, b - a, date_us, date_ok, n_docs, occ_off, occ_ti, occ_rank, occ_lo,
                                              occ_hi, invalid_rx, keys, key_off, n_tickers, rd[t], rt[t], rc_, ob[t],
                                              oo[t], oc);
            if (r == -1) { rc_ *= 2; oc *= 2; continue; }
            rows[t] = r;
            break;
        }
    }
    int64_t rc = 0, nr = 0, nb = 0;
    for (int64_t t = 0; t < nt && rc == 0; ++t) {
        if (rows[t] < 0) rc = rows[t];
        else { nr += rows[t]; nb += rows[t] ? oo[t][2 * rows[t]] : 0; }
    }
    if (rc == 0) {
        need[0] = nr;
        need[1] = nb;
        if (nr > row_cap || nb > out_cap) rc = -1;
    }
    if (rc == 0) {
        int64_t *r0 = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nt + 1));
        int64_t *b0 = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nt + 1));
        if (!r0 || !b0) rc = -3;
        else {
            r0[0] = b0[0] = 0;
            for (int64_t t = 0; t < nt; ++t) {
                r0[t + 1] = r0[t] + rows[t];
                b0[t + 1] = b0[t] + (rows[t] ? oo[t][2 * rows[t]] : 0);
            }
            out_off[0] = 0;
            #pragma omp parallel for num_threads(nt) schedule(static)
            for (int64_t t = 0; t < nt; ++t) {
                const int64_t k = rows[t];
                if (!k) continue;
                memcpy(row_doc + r0[t], rd[t], sizeof(int32_t) * (size_t)k);
                memcpy(row_ti + r0[t], rt[t], sizeof(int32_t) * (size_t)k);
                memcpy(out + b0[t], ob[t], (size_t)oo[t][2 * k]);
                for (int64_t j = 1; j <= 2 * k; ++j) out_off[2 * r0[t] + j] = oo[t][j] + b0[t];
            }
            rc = nr;
        }
        free(r0);
        free(b0);
    }
    for (int64_t t = 0; t < nt; ++t) { free(rd[t]); free(rt[t]); free(ob[t]); free(oo[t]); }
    free(cut); free(rows); free(rd); free(rt); free(ob); free(oo);
    return rc;
}
