/*
 * kwcsv.c -- host-side CSV tokenizer for the article ingest and the output sort (libkwcsv.so).
 *
 * The reference reads the article CSV with pandas' C parser in 20 000-row chunks
 * (match_keywords.py:230) and later re-reads every per-ticker output file to sort it
 * (:195-217).  This tokenizer reproduces the parser's default dialect for both: ',' delimiter,
 * '"' quoting with doubled quotes, "\n", "\r\n" and lone "\r" record ends, blank lines skipped,
 * and the default NA strings (pandas' STR_NA_VALUES, passed in by the caller) -- quoted or not --
 * mark a cell as NaN.  It does not guess dtypes: every cell carries a flag telling whether it is a
 * witness that its column stays text (a character no number or bool literal holds); the caller
 * hands a chunk back to pandas when a needed column has no witness, and on any record it cannot
 * tokenize exactly (a field count different from the header's, a character after a closing quote),
 * so the fast path is only taken where its result equals pandas'.
 *
 * kwcsv_parse   records -> unescaped cell bytes + offsets + flags
 * kwcsv_pack    the text / title cells of parsed records -> the matcher's byte arena (NaN -> "nan",
 *               match_keywords.py:150-151) and its 2n+1 offsets
 * kwcsv_utf8_ok validity of UTF-8 cells (pandas raises UnicodeDecodeError on the others)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KWCSV_QUOTED 1u   /* the cell was quoted */
#define KWCSV_NA 2u       /* the cell is one of the NA strings: NaN */
#define KWCSV_TEXT 4u     /* the cell proves its column is text (see kwcsv_text_witness) */
#define KWCSV_CANON 8u    /* quoted iff the value holds ',', '"' or '\n': the csv writer's QUOTE_MINIMAL form */

static int is_na(const uint8_t *s, int64_t n, const uint8_t *na, const int32_t *na_off, int32_t n_na)
{
    for (int32_t k = 0; k < n_na; ++k) {
        const int32_t a = na_off[k], b = na_off[k + 1];
        if (b - a == n && memcmp(na + a, s, (size_t)n) == 0) return 1;
    }
    return 0;
}

static int ieq(const uint8_t *s, int64_t n, const char *lit)
{
    const int64_t m = (int64_t)strlen(lit);
    if (m != n) return 0;
    for (int64_t i = 0; i < n; ++i) {
        uint8_t c = s[i];
        if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
        if (c != (uint8_t)lit[i]) return 0;
    }
    return 1;
}

/* A non-NA cell that neither a number (ints, floats with '.', exponent, sign, surrounding blanks,
 * inf / infinity) nor a bool literal can be: its column keeps dtype object in pandas' inference. */
static int kwcsv_text_witness(const uint8_t *s, int64_t n)
{
    int64_t a = 0, b = n;
    while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
    if (a == b) return 1;   /* blanks only: no number */
    const uint8_t *t = s + a;
    const int64_t m = b - a;
    if (ieq(t, m, "true") || ieq(t, m, "false")) return 0;
    int64_t i = (t[0] == '+' || t[0] == '-') ? 1 : 0;
    if (ieq(t + i, m - i, "inf") || ieq(t + i, m - i, "infinity")) return 0;
    for (int64_t k = 0; k < m; ++k) {
        const uint8_t c = t[k];
        if (!((c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E')) return 1;
    }
    return 0;
}

/*
 * Parse up to max_rows records of buf[pos, len) with ncols fields each.  Cell bytes (quotes removed,
 * doubled quotes undone) go to out (cap bytes); cell i of record r spans out[coff[r*ncols+i],
 * coff[r*ncols+i+1]); cfl gets its KWCSV_* flags.  *pos_out = the position after the last record.
 * Returns the records parsed (0 at the end of the input), -1 if out is too small, -2 for a record
 * this tokenizer does not reproduce exactly (the caller falls back to pandas), -3 for a record whose
 * field count differs from ncols.  rspan (optional, 2 per record) gets each record's byte span without
 * its terminator.
 */
int64_t kwcsv_parse(const uint8_t *buf, int64_t len, int64_t pos, int64_t max_rows, int32_t ncols,
                    const uint8_t *na, const int32_t *na_off, int32_t n_na, uint8_t *out, int64_t cap,
                    int64_t *coff, uint8_t *cfl, int64_t *pos_out, int64_t *rspan)
{
    int64_t p = pos, o = 0, rows = 0;
    coff[0] = 0;
    while (rows < max_rows) {
        /* blank lines -- empty or blanks only -- are skipped, as pandas' skip_blank_lines does */
        for (;;) {
            int64_t k = p;
            while (k < len && (buf[k] == ' ' || buf[k] == '\t')) ++k;
            if (k < len && (buf[k] == '\n' || buf[k] == '\r')) { p = k + 1; continue; }
            if (k >= len) p = k;
            break;
        }
        if (p >= len) break;
        if (rspan) rspan[2 * rows] = p;
        int32_t f = 0;
        for (;;) {
            const int64_t cell0 = o;
            uint8_t flags = 0;
            if (p < len && buf[p] == '"') {
                flags |= KWCSV_QUOTED;
                ++p;
                for (;;) {
                    const uint8_t *q = p < len ? (const uint8_t *)memchr(buf + p, '"', (size_t)(len - p)) : NULL;
                    if (!q) return -2;   /* unterminated quote */
                    const int64_t k = (int64_t)(q - buf);
                    if (o + (k - p) + 1 > cap) return -1;
                    memcpy(out + o, buf + p, (size_t)(k - p));
                    o += k - p;
                    p = k + 1;
                    if (p < len && buf[p] == '"') { out[o++] = '"'; ++p; continue; }
                    break;
                }
                if (p < len && buf[p] != ',' && buf[p] != '\n' && buf[p] != '\r') return -2;
            } else {
                int64_t k = p;
                while (k < len && buf[k] != ',' && buf[k] != '\n' && buf[k] != '\r') ++k;
                if (o + (k - p) > cap) return -1;
                memcpy(out + o, buf + p, (size_t)(k - p));
                o += k - p;
                p = k;
            }
            if (f >= ncols) return -3;
            {
                const int64_t n = o - cell0;
                const int needq = n > 0 && (memchr(out + cell0, ',', (size_t)n) || memchr(out + cell0, '"', (size_t)n) ||
                                            memchr(out + cell0, '\n', (size_t)n));
                if (needq == ((flags & KWCSV_QUOTED) != 0)) flags |= KWCSV_CANON;
            }
            if (is_na(out + cell0, o - cell0, na, na_off, n_na)) flags |= KWCSV_NA;
            else if (kwcsv_text_witness(out + cell0, o - cell0)) flags |= KWCSV_TEXT;
            cfl[rows * ncols + f] = flags;
            coff[rows * ncols + f + 1] = o;
            ++f;
            if (p < len && buf[p] == ',') { ++p; continue; }
            if (rspan) rspan[2 * rows + 1] = p;
            /* record end: "\n", "\r\n", "\r" or the end of the input */
            if (p < len && buf[p] == '\r') ++p;
            if (p < len && buf[p] == '\n' && buf[p - 1] != '\n') ++p;
            break;
        }
        if (f != ncols) return -3;
        ++rows;
    }
    *pos_out = p;
    return rows;
}

/* Every cell of column `col` of rows [0, nrows) is valid UTF-8 (or NA).  Returns 1 / 0. */
int32_t kwcsv_utf8_ok(const uint8_t *out, const int64_t *coff, const uint8_t *cfl, int64_t nrows, int32_t ncols,
                      int32_t col)
{
    for (int64_t r = 0; r < nrows; ++r) {
        const int64_t c = r * ncols + col;
        if (cfl[c] & KWCSV_NA) continue;
        const uint8_t *s = out + coff[c];
        const int64_t n = coff[c + 1] - coff[c];
        for (int64_t i = 0; i < n;) {
            const uint8_t b = s[i];
            int64_t k;
            uint32_t cp;
            if (b < 0x80) { ++i; continue; }
            if (b >= 0xC2 && b <= 0xDF) { k = 1; cp = b & 0x1F; }
            else if (b >= 0xE0 && b <= 0xEF) { k = 2; cp = b & 0x0F; }
            else if (b >= 0xF0 && b <= 0xF4) { k = 3; cp = b & 0x07; }
            else return 0;
            for (int64_t j = 1; j <= k; ++j) {
                if (i + j >= n || (s[i + j] & 0xC0) != 0x80) return 0;
                cp = (cp << 6) | (s[i + j] & 0x3F);
            }
            if ((k == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (k == 3 && (cp < 0x10000 || cp > 0x10FFFF)))
                return 0;
            i += k + 1;
        }
    }
    return 1;
}

/*
 * The matcher's arena for parsed rows: document r = text cell then title cell (column ct, ci); an NA
 * cell is "nan" (str(NaN), match_keywords.py:150-151).  off gets 2*nrows+1 offsets.  Returns the
 * arena bytes, or -1 if cap is too small.
 */
int64_t kwcsv_pack(const uint8_t *out, const int64_t *coff, const uint8_t *cfl, int64_t nrows, int32_t ncols,
                   int32_t ct, int32_t ci, uint8_t *arena, int64_t cap, int64_t *off)
{
    int64_t a = 0;
    off[0] = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        for (int k = 0; k < 2; ++k) {
            const int64_t c = r * ncols + (k ? ci : ct);
            const uint8_t *s = out + coff[c];
            int64_t n = coff[c + 1] - coff[c];
            if (cfl[c] & KWCSV_NA) { s = (const uint8_t *)"nan"; n = 3; }
            if (a + n > cap) return -1;
            memcpy(arena + a, s, (size_t)n);
            a += n;
            off[2 * r + k + 1] = a;
        }
    }
    return a;
}

/*
 * Record boundaries only (the --gpus N ingest: every rank finds a chunk's records, then tokenizes just its
 * own byte-balanced share with kwcsv_parse).  The same record split as kwcsv_parse: blank lines skipped,
 * '"' quoting with doubled quotes, "\n" / "\r\n" / "\r" ends.  starts[r] = the first byte of record r
 * (r < rows), starts[rows] = the position after the last record (= kwcsv_parse's *pos_out).  Returns the
 * records found (at most max_rows; 0 at the end of the input), -2 for a record kwcsv_parse would not
 * reproduce (a character after a closing quote, an unterminated quote), -3 for a field count other than
 * ncols.
 */
int64_t kwcsv_records(const uint8_t *buf, int64_t len, int64_t pos, int64_t max_rows, int32_t ncols, int64_t *starts)
{
    int64_t p = pos, rows = 0;
    while (rows < max_rows) {
        for (;;) {
            int64_t k = p;
            while (k < len && (buf[k] == ' ' || buf[k] == '\t')) ++k;
            if (k < len && (buf[k] == '\n' || buf[k] == '\r')) { p = k + 1; continue; }
            if (k >= len) p = k;
            break;
        }
        if (p >= len) break;
        starts[rows] = p;
        int32_t f = 0;
        for (;;) {
            if (p < len && buf[p] == '"') {
                ++p;
                for (;;) {
                    const uint8_t *q = p < len ? (const uint8_t *)memchr(buf + p, '"', (size_t)(len - p)) : NULL;
                    if (!q) return -2;
                    p = (int64_t)(q - buf) + 1;
                    if (p < len && buf[p] == '"') { ++p; continue; }
                    break;
                }
                if (p < len && buf[p] != ',' && buf[p] != '\n' && buf[p] != '\r') return -2;
            } else {
                while (p < len && buf[p] != ',' && buf[p] != '\n' && buf[p] != '\r') ++p;
            }
            if (f >= ncols) return -3;
            ++f;
            if (p < len && buf[p] == ',') { ++p; continue; }
            if (p < len && buf[p] == '\r') ++p;
            if (p < len && buf[p] == '\n' && buf[p - 1] != '\n') ++p;
            break;
        }
        if (f != ncols) return -3;
        ++rows;
    }
    starts[rows] = p;
    return rows;
}

/* one cell of an output row (0, or -1 when out is full) */
static int put_cell(uint8_t *out, int64_t cap, int64_t *o, const uint8_t *s, int64_t n)
{
    /* the csv writer's QUOTE_MINIMAL (pandas to_csv): quoted iff the value holds ',', '"' or '\n' (the
     * line terminator), quotes doubled; '\r' alone is written as it is */
    int q = n > 0 && (memchr(s, ',', (size_t)n) || memchr(s, '"', (size_t)n) || memchr(s, '\n', (size_t)n));
    if (!q) {
        if (*o + n > cap) return -1;
        memcpy(out + *o, s, (size_t)n);
        *o += n;
        return 0;
    }
    if (*o + 2 * n + 2 > cap) return -1;
    out[(*o)++] = '"';
    for (int64_t i = 0; i < n; ++i) {
        if (s[i] == '"') out[(*o)++] = '"';
        out[(*o)++] = s[i];
    }
    out[(*o)++] = '"';
    return 0;
}

/*
 * The output rows of a native chunk as CSV bytes (match_keywords.py:131-146: one row per (article, ticker),
 * columns time_unix, date_time, text_matches, title_matches, title, url, source, source_url, article_text),
 * written as the reference's per-row DataFrame.to_csv writes them: the time stamp as a decimal integer, the
 * JSON cells as given, every other cell from the chunk's tokenized cells (an NA cell = NaN -> empty), each
 * in QUOTE_MINIMAL form, "\n" line ends.  Rows are emitted in the given order; row r's line is
 * out[line_off[r], line_off[r + 1]).  cols[6] = the chunk columns of date_time, title, url, source,
 * source_url, article_text; json3[3r .. 3r+2] = row r's text_matches JSON json[json3[3r], json3[3r+1]) and
 * title_matches JSON json[json3[3r+1], json3[3r+2]).  flags[r]: bit c (c = 0..7 for output columns 1..8) = that cell is a text
 * witness (KWCSV_TEXT: no number or bool literal; the JSON cells always are), bit 8 + c = that cell is NA,
 * bit 16 = a cell holds '\r' (pandas' re-read would split the record there).  Returns 0, -1 when out is too
 * small, -2 for a NUL character in a cell (the caller's pandas path raises as the reference does).
 */
/* one chunk cell of an output row into out (NA: empty); *fl gets its bits for output column c; 0, -1 when out
 * is full, -2 for a NUL character */
static int emit_chunk_cell(const uint8_t *cells, const int64_t *coff, const uint8_t *cfl, int64_t cell, int c,
                           uint8_t *out, int64_t cap, int64_t *o, uint32_t *fl)
{
    const uint8_t *s = cells + coff[cell];
    int64_t n = coff[cell + 1] - coff[cell];
    const int na = (cfl[cell] & KWCSV_NA) != 0;
    if (na) n = 0;
    if (n > 0 && memchr(s, 0, (size_t)n)) return -2;
    if (n > 0 && memchr(s, '\r', (size_t)n)) *fl |= 1u << 16;
    if (na) *fl |= 1u << (8 + c);
    else if (kwcsv_text_witness(s, n)) *fl |= 1u << c;
    return put_cell(out, cap, o, s, n) ? -1 : 0;
}

int64_t kwcsv_emit(const uint8_t *cells, const int64_t *coff, const uint8_t *cfl, int32_t ncols, const int32_t *cols,
                   const int32_t *row_doc, const int64_t *row_stamp, int64_t nrows, const uint8_t *json,
                   const int64_t *json3, uint8_t *out, int64_t cap, int64_t *line_off, uint32_t *flags)
{
    /* An article's chunk cells are the same in every row it has (one per matched ticker): each article's
     * date_time cell and its title .. article_text cells are rendered (QUOTE_MINIMAL, flags) once, at the
     * end of out, and copied into its rows. */
    int32_t dmax = -1;
    for (int64_t r = 0; r < nrows; ++r) if (row_doc[r] > dmax) dmax = row_doc[r];
    int64_t *part = (int64_t *)malloc(sizeof(int64_t) * 3 * (size_t)(dmax + 1));   /* A start, B start, B end */
    uint32_t *dfl = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(dmax + 1));
    if (!part || !dfl) { free(part); free(dfl); return -3; }
    for (int32_t d = 0; d <= dmax; ++d) part[3 * d] = -1;
    int64_t hi = cap;   /* the rendered articles grow down from the end of out */
    int64_t rc = 0;
    for (int64_t r = 0; r < nrows && rc == 0; ++r) {
        const int32_t d = row_doc[r];
        if (part[3 * d] >= 0) continue;
        /* render into a scratch position after the rows' room: measure first by rendering at the low end
         * of the free space [hi - need, hi) is unknown, so render at a fixed probe offset below hi */
        const int64_t base = (int64_t)d * ncols;
        int64_t need = 16;
        for (int c = 0; c < 6; ++c) {
            const int64_t cell = base + cols[c];
            need += 2 * (coff[cell + 1] - coff[cell]) + 3;
        }
        if (hi - need < 0) { rc = -1; break; }
        int64_t o = hi - need;
        const int64_t a0 = o;
        uint32_t fl = 0;
        int e = emit_chunk_cell(cells, coff, cfl, base + cols[0], 0, out, cap, &o, &fl);
        const int64_t b0 = o;
        for (int c = 3; c < 8 && e == 0; ++c) {
            if (c > 3) out[o++] = ',';
            e = emit_chunk_cell(cells, coff, cfl, base + cols[c - 2], c, out, cap, &o, &fl);
        }
        if (e) { rc = e; break; }
        /* move the rendering to the top of the free space */
        const int64_t len = o - a0;
        memmove(out + hi - len, out + a0, (size_t)len);
        part[3 * d] = hi - len;
        part[3 * d + 1] = hi - len + (b0 - a0);
        part[3 * d + 2] = hi;
        dfl[d] = fl;
        hi -= len;
    }
    int64_t o = 0;
    line_off[0] = 0;
    for (int64_t r = 0; r < nrows && rc == 0; ++r) {
        const int32_t d = row_doc[r];
        uint32_t fl = dfl[d] | 6u;   /* the JSON cells are text witnesses */
        char num[24];
        int k = 24;
        int64_t v = row_stamp[r];
        uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1u : (uint64_t)v;
        do { num[--k] = (char)('0' + u % 10); u /= 10; } while (u);
        if (v < 0) num[--k] = '-';
        const int64_t la = part[3 * d + 1] - part[3 * d], lb = part[3 * d + 2] - part[3 * d + 1];
        if (o + (24 - k) + la + lb + 8 > hi) { rc = -1; break; }
        memcpy(out + o, num + k, (size_t)(24 - k));
        o += 24 - k;
        out[o++] = ',';
        memcpy(out + o, out + part[3 * d], (size_t)la);
        o += la;
        for (int c = 1; c < 3; ++c) {
            const uint8_t *s = json + json3[3 * r + (c - 1)];
            const int64_t n = json3[3 * r + c] - json3[3 * r + (c - 1)];
            if (n > 0 && memchr(s, 0, (size_t)n)) { rc = -2; break; }
            if (n > 0 && memchr(s, '\r', (size_t)n)) fl |= 1u << 16;
            out[o++] = ',';
            if (put_cell(out, hi - 1, &o, s, n)) { rc = -1; break; }
        }
        if (rc) break;
        if (o + lb + 2 > hi) { rc = -1; break; }
        out[o++] = ',';
        memcpy(out + o, out + part[3 * d + 1], (size_t)lb);
        o += lb;
        out[o++] = '\n';
        line_off[r + 1] = o;
        flags[r] = fl;
    }
    free(part);
    free(dfl);
    return rc;
}
