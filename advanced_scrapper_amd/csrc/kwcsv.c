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
 *
 * The *_mt entry points split a chunk's records over host threads (OpenMP; the reference spreads its
 * per-article work over mp.cpu_count() processes, match_keywords.py:231-236): kwcsv_parse_mt tokenizes row
 * ranges in parallel and compacts them into kwcsv_parse's exact layout, kwcsv_utf8_ok_mt checks several
 * columns at once, kwcsv_pack_mt packs the arena, kwcsv_dates parses the dataset's date layout.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

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
/* kwcsv_parse without writing coff[0] (the threaded form's ranges share that slot with the previous range) */
static int64_t parse_body(const uint8_t *buf, int64_t len, int64_t pos, int64_t max_rows, int32_t ncols,
                          const uint8_t *na, const int32_t *na_off, int32_t n_na, uint8_t *out, int64_t cap,
                          int64_t *coff, uint8_t *cfl, int64_t *pos_out, int64_t *rspan)
{
    int64_t p = pos, o = 0, rows = 0;
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

/* one cell is valid UTF-8 (strict: no overlongs, surrogates or code points above U+10FFFF); ASCII runs are
 * skipped eight bytes at a time */
static int utf8_cell_ok(const uint8_t *s, int64_t n)
{
    int64_t i = 0;
    while (i < n) {
        while (i + 8 <= n) {
            uint64_t w;
            memcpy(&w, s + i, 8);
            if (w & 0x8080808080808080ull) break;
            i += 8;
        }
        if (i >= n) break;
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
    return 1;
}

int64_t kwcsv_parse(const uint8_t *buf, int64_t len, int64_t pos, int64_t max_rows, int32_t ncols,
                    const uint8_t *na, const int32_t *na_off, int32_t n_na, uint8_t *out, int64_t cap,
                    int64_t *coff, uint8_t *cfl, int64_t *pos_out, int64_t *rspan)
{
    coff[0] = 0;
    return parse_body(buf, len, pos, max_rows, ncols, na, na_off, n_na, out, cap, coff, cfl, pos_out, rspan);
}

/* Every cell of column `col` of rows [0, nrows) is valid UTF-8 (or NA).  Returns 1 / 0. */
int32_t kwcsv_utf8_ok(const uint8_t *out, const int64_t *coff, const uint8_t *cfl, int64_t nrows, int32_t ncols,
                      int32_t col)
{
    for (int64_t r = 0; r < nrows; ++r) {
        const int64_t c = r * ncols + col;
        if (cfl[c] & KWCSV_NA) continue;
        if (!utf8_cell_ok(out + coff[c], coff[c + 1] - coff[c])) return 0;
    }
    return 1;
}

/* kwcsv_utf8_ok of ncheck columns at once over nthreads threads: ok[k] = 1 / 0 for column cols[k]. */
void kwcsv_utf8_ok_mt(const uint8_t *out, const int64_t *coff, const uint8_t *cfl, int64_t nrows, int32_t ncols,
                      const int32_t *cols, int32_t ncheck, int32_t *ok, int32_t nthreads)
{
    for (int32_t k = 0; k < ncheck; ++k) ok[k] = 1;
    const int64_t nt = nthreads > 1 ? nthreads : 1;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t a = nrows * t / nt, b = nrows * (t + 1) / nt;
        for (int32_t k = 0; k < ncheck; ++k) {
            int good = 1;
            for (int64_t r = a; r < b && good; ++r) {
                const int64_t c = r * ncols + cols[k];
                if (!(cfl[c] & KWCSV_NA) && !utf8_cell_ok(out + coff[c], coff[c + 1] - coff[c])) good = 0;
            }
            if (!good) {
                #pragma omp atomic write
                ok[k] = 0;
            }
        }
    }
}

/*
 * kwcsv_parse of exactly `rows` records whose starts kwcsv_records found (starts[0..rows]), over nthreads
 * threads: each tokenizes a contiguous row range into out at its records' own byte offset (a record's cells
 * never take more than its bytes), then the ranges are moved down, in order, so out / coff / cfl are exactly
 * kwcsv_parse's.  out needs starts[rows] - starts[0] + 16 bytes.  Returns rows, or kwcsv_parse's negative
 * code of the first failing range.
 */
int64_t kwcsv_parse_mt(const uint8_t *buf, int64_t len, const int64_t *starts, int64_t rows, int32_t ncols,
                       const uint8_t *na, const int32_t *na_off, int32_t n_na, uint8_t *out, int64_t *coff,
                       uint8_t *cfl, int32_t nthreads)
{
    int64_t nt = nthreads > 1 ? nthreads : 1;
    if (nt > rows / 64 + 1) nt = rows / 64 + 1;
    int64_t *used = (int64_t *)calloc((size_t)nt, sizeof(int64_t));
    int64_t *rc = (int64_t *)calloc((size_t)nt, sizeof(int64_t));
    if (!used || !rc) { free(used); free(rc); return -4; }
    coff[0] = 0;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t t = 0; t < nt; ++t) {
        const int64_t a = rows * t / nt, b = rows * (t + 1) / nt;
        if (b <= a) continue;
        const int64_t base = starts[a] - starts[0];
        int64_t pos_out = 0;
        /* offsets relative to the range's own start; coff[a * ncols] is range t - 1's last end */
        const int64_t got = parse_body(buf, len, starts[a], b - a, ncols, na, na_off, n_na, out + base,
                                       starts[b] - starts[a] + 16, coff + a * ncols, cfl + a * ncols, &pos_out,
                                       NULL);
        rc[t] = got == b - a ? 0 : (got < 0 ? got : -2);
        used[t] = got == b - a ? coff[b * ncols] : 0;
    }
    /* the ranges are separate: move each down to the end of the previous one, in order (dest <= source) */
    int64_t dest = 0, err = 0;
    for (int64_t t = 0; t < nt && !err; ++t) {
        const int64_t a = rows * t / nt, b = rows * (t + 1) / nt;
        if (rc[t]) { err = rc[t]; break; }
        if (b <= a) continue;
        const int64_t base = starts[a] - starts[0];
        if (dest != base) memmove(out + dest, out + base, (size_t)used[t]);
        const int64_t shift = dest;
        for (int64_t j = a * ncols + 1; j <= b * ncols; ++j) coff[j] += shift;
        dest += used[t];
    }
    free(used);
    free(rc);
    return err ? err : rows;
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

/* kwcsv_pack over nthreads threads (row lengths, one prefix sum, parallel copies): the same arena / offsets. */
int64_t kwcsv_pack_mt(const uint8_t *out, const int64_t *coff, const uint8_t *cfl, int64_t nrows, int32_t ncols,
                      int32_t ct, int32_t ci, uint8_t *arena, int64_t cap, int64_t *off, int32_t nthreads)
{
    const int64_t nt = nthreads > 1 ? nthreads : 1;
    off[0] = 0;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t r = 0; r < nrows; ++r)
        for (int k = 0; k < 2; ++k) {
            const int64_t c = r * ncols + (k ? ci : ct);
            off[2 * r + k + 1] = (cfl[c] & KWCSV_NA) ? 3 : coff[c + 1] - coff[c];
        }
    for (int64_t i = 1; i <= 2 * nrows; ++i) off[i] += off[i - 1];
    if (off[2 * nrows] > cap) return -1;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t r = 0; r < nrows; ++r)
        for (int k = 0; k < 2; ++k) {
            const int64_t c = r * ncols + (k ? ci : ct);
            if (cfl[c] & KWCSV_NA) memcpy(arena + off[2 * r + k], "nan", 3);
            else memcpy(arena + off[2 * r + k], out + coff[c], (size_t)(coff[c + 1] - coff[c]));
        }
    return off[2 * nrows];
}

static int64_t days_from_civil(int64_t y, int64_t m, int64_t d)
{
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

/*
 * The article dates of column `col` (match_keywords.py:152: dateutil.parse(str(v)) if notna(v) else None),
 * for the cells whose answer needs no dateutil: kind[r] = 2 for an NA cell (None); kind[r] = 1 for a cell of
 * exactly the dataset's layout 'YYYY-MM-DD HH:MM:SS' ('T' or ' ' between date and time, ASCII digits)
 * forming a valid date and time with year >= 1000, which dateutil parses to the naive datetime of those
 * fields -- us[r] = its epoch microseconds, naive read as UTC (kb.epoch_us); kind[r] = 0 otherwise (the
 * caller runs dates.parse_date, i.e. dateutil, on that cell).  The same rule as dates.parse_date's fast path.
 */
void kwcsv_dates(const uint8_t *out, const int64_t *coff, const uint8_t *cfl, int64_t nrows, int32_t ncols,
                 int32_t col, int64_t *us, uint8_t *kind, int32_t nthreads)
{
    static const int dim[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    const int64_t nt = nthreads > 1 ? nthreads : 1;
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t r = 0; r < nrows; ++r) {
        const int64_t c = r * ncols + col;
        us[r] = 0;
        if (cfl[c] & KWCSV_NA) { kind[r] = 2; continue; }
        kind[r] = 0;
        const uint8_t *s = out + coff[c];
        if (coff[c + 1] - coff[c] != 19) continue;
        static const int8_t digit_at[19] = {1, 1, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1, 0, 1, 1};
        int ok = s[4] == '-' && s[7] == '-' && (s[10] == ' ' || s[10] == 'T') && s[13] == ':' && s[16] == ':';
        for (int i = 0; i < 19 && ok; ++i)
            if (digit_at[i] && (s[i] < '0' || s[i] > '9')) ok = 0;
        if (!ok) continue;
#define D2(i) ((int64_t)(s[i] - '0') * 10 + (s[(i) + 1] - '0'))
        const int64_t y = D2(0) * 100 + D2(2), mo = D2(5), d = D2(8), hh = D2(11), mi = D2(14), ss = D2(17);
#undef D2
        if (y < 1000 || mo < 1 || mo > 12 || hh >= 24 || mi >= 60 || ss >= 60) continue;
        const int leap = (y % 4 == 0) && (y % 100 != 0 || y % 400 == 0);
        const int64_t md = (mo == 2 && leap) ? 29 : dim[mo - 1];
        if (d < 1 || d > md) continue;
        us[r] = ((days_from_civil(y, mo, d) * 86400) + hh * 3600 + mi * 60 + ss) * 1000000;
        kind[r] = 1;
    }
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

/* QUOTE_MINIMAL length of one cell (put_cell's output length) */
static int64_t cell_len_q(const uint8_t *s, int64_t n)
{
    if (n <= 0) return 0;
    if (!memchr(s, ',', (size_t)n) && !memchr(s, '"', (size_t)n) && !memchr(s, '\n', (size_t)n)) return n;
    int64_t q = 0;
    for (const uint8_t *p = s; (p = (const uint8_t *)memchr(p, '"', (size_t)(s + n - p))) != NULL; ++p) ++q;
    return n + q + 2;
}

/*
 * kwcsv_emit over nthreads threads, the same bytes, line_off and flags: (1) each article that has rows renders
 * its date_time cell and its title .. article_text cells once, in parallel, into `art` (at a bound computed
 * from its cell lengths); (2) every row's line length (its time stamp digits, the article's two parts, its
 * quoted JSON cells) and a prefix sum give each row its offset; (3) the rows are written in parallel.
 * art needs kwcsv_emit_art_bytes() bytes.  Returns 0, -1 when out is too small (line_off[nrows] then holds
 * the bytes needed), -2 for a NUL character in a cell, -3 on an allocation failure.
 */
int64_t kwcsv_emit_art_bytes(const int64_t *coff, int32_t ncols, const int32_t *cols, const int32_t *row_doc,
                             int64_t nrows)
{
    int32_t dmax = -1;
    for (int64_t r = 0; r < nrows; ++r) if (row_doc[r] > dmax) dmax = row_doc[r];
    int64_t total = 0;
    for (int32_t d = 0; d <= dmax; ++d) {
        const int64_t base = (int64_t)d * ncols;
        total += 16;
        for (int c = 0; c < 6; ++c) total += 2 * (coff[base + cols[c] + 1] - coff[base + cols[c]]) + 3;
    }
    return total + 64;
}

/* put_cell without a capacity check: the caller sized the line with cell_len_q */
static void put_cell_sized(uint8_t *out, int64_t *o, const uint8_t *s, int64_t n)
{
    if (cell_len_q(s, n) == n) {
        memcpy(out + *o, s, (size_t)n);
        *o += n;
        return;
    }
    out[(*o)++] = '"';
    for (int64_t i = 0; i < n; ++i) {
        if (s[i] == '"') out[(*o)++] = '"';
        out[(*o)++] = s[i];
    }
    out[(*o)++] = '"';
}

static int stamp_digits(int64_t v, char *num)   /* decimal text of v at the end of num[24]; returns the start */
{
    int k = 24;
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1u : (uint64_t)v;
    do { num[--k] = (char)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) num[--k] = '-';
    return k;
}

int64_t kwcsv_emit_mt(const uint8_t *cells, const int64_t *coff, const uint8_t *cfl, int32_t ncols,
                      const int32_t *cols, const int32_t *row_doc, const int64_t *row_stamp, int64_t nrows,
                      const uint8_t *json, const int64_t *json3, uint8_t *out, int64_t cap, int64_t *line_off,
                      uint32_t *flags, uint8_t *art, int32_t nthreads)
{
    const int64_t nt = nthreads > 1 ? nthreads : 1;
    int32_t dmax = -1;
    for (int64_t r = 0; r < nrows; ++r) if (row_doc[r] > dmax) dmax = row_doc[r];
    const int64_t nd = (int64_t)dmax + 1;
    int64_t *part = (int64_t *)malloc(sizeof(int64_t) * 3 * (size_t)(nd > 0 ? nd : 1));   /* A start, B start, B end */
    int64_t *abase = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nd + 1));
    uint32_t *dfl = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(nd > 0 ? nd : 1));
    uint8_t *used = (uint8_t *)calloc((size_t)(nd > 0 ? nd : 1), 1);
    if (!part || !abase || !dfl || !used) { free(part); free(abase); free(dfl); free(used); return -3; }
    for (int64_t r = 0; r < nrows; ++r) used[row_doc[r]] = 1;
    abase[0] = 0;
    for (int64_t d = 0; d < nd; ++d) {
        const int64_t base = d * ncols;
        int64_t need = 16;
        for (int c = 0; c < 6; ++c) need += 2 * (coff[base + cols[c] + 1] - coff[base + cols[c]]) + 3;
        abase[d + 1] = abase[d] + (used[d] ? need : 0);
    }
    int64_t err = 0;
    /* (1) the articles' shared cells */
    #pragma omp parallel for num_threads(nt) schedule(dynamic, 64) reduction(min : err)
    for (int64_t d = 0; d < nd; ++d) {
        if (!used[d]) continue;
        const int64_t base = d * ncols;
        const int64_t lim = abase[d + 1];
        int64_t o = abase[d];
        uint32_t fl = 0;
        int e = emit_chunk_cell(cells, coff, cfl, base + cols[0], 0, art, lim, &o, &fl);
        const int64_t b0 = o;
        for (int c = 3; c < 8 && e == 0; ++c) {
            if (c > 3) art[o++] = ',';
            e = emit_chunk_cell(cells, coff, cfl, base + cols[c - 2], c, art, lim, &o, &fl);
        }
        if (e) { err = e < err ? e : err; continue; }
        part[3 * d] = abase[d];
        part[3 * d + 1] = b0;
        part[3 * d + 2] = o;
        dfl[d] = fl;
    }
    if (err) { free(part); free(abase); free(dfl); free(used); return err; }
    /* (2) line lengths -> offsets */
    #pragma omp parallel for num_threads(nt) schedule(static) reduction(min : err)
    for (int64_t r = 0; r < nrows; ++r) {
        const int32_t d = row_doc[r];
        char num[24];
        int64_t n = 24 - stamp_digits(row_stamp[r], num);
        n += 1 + (part[3 * d + 1] - part[3 * d]);
        uint32_t fl = dfl[d] | 6u;   /* the JSON cells are text witnesses */
        for (int c = 1; c < 3; ++c) {
            const uint8_t *s = json + json3[3 * r + (c - 1)];
            const int64_t m = json3[3 * r + c] - json3[3 * r + (c - 1)];
            if (m > 0 && memchr(s, 0, (size_t)m)) err = -2;
            if (m > 0 && memchr(s, '\r', (size_t)m)) fl |= 1u << 16;
            n += 1 + cell_len_q(s, m);
        }
        n += 1 + (part[3 * d + 2] - part[3 * d + 1]) + 1;
        line_off[r + 1] = n;
        flags[r] = fl;
    }
    if (err) { free(part); free(abase); free(dfl); free(used); return err; }
    line_off[0] = 0;
    for (int64_t r = 0; r < nrows; ++r) line_off[r + 1] += line_off[r];
    if (line_off[nrows] > cap) { free(part); free(abase); free(dfl); free(used); return -1; }
    /* (3) the rows */
    #pragma omp parallel for num_threads(nt) schedule(static)
    for (int64_t r = 0; r < nrows; ++r) {
        const int32_t d = row_doc[r];
        char num[24];
        const int k = stamp_digits(row_stamp[r], num);
        int64_t o = line_off[r];
        memcpy(out + o, num + k, (size_t)(24 - k));
        o += 24 - k;
        out[o++] = ',';
        const int64_t la = part[3 * d + 1] - part[3 * d], lb = part[3 * d + 2] - part[3 * d + 1];
        memcpy(out + o, art + part[3 * d], (size_t)la);
        o += la;
        for (int c = 1; c < 3; ++c) {
            const uint8_t *s = json + json3[3 * r + (c - 1)];
            const int64_t m = json3[3 * r + c] - json3[3 * r + (c - 1)];
            out[o++] = ',';
            put_cell_sized(out, &o, s, m);
        }
        out[o++] = ',';
        memcpy(out + o, art + part[3 * d + 1], (size_t)lb);
        o += lb;
        out[o++] = '\n';
    }
    free(part);
    free(abase);
    free(dfl);
    free(used);
    return 0;
}
