/* libkwmatch — CDX link-row normalise + keep-first dedup on the GPU (gfx950).
 *
 * Replaces the pandas steps of the reference's link harvester
 * (lwowlwowl/advanced_scrapper yahoo_links_selenium.py):
 *
 *   :63       df[df['url'].str.contains('.html')]                  (regex: any code point but '\n', then "html")
 *   :66       df['url'].str.split('.html').str[0] + '.html'        (cut before the first such match)
 *   :67       .str.replace(':80', '', regex=False)
 *   :68       .str.replace('http:', 'https:', regex=False)
 *   :75-76    drop rows containing 'news/%' or "news/'"
 *   :79, :174 drop_duplicates(subset=['url']) keep='first'           (per part, then over the glob-ordered concat)
 *
 * Keep-first over the concatenation of the parts equals the per-part dedup
 * followed by the merge dedup, so one call over all rows (parts concatenated
 * in glob order) gives the final yfin_urls.csv rows.
 *
 * Rows are UTF-8 URL strings in a caller-owned device arena: row i is
 * d_arena[d_off[i], d_off[i+1]); the arena must be readable 32 bytes past
 * d_off[n].  Every function returns 0 or a negative KW_E* code (kwmatch.h);
 * kw_dedup_last_error gives the message.  A handle is not thread-safe.
 */
#ifndef KWDEDUP_H
#define KWDEDUP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-row outcome codes written to d_code */
#define KW_URL_NO_HTML 0      /* dropped by :63 */
#define KW_URL_KEPT 1         /* first occurrence of its normalised URL */
#define KW_URL_FILTERED 2     /* dropped by :75-76 */
#define KW_URL_DUPLICATE 3    /* dropped by :79 / :174 */

typedef struct kw_dedup kw_dedup;

int kw_dedup_create(int32_t device, kw_dedup **out);

/* flags of kw_dedup_run */
#define KW_DEDUP_NORMALIZE 1  /* apply :63-76 before the keep-first; without it the keep-first runs on the raw
                                 strings (the merge step :174 over part CSVs that are already normalised) */

/* Classify n rows; d_code (caller-owned, n bytes) receives one KW_URL_* code per
 * row.  Runs on `stream` (a hipStream_t, NULL = default) and returns when the
 * codes are final (the rare 64-bit hash-tag collisions are resolved by an exact
 * host pass over the colliding rows). */
int kw_dedup_run(kw_dedup *h, const uint8_t *d_arena, const int64_t *d_off, int64_t n, int32_t flags,
                 uint8_t *d_code, void *stream);

/* Row counts per code of the last run: counts[KW_URL_*] (4 values). */
int kw_dedup_counts(kw_dedup *h, int64_t *counts);

/* Size of the last run's kept rows: their number and the bytes of their normalised URLs. */
int kw_dedup_kept_size(kw_dedup *h, int64_t *n_kept, int64_t *n_bytes);

/* The kept rows, dense and in row order, into caller-owned device buffers:
 * d_bytes (n_bytes), d_off (n_kept + 1 offsets into d_bytes), d_rows (n_kept source row indices). */
int kw_dedup_kept_copy(kw_dedup *h, uint8_t *d_bytes, int64_t *d_off, int64_t *d_rows, void *stream);

/* Device times (ms) of the last run: [0] transform + hash + table insert, [1] the byte-serial rows
 * (rewrite + insert), [2] decide (rep compare), [3] kept compaction, [4] total; k <= 5 values. */
int kw_dedup_last_ms(kw_dedup *h, float *ms, int32_t k);

const char *kw_dedup_last_error(kw_dedup *h);
int kw_dedup_destroy(kw_dedup *h);

/* One-shot form: d_keep_mask[i] = 1 iff row i is kept. */
int dedup_urls(const uint8_t *d_arena, const int64_t *d_off, int64_t n, uint8_t *d_keep_mask, void *stream);

#ifdef __cplusplus
}
#endif

#endif
