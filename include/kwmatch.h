/*
 * kwmatch.h — C-ABI of libkwmatch.so, the MI355X (gfx950) ticker<->news
 * keyword matcher.
 *
 * What it replaces.  The reference has no FFI on this path: its operator
 * boundary is the Python function
 *     process_chunk(source_name, chunk, processed_data)   match_keywords.py:148
 * whose inner loops (match_keywords.py:159-180) run, per article and per name,
 *   - the uppercase branch  re.finditer(r'\b'+re.escape(name)+r'\b', s)      :165-173
 *   - the fuzzy branch      rapidfuzz.fuzz.partial_ratio(s, name) > 95        :174-176
 *                           followed by re.finditer(name, s)                  :177-180
 * on s = article_text and s = title (:150-151).  This library computes exactly
 * those per-(article, field, name) results on the GPU.  Everything around them
 * (knowledge-base loading :40-120, the period filter :17-37/:164, the
 * per-ticker dict assembly :159-187, CSV egress :128-146/:195-217) stays in the
 * host module advanced_scrapper_amd/match_keywords.py, which is the drop-in
 * replacement of the reference script and binds this header with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions: every function returns 0 on success or a negative KW_E* code;
 * kw_last_error(h) gives a message.  Handles are not thread-safe: use one
 * handle per device and per host thread.  Device pointers passed to kw_scan are
 * caller-owned (e.g. torch uint8/int64 tensors); kw_scan is asynchronous on the
 * given HIP stream.
 */
#ifndef KWMATCH_H
#define KWMATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes */
#define KW_OK 0
#define KW_EINVAL -1        /* bad argument */
#define KW_EUNSUPPORTED -2  /* pattern outside the supported subset (see kw_compile) */
#define KW_EHIP -3          /* HIP runtime error */
#define KW_EOVERFLOW -4     /* a device work buffer overflowed; see kw_last_error */
#define KW_ESTATE -5        /* call out of order (e.g. kw_hits before kw_scan) */

/* pattern classes (match_keywords.py:165-174) */
#define KW_CLASS_UPPER 'U'  /* name.isupper() and len(name) > 1: \b-bounded literal */
#define KW_CLASS_FUZZY 'F'  /* the fuzzy branch: partial_ratio > 95, then re.finditer */

/* regex atom program of a fuzzy-class name, used for the positions of
 * re.finditer(name, s) (match_keywords.py:177-180).  Four int32 per atom:
 * {op, value, min, max}; op 0 = literal code point `value`, op 1 = '.'
 * (any code point except '\n'); the atom repeats greedily min..max times
 * (max = -1: unbounded).  A pattern with rx_off[i] == rx_off[i+1] is matched
 * literally (its atoms are its code points). */
#define KW_RX_LIT 0
#define KW_RX_ANY 1

typedef struct kw_handle kw_handle;

/* One result record.  pos is a code-point offset (str index) of a match start
 * in the field; KW_NOPOS marks a fuzzy-branch match whose re.finditer found
 * no position (the reference stores `name: []`, match_keywords.py:177-180). */
typedef struct {
    uint32_t doc;      /* document index within the scanned batch */
    uint32_t pattern;  /* pattern index as passed to kw_compile */
    uint32_t pos;      /* code-point offset or KW_NOPOS */
    uint32_t field;    /* 0 = article_text, 1 = title */
} kw_hit;
#define KW_NOPOS 0xFFFFFFFFu

/* Compile the active names into device tables on `device`.
 *   pat_bytes/pat_off : UTF-8 of n_pat names, name i = pat_bytes[pat_off[i]:pat_off[i+1]]
 *   pat_class         : KW_CLASS_UPPER or KW_CLASS_FUZZY per name.  Names of the
 *                       other two reference classes (single uppercase char,
 *                       lowercase-alpha) never match and must not be passed.
 *                       Order: all 'U' names first, then the 'F' names sorted by
 *                       code-point length, longest first.
 *   rx_atoms/rx_off   : regex programs (see KW_RX_*), rx_off has n_pat+1 entries;
 *                       may be NULL (all names literal).
 *   word_bitmap       : 0x110000 bits, bit c set iff chr(c).isalnum() or c == '_'
 *                       (CPython's \b word class, Unicode database of the host).
 *   bg/bg_len         : optional background sample of the article text (UTF-8).  Its
 *                       4-byte q-gram counts price the anchor substrings and the
 *                       pigeonhole piece cuts; any sample (or none) gives the same
 *                       results, only the speed changes.
 * Fuzzy names longer than 64 code points or one byte long are KW_EUNSUPPORTED
 * (rapidfuzz switches algorithm above 64). */
int kw_compile(const uint8_t *pat_bytes, const int64_t *pat_off, const uint8_t *pat_class, int32_t n_pat,
               const int32_t *rx_atoms, const int64_t *rx_off, const uint32_t *word_bitmap, const uint8_t *bg,
               int64_t bg_len, int32_t device, kw_handle **out);

/* Scan n_docs documents.  d_arena: UTF-8 bytes; d_doc_off: 2*n_docs+1 int64
 * byte offsets, text of doc d = [off[2d], off[2d+1]), title = [off[2d+1],
 * off[2d+2]).  The host has already applied the str()/NaN rules of
 * match_keywords.py:150-151 (NaN -> "nan").  stream: a hipStream_t (NULL =
 * default stream).  Asynchronous. */
int kw_scan(kw_handle *h, const uint8_t *d_arena, const int64_t *d_doc_off, int64_t n_docs, void *stream);

/* Wait for the last scan and return its records (device memory owned by the
 * library, valid until the next kw_scan or kw_destroy).  Records are grouped
 * by document but not sorted. */
int kw_hits(kw_handle *h, int64_t *n_hits, const kw_hit **d_hits);

/* Copy the last scan's records into a caller-owned device buffer of capacity
 * `cap` records (asynchronous on `stream`); *n_hits receives the count. */
int kw_hits_copy(kw_handle *h, kw_hit *d_dst, int64_t cap, int64_t *n_hits, void *stream);

/* Scan statistics of the last kw_scan (after kw_hits), up to KW_N_STATS values:
 * [0] byte positions that passed the stage-1 LDS filter, [1] anchor
 * occurrences, [2] LCS windows evaluated, [3] fuzzy verifications, [4]
 * documents handed to the generic kernel, of which [5] had more anchor items
 * than the fast path holds and [6] had a long non-ASCII field, [7] one-deletion
 * edge windows found (fuzzy names of 11..20 code points), [8] candidates that
 * passed the stage-2 filter, [9] documents the resolve kernel worked on,
 * [10] regex-position searches of decided regex-class names, of which [11]
 * ran the backtracking engine (quantified atoms), [12] 2048-position rounds of
 * the shift-and search; the all-ASCII documents the epilogue deferred because
 * [13] a name had more than 64 items in a field, [14] a field had more items
 * than the fast path holds, [15] the probe or filter flagged them (an item batch
 * beyond the probe's pool, a field beyond 8 MiB); [16] all-ASCII documents
 * finished by the big-document epilogue (more than 512 / 64 items); [17] times
 * the batch was scanned again after a device buffer grew (0 once the buffers
 * fit the workload: growth persists across kw_scan calls); documents with a
 * non-ASCII field that [18] the epilogue finished on their transcoded view (one
 * byte per code point) or [19] it left to the resolve kernel; [20] why the
 * batch was scanned again: the KW_RESCAN_* bits of every buffer that overflowed
 * in a scan that was redone. */
#define KW_N_STATS 21
#define KW_RESCAN_GENERIC_ITEMS 1   /* the generic kernel's items per field */
#define KW_RESCAN_RESULTS 2         /* a wave's result region */
#define KW_RESCAN_GENERIC_CPS 4     /* the generic kernel's code points per field */
#define KW_RESCAN_REGEX_QUEUE 16    /* a resolve wave's regex-search queue */
#define KW_RESCAN_TASK_QUEUES 32    /* a scan wave's verify / short / regex task queues */
#define KW_RESCAN_DECIDED_SET 64    /* the decided (doc, field, name) set */
#define KW_RESCAN_REGIONS 128       /* a filter region's candidates or a probe region's items */
int kw_stats(kw_handle *h, int64_t *stats, int32_t n_stats);

/* Device times (ms) of the last kw_scan, from HIP events on the scan's streams
 * (valid after kw_hits): the fast path up to the generic kernel's start (scan +
 * resolve kernels), the generic kernel that redoes deferred documents, and
 * everything including result compaction. */
int kw_last_kernel_ms(kw_handle *h, float *fast_ms, float *generic_ms, float *total_ms);

/* Per-kernel device times (ms) of the last kw_scan, up to 10 values: [0] scan
 * (filter + probe + epilogue kernels), [1] resolve phase (the resolve kernels
 * on the side stream, from the epilogue's end to the generic kernel's start),
 * [2] generic (side stream, beside the task kernels), [3] result compaction
 * and any wait for the task kernels, [4] total, [5] filter kernel, [6] probe
 * kernel, [7] epilogue kernel, [8] resolve kernel (side stream), [9] task
 * kernels (from the epilogue's end). */
int kw_last_kernel_times(kw_handle *h, float *ms, int32_t n);

/* Which kernel finished each document of the last scan (after kw_hits):
 * routes[d] = KW_ROUTE_SCAN (the scan kernel's epilogue and its task kernels),
 * KW_ROUTE_TRANSCODE (a non-ASCII field: the epilogue on the document's
 * transcoded view, then the task kernels), KW_ROUTE_RESOLVE (the resolve kernels: non-ASCII
 * fields the view cannot take, big documents past an epilogue queue) or KW_ROUTE_GENERIC (deferred
 * to the generic kernel: capacity limits).  For tests and tuning. */
#define KW_ROUTE_SCAN 0
#define KW_ROUTE_RESOLVE 1
#define KW_ROUTE_GENERIC 2
#define KW_ROUTE_TRANSCODE 3
int kw_doc_routes(kw_handle *h, uint8_t *routes, int64_t n);

/* Host-buffer forms of kw_scan / kw_hits_copy for callers with no device allocator of their own (the
 * drop-in driver's single-GPU path runs without torch).  kw_scan_host copies the host arena
 * (arena_bytes bytes) and the 2*n_docs+1 offsets into library-owned device buffers (grown on demand, kept
 * across calls) on a stream of the handle, then scans them (asynchronous; the host buffers may be reused
 * once kw_hits_host returns).  kw_hits_host waits for the scan and copies its records into dst (host, cap
 * records); *n_hits receives the count. */
int kw_scan_host(kw_handle *h, const uint8_t *arena, int64_t arena_bytes, const int64_t *doc_off, int64_t n_docs);
int kw_hits_host(kw_handle *h, kw_hit *dst, int64_t cap, int64_t *n_hits);

/* HIP devices visible to this process (0 when the runtime finds none). */
int kw_device_count(int32_t *n);

/* Select `device` and create its context, so a caller can start the HIP runtime early (e.g. on a
 * thread, while it reads its inputs); every other entry point does this on first use anyway. */
int kw_device_init(int32_t device);

const char *kw_last_error(kw_handle *h);
int kw_destroy(kw_handle *h);

/* ---- multi-GPU exchange (RCCL over xGMI; advanced_scrapper_amd/csrc/kwcomm.hip)
 *
 * Replaces the reference's process pool over article sub-chunks
 * (match_keywords.py:230-238, np.array_split + Pool.starmap; the workers'
 * only exchange is the shared per-ticker CSV files).  Here each rank (one
 * process per GPU) scans a contiguous, byte-balanced document range; the hit
 * counts and the packed kw_hit records are then exchanged so that the writing
 * rank holds the batch's records in document order.  RCCL is loaded at run
 * time; without it these calls return KW_EUNSUPPORTED. */
typedef struct kw_comm kw_comm;
#define KW_COMM_ID_BYTES 128

/* A fresh communicator id (ncclGetUniqueId), made by ONE rank and shared with
 * the others by the caller (e.g. torch.distributed's store). */
int kw_comm_unique_id(uint8_t *id_out /* KW_COMM_ID_BYTES */);

/* Join the communicator `id` as `rank` of `nranks` on HIP device `device`. */
int kw_comm_init(int32_t nranks, int32_t rank, const uint8_t *id, int32_t device, kw_comm **out);

/* All-gather one count per rank into counts[nranks] (host).  Blocking.  A rank
 * that cannot take part in the step's record exchange (e.g. its global
 * document ids would pass 2^32) sends count = -1: every rank's
 * kw_allgather_hits_planned on those counts then returns KW_EINVAL before
 * anything is posted. */
int kw_allgather_counts(kw_comm *c, int64_t count, int64_t *counts, void *stream);

/* Exchange hit records (e.g. a kw_hits_copy of this rank's last scan: d_local,
 * n records).  Every record's doc gets doc_base added (the rank's first global
 * document).  root < 0: every rank receives all records; root >= 0: only rank
 * `root` does (d_out may be NULL elsewhere).  The receiver's d_out (cap
 * records) gets the ranks' records concatenated in rank order = global
 * document order.  *n_total = records over all ranks; counts[nranks] (host,
 * optional) the per-rank counts.  One blocking exchange of (count, receiver
 * capacity, error flag) triples (every rank must call), then the records move
 * asynchronously on `stream` (RCCL send/recv over the xGMI mesh), so the next
 * kw_scan can run beside them on another stream.  A receiver whose cap cannot
 * hold the total makes EVERY rank return KW_EOVERFLOW, and a rank whose global
 * document ids pass 2^32 makes every rank return KW_EINVAL, before any record
 * moves.  Use one stream per communicator. */
int kw_allgather_hits(kw_comm *c, const kw_hit *d_local, int64_t n, int64_t doc_base, int32_t root, kw_hit *d_out,
                      int64_t cap, int64_t *n_total, int64_t *counts, void *stream);

/* kw_allgather_hits with the counts of this step already exchanged
 * (counts[nranks] from kw_allgather_counts, the same array on every rank, and
 * counts[rank] == n): no further exchange and no host wait, so one step costs
 * one blocking counts exchange (the caller sizes d_out from it).  A receiver
 * whose d_out is short still receives (into a library buffer) so that no peer
 * waits, and returns KW_EOVERFLOW; the other ranks return KW_OK.  Counts with
 * a negative entry fail every rank (KW_EINVAL) before anything is posted.  A
 * rank whose own arguments disagree with them (counts[rank] != n, ids past
 * 2^32) still posts its matching sends / receives (zero records of the
 * agreed sizes) so no peer waits, and returns KW_EINVAL. */
int kw_allgather_hits_planned(kw_comm *c, const kw_hit *d_local, int64_t n, int64_t doc_base, int32_t root,
                              const int64_t *counts, kw_hit *d_out, int64_t cap, int64_t *n_total, void *stream);

/* The capacity rule kw_allgather_hits agrees on (pure host): KW_OK when every
 * receiving rank r (root < 0: all; else root) has caps[r] >= the sum of
 * counts; else KW_EOVERFLOW with *bad_rank = the first short receiver.  Given
 * the same gathered (counts, caps), every rank reaches the same verdict. */
int kw_exchange_caps_ok(int32_t nranks, int32_t root, const int64_t *counts, const int64_t *caps, int32_t *bad_rank);

/* The exchange plan kw_allgather_hits runs, as a pure host function (no GPU,
 * no RCCL; tests check it against a gloo execution): given every rank's
 * record count counts[nranks] and the root (< 0: all ranks receive), rank
 * `rank`'s part of the plan:
 *   recv_off[nranks + 1]  where each rank's records land in a receiver's
 *                         output (the prefix sums: rank order = document order)
 *   ops[nranks]           per peer p: KW_PLAN_SEND (this rank sends its records
 *                         to p), KW_PLAN_RECV (it receives cnt[p] records of p
 *                         at recv_off[p]); 0 for itself and idle pairs
 *   *n_total              all records; *n_recv: records this rank ends with
 *                         (n_total on a receiver, else 0)
 * Returns KW_EINVAL on bad arguments (rank/root out of range, a negative count). */
#define KW_PLAN_SEND 1
#define KW_PLAN_RECV 2
int kw_exchange_plan(int32_t nranks, int32_t rank, int32_t root, const int64_t *counts, int64_t *recv_off,
                     int32_t *ops, int64_t *n_total, int64_t *n_recv);

const char *kw_comm_last_error(kw_comm *c);
int kw_comm_destroy(kw_comm *c);

#ifdef __cplusplus
}
#endif
#endif
