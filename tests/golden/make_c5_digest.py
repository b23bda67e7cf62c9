"""Pin config 5 at its stated size: the CPU oracle's keep-first over bench.py's 500M synthetic CDX rows.

Input: rows 0..499 999 999 of the seeded URL generator (csrc/synth.c ``generate_urls``, seed 20250905,
``n_articles = int(1.31 * 500M)``: exactly what ``bench.py --workload dedup`` at N = 1 and
``synth.generate_urls(500_000_000, seed)`` produce).  Every row goes through the oracle's
``url_transform`` (oracle/dedup_oracle.py, the restatement of yahoo_links_selenium.py:63-76 pinned by the
reference-run fixtures in dedup_golden.json.gz) and the keep-first of :79/:174
(``drop_duplicates(subset=['url'])``, keep='first').

The keep-first runs hash-partitioned so it fits in memory: each transformed URL's 128-bit xxh3 picks one
of 64 partitions; equal URLs land in the same partition, in row order, so the first row of each distinct
URL inside its partition is its first row overall.  Within a partition, rows are grouped by the 128-bit
hash (a collision between two different URLs among 5e8 rows has probability ~4e-22; the hash stands in
for the byte compare only there).

Committed (tests/golden/c5_digest.json, < 1 KB): the four row counts per KW_URL_* code, the kept bytes,
and two order-independent digests of the kept set (tests/bytes_digest.py): of the kept row indices and of
the kept normalised URLs' bytes.  tests/test_gpu_dedup.py::test_c5_500m_rows_vs_oracle_digest compares
kw_dedup_run's result on the GPU box with them.

    python tests/golden/make_c5_digest.py [--procs 6] [--rows 500000000]

Runs in the build container on CPU (~3 us of Python per row), never on GPU minutes.  Partition files go
to tests/golden/_local/c5/ (git-ignored, deleted at the end).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import shutil
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

SEED = 20250905
CHUNK = 2_000_000
NPART = 64
REC = np.dtype([('hi', '<u8'), ('lo', '<u8'), ('row', '<i8'), ('bh', '<u8'), ('len', '<u4')])


def _chunk(args):
    lo, hi, n_articles = args
    import xxhash
    from advanced_scrapper_amd import synth
    from oracle import dedup_oracle as orc
    from tests import bytes_digest as ud
    u = synth.generate_urls(hi - lo, seed=SEED, row_base=lo, n_articles=n_articles)
    n = hi - lo
    counts = np.zeros(4, np.int64)              # KW_URL_NO_HTML, KEPT (valid here), FILTERED, DUPLICATE
    rows, keys = [], []
    html = orc._HTML
    for i in range(n):
        s = u.url(i)
        k = orc.url_transform(s)
        if k is None:
            counts[0 if html.search(s) is None else 2] += 1
            continue
        rows.append(lo + i)
        keys.append(k.encode('utf-8', 'surrogatepass'))
    counts[1] = len(rows)
    rec = np.zeros(len(rows), REC)
    rec['row'] = rows
    h = [xxhash.xxh3_128_intdigest(k) for k in keys]
    rec['hi'] = np.array([x >> 64 for x in h], dtype=np.uint64)
    rec['lo'] = np.array([x & 0xFFFFFFFFFFFFFFFF for x in h], dtype=np.uint64)
    lens = np.fromiter((len(k) for k in keys), dtype=np.int64, count=len(keys))
    rec['len'] = lens
    off = np.zeros(len(keys) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    arena = np.frombuffer(b''.join(keys), dtype=np.uint8)
    rec['bh'] = ud.bytehash_np(arena, off)
    part = (rec['hi'] >> np.uint64(58)).astype(np.int64)
    order = np.argsort(part, kind='stable')
    rec, part = rec[order], part[order]
    cuts = np.searchsorted(part, np.arange(NPART + 1))
    return lo, counts, [rec[cuts[p]:cuts[p + 1]].tobytes() for p in range(NPART)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=6)
    ap.add_argument('--rows', type=int, default=500_000_000)
    ap.add_argument('--out', default=os.path.join(HERE, 'c5_digest.json'))
    args = ap.parse_args()
    from tests import bytes_digest as ud
    n = args.rows
    n_articles = int(1.31 * n)
    work = os.path.join(HERE, '_local', 'c5')
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    fh = [open(os.path.join(work, f'p{p:02d}.bin'), 'wb') for p in range(NPART)]
    jobs = [(lo, min(lo + CHUNK, n), n_articles) for lo in range(0, n, CHUNK)]
    counts = np.zeros(4, np.int64)
    t0 = time.time()
    with mp.get_context('spawn').Pool(args.procs) as pool:
        for k, (lo, c, parts) in enumerate(pool.imap(_chunk, jobs)):      # ordered: files stay in row order
            counts += c
            for p in range(NPART):
                fh[p].write(parts[p])
            if k % 10 == 0:
                print(f'{k + 1}/{len(jobs)} chunks, {time.time() - t0:.0f} s', flush=True)
    for f in fh:
        f.close()
    t1 = time.time()
    n_valid = int(counts[1])
    kept_rows = kept_bytes = 0
    rdig = bdig = 0
    for p in range(NPART):
        rec = np.fromfile(os.path.join(work, f'p{p:02d}.bin'), dtype=REC)
        assert np.all(np.diff(rec['row']) > 0)
        order = np.lexsort((rec['row'], rec['lo'], rec['hi']))
        r = rec[order]
        first = np.r_[True, (r['hi'][1:] != r['hi'][:-1]) | (r['lo'][1:] != r['lo'][:-1])]
        k = r[first]
        kept_rows += len(k)
        kept_bytes += int(k['len'].sum(dtype=np.int64))
        rdig = (rdig + ud.row_digest(k['row'])) & 0xFFFFFFFFFFFFFFFF
        bdig = (bdig + ud.bytes_digest(k['bh'], k['len'])) & 0xFFFFFFFFFFFFFFFF
        del rec, r, k
    shutil.rmtree(work, ignore_errors=True)
    counts[1] = kept_rows
    counts[3] = n_valid - kept_rows
    meta = {'generator': 'tests/golden/make_c5_digest.py (CPU oracle, oracle/dedup_oracle.py url_transform + '
                         'keep-first, hash-partitioned)',
            'seed': SEED, 'rows': n, 'n_articles': n_articles,
            'counts': {'no_html': int(counts[0]), 'kept': int(counts[1]), 'filtered': int(counts[2]),
                       'duplicate': int(counts[3])},
            'kept_bytes': kept_bytes, 'row_digest': f'{rdig:016x}', 'bytes_digest': f'{bdig:016x}',
            'oracle_seconds': round(t1 - t0, 1), 'keep_first_seconds': round(time.time() - t1, 1),
            'procs': args.procs}
    with open(args.out, 'w') as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == '__main__':
    main()
