"""Pin the WHOLE config-2 (and config-4) bench corpus: per-document oracle digests (tests/golden/c2_digests.npz,
tests/golden/c4_digests.npz).

The bench corpus is bench.py's: 1M synthetic ~2 KB articles (csrc/synth.c,
seed 20250905, documents 0..999 999) against the reference KB
(tests/golden/kb_processed.json.gz).  For every document the CPU oracle
(oracle/kwmatch_oracle.py, match_keywords.py:155-180 per field) gives
``name -> positions`` for the text and the title; those become kw_scan-shaped
records ``(doc, pattern, pos, field)`` (tests/corpus_digest.py) and the
document's digest is the wrapping sum of bench.hits_digest's record mix.  The
sum over all documents is the bench line's ``hits_digest``.

Runs in the build container on CPU (a spawn pool, ~5 ms of oracle per
article), never on GPU minutes:

    python tests/golden/make_c2_digests.py [--procs 7] [--docs 1000000]
    python tests/golden/make_c2_digests.py --config 4     # bench.py --workload kb50k's corpus and KB
                                                          # (~40 ms of oracle per article: ~1.5 h on 7 cores)
    python tests/golden/make_c2_digests.py --lo 1000000 --docs 10000000 --blocks c3_blocks
                                          # config 3's 10M documents: per-1000-document block digests
                                          # (documents 0..999 999 come from c2_digests.npz); ~1.7 h on 6 cores
    python tests/golden/make_c2_digests.py --config 4 --strided 10 --blocks c4_blocks
                                          # config 4: 10 strided 1000-document blocks in 1M..10M

Block mode (--blocks NAME): the output is NAME.npz (digest uint64[n_blocks], count uint32[n_blocks], the
wrapping sums over each 1000-document block of documents [0, --docs)) + NAME.json; the per-document arrays
go to tests/golden/_local/ (git-ignored, resumable checkpoint).  Blocks below --lo are taken from the
config's 1M per-document file.

Output: c2_digests.npz (digest uint64[n], count uint16[n]) + c2_digests.json
(seed, n_docs, corpus fingerprint, total digest, total records).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

SEED = 20250905
BLOCK = 2000
DBLOCK = 1000          # documents per committed block digest (block mode)
_W = {}


def kb_for(config: int):
    """The bench's KB of a config: 2 = the reference's info/ticker subset, 4 = synth_kb's ~52k names."""
    if config == 4:
        from advanced_scrapper_amd.synth_kb import synthetic_kb
        return synthetic_kb(2300, SEED)
    from tests import golden_data
    return golden_data.kb_processed()


def _init(config):
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from oracle import kwmatch_oracle as orc
    processed = kb_for(config)
    ckb = compile_kb(processed)
    _W['names'] = synth.injectable_names(ckb)
    _W['pid'] = {n: i for i, n in enumerate(ckb.names)}
    _W['oracle'] = orc.Oracle(processed)


def _field(s):
    import re
    from oracle import kwmatch_oracle as orc
    O = _W['oracle']
    out = {}
    for n in O.upper:
        pos = orc.upper_positions(n, s)
        if pos:
            out[n] = pos
    for n, hit in zip(O.fuzzy, O.fset.decide(s)):
        if hit:
            try:
                out[n] = orc.regex_positions(n, s)
            except re.error:
                out[n] = []
    return out


def _block(lo_hi):
    from advanced_scrapper_amd import synth
    from tests import corpus_digest as cd
    lo, hi = lo_hi
    names, kinds = _W['names']
    c = synth.generate(hi - lo, names, kinds, seed=SEED, doc_base=lo)
    rows = []
    for i in range(hi - lo):
        rows += cd.oracle_records(lo + i, [_field(c.text(i)), _field(c.title(i))], _W['pid'])
    a = np.asarray(rows, dtype=np.uint32).reshape(-1, 4)
    rec = np.ascontiguousarray(a).view(np.dtype([('doc', '<u4'), ('pattern', '<u4'), ('pos', '<u4'),
                                                   ('field', '<u4')])).reshape(-1)
    dig, cnt = cd.per_doc(rec, hi - lo, lo)
    return lo, dig, cnt


def _slice_fingerprints(n_docs, names, kinds, piece=1_000_000):
    """corpus_fingerprint of every 1M-document slice [k*piece, (k+1)*piece) of the first n_docs documents
    (slice 0 equals the 1M files' fingerprint)."""
    from advanced_scrapper_amd import synth
    from tests import corpus_digest as cd
    fps, nbytes = [], 0
    for lo in range(0, n_docs, piece):
        c = synth.generate(min(piece, n_docs - lo), names, kinds, seed=SEED, doc_base=lo)
        fps.append(cd.corpus_fingerprint(c))
        nbytes += c.n_bytes
        del c
    return fps, nbytes


def main_blocks(args):
    """Block mode: per-1000-document digests of documents [0, --docs), oracle-run for [--lo, --docs)."""
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from tests import corpus_digest as cd
    n, lo0 = args.docs, args.lo
    assert n % DBLOCK == 0 and lo0 % DBLOCK == 0
    ckb = compile_kb(kb_for(args.config))
    names, kinds = synth.injectable_names(ckb)
    local = os.path.join(HERE, '_local')
    os.makedirs(local, exist_ok=True)
    ck = os.path.join(local, f'{args.blocks}_perdoc.npz')
    dig = np.zeros(n, np.uint64)
    cnt = np.zeros(n, np.int64)
    done = np.zeros(n // DBLOCK, bool)
    if args.strided:                      # config 4 spot blocks: evenly strided over [lo, n)
        want = np.zeros(n // DBLOCK, bool)
        idx = np.linspace(lo0 // DBLOCK, n // DBLOCK - 1, args.strided).round().astype(np.int64)
        want[idx] = True
    else:
        want = np.zeros(n // DBLOCK, bool)
        want[lo0 // DBLOCK:] = True
    base = np.load(os.path.join(HERE, f'c{args.config}_digests.npz'))
    nb = min(len(base['digest']), lo0)
    dig[:nb] = base['digest'][:nb]
    cnt[:nb] = base['count'][:nb].astype(np.int64)
    done[:nb // DBLOCK] = True
    want[:nb // DBLOCK] = False
    if os.path.exists(ck):
        z = np.load(ck)
        if len(z['digest']) == n:
            m = np.repeat(z['done'], DBLOCK)
            dig[m], cnt[m] = z['digest'][m], z['count'][m]
            done |= z['done']
            print(f'resumed: {int(z["done"].sum())} blocks from {ck}', flush=True)
    todo = [(b * DBLOCK, (b + 1) * DBLOCK) for b in np.flatnonzero(want & ~done)]
    t0 = time.time()
    last = t0
    ctx = mp.get_context('spawn')
    with ctx.Pool(args.procs, initializer=_init, initargs=(args.config,)) as pool:
        for k, (lo, d, c) in enumerate(pool.imap_unordered(_block, todo)):
            dig[lo:lo + len(d)] = d
            cnt[lo:lo + len(c)] = c
            done[lo // DBLOCK] = True
            if k % 100 == 0 or time.time() - last > 600:
                print(f'{k + 1}/{len(todo)} blocks, {time.time() - t0:.0f} s', flush=True)
                if time.time() - last > 600:
                    np.savez(ck, digest=dig, count=cnt, done=done)
                    last = time.time()
    np.savez(ck, digest=dig, count=cnt, done=done)
    sel = np.flatnonzero(done)
    with np.errstate(over='ignore'):
        bdig = dig.reshape(-1, DBLOCK).sum(axis=1, dtype=np.uint64)
    bcnt = cnt.reshape(-1, DBLOCK).sum(axis=1)
    fps, nbytes = _slice_fingerprints(n, names, kinds)
    np.savez_compressed(os.path.join(HERE, args.blocks + '.npz'), block=sel.astype(np.uint32),
                        digest=bdig[sel], count=bcnt[sel].astype(np.uint32))
    meta = {'generator': 'tests/golden/make_c2_digests.py --blocks (CPU oracle, oracle/kwmatch_oracle.py)',
            'seed': SEED, 'n_docs': n, 'docs_per_block': DBLOCK, 'n_blocks_pinned': int(len(sel)),
            'all_blocks': bool(done.all()), 'corpus_bytes': nbytes, 'slice_docs': 1_000_000,
            'slice_fingerprints': fps, 'config': args.config,
            'kb': ('advanced_scrapper_amd/synth_kb.py synthetic_kb(2300, seed)' if args.config == 4
                   else 'tests/golden/kb_processed.json.gz'),
            'oracle_docs_from': lo0, 'per_document_source_below': f'c{args.config}_digests.npz',
            'total_records': int(bcnt[sel].sum()),
            'hits_digest': cd.total(bdig[sel]), 'oracle_seconds': round(time.time() - t0, 1), 'procs': args.procs}
    with open(os.path.join(HERE, args.blocks + '.json'), 'w') as fh:
        json.dump(meta, fh, indent=1)
    print(json.dumps(meta, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=7)
    ap.add_argument('--docs', type=int, default=1_000_000)
    ap.add_argument('--config', type=int, choices=(2, 4), default=2)
    ap.add_argument('--out', default=None)
    ap.add_argument('--lo', type=int, default=0, help='block mode: first document the oracle runs on')
    ap.add_argument('--blocks', default=None, help='block mode: output name (per-1000-document digests)')
    ap.add_argument('--strided', type=int, default=0, help='block mode: only this many strided blocks in [lo, docs)')
    args = ap.parse_args()
    if args.blocks:
        return main_blocks(args)
    args.out = args.out or os.path.join(HERE, f'c{args.config}_digests')
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from tests import corpus_digest as cd
    n = args.docs
    ckb = compile_kb(kb_for(args.config))
    names, kinds = synth.injectable_names(ckb)
    corpus = synth.generate(n, names, kinds, seed=SEED, doc_base=0)
    fp = cd.corpus_fingerprint(corpus)
    n_bytes = corpus.n_bytes
    del corpus
    dig = np.zeros(n, np.uint64)
    cnt = np.zeros(n, np.int64)
    blocks = [(lo, min(lo + BLOCK, n)) for lo in range(0, n, BLOCK)]
    t0 = time.time()
    ctx = mp.get_context('spawn')
    with ctx.Pool(args.procs, initializer=_init, initargs=(args.config,)) as pool:
        for k, (lo, d, c) in enumerate(pool.imap_unordered(_block, blocks)):
            dig[lo:lo + len(d)] = d
            cnt[lo:lo + len(c)] = c
            if k % 25 == 0:
                print(f'{k + 1}/{len(blocks)} blocks, {time.time() - t0:.0f} s', flush=True)
    assert cnt.max() < 65536
    np.savez_compressed(args.out + '.npz', digest=dig, count=cnt.astype(np.uint16))
    meta = {'generator': 'tests/golden/make_c2_digests.py (CPU oracle, oracle/kwmatch_oracle.py)',
            'seed': SEED, 'n_docs': n, 'corpus_bytes': n_bytes, 'corpus_fingerprint': fp,
            'kb': ('advanced_scrapper_amd/synth_kb.py synthetic_kb(2300, seed)' if args.config == 4
                   else 'tests/golden/kb_processed.json.gz'), 'config': args.config, 'total_records': int(cnt.sum()),
            'hits_digest': cd.total(dig), 'oracle_seconds': round(time.time() - t0, 1), 'procs': args.procs}
    with open(args.out + '.json', 'w') as fh:
        json.dump(meta, fh, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == '__main__':
    main()
