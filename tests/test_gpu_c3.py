"""Config 3's workload on one GPU: all 10M synthetic articles of the bench generator
(csrc/synth.c, bench.py's seed; documents 0..9 999 999 = the union of every rank's
shard under ``bench.py --gpus N``) against the reference KB, bit-exact.

* one kw_scan over the whole 10M-document arena (~22.9 GB resident in HBM);
* documents 0..999 999: per-document digests and counts equal the CPU oracle's
  (tests/golden/c2_digests.npz); documents 1M..10M: every 1000-document block's
  digest and count equals the oracle's (tests/golden/c3_blocks.npz, made in the
  build container by ``make_c2_digests.py --lo 1000000 --docs 10000000
  --blocks c3_blocks``).  A differing block is re-run through the oracle here
  to name its first differing documents and their fields;
* the one-shot scan equals the same documents scanned as ten 1M-document
  scans (config 3's contiguous shards at N = 10), document by document.

Reference: match_keywords.py:148-192 per article, :230-238 over the whole CSV.
"""
import json
import os
import time

import numpy as np
import pytest

from tests import oracle_pool

pytestmark = pytest.mark.gpu

SEED = 20250905
N_DOCS = 10_000_000
BLOCK = 1000
SLICE = 1_000_000


def _log(msg):
    print(f'[c3 {time.strftime("%H:%M:%S")}] {msg}', flush=True)


def _per_doc(hits, n, base=0):
    from advanced_scrapper_amd.matcher import records_from_tensor
    from tests import corpus_digest as cd
    return cd.per_doc(records_from_tensor(hits), n, base)


@pytest.fixture(scope='module')
def c3_scan(golden):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher, background_sample
    processed = golden.kb_processed()
    ckb = compile_kb(processed)
    names, kinds = synth.injectable_names(ckb)
    _log('generating 10M documents')
    corpus = synth.generate(N_DOCS, names, kinds, seed=SEED, doc_base=0)
    bg = synth.generate(2000, names, kinds, seed=SEED + 7777, doc_base=0)
    m = GpuMatcher(ckb, 0, background_sample(bg.texts() + bg.titles()))
    _log(f'uploading {corpus.n_bytes / 1e9:.2f} GB')
    d_arena, d_off = m.upload(corpus.arena, corpus.off)
    _log('scanning')
    m.scan(d_arena, d_off, N_DOCS)
    hits = m.hits_device()
    torch.cuda.synchronize()
    _log(f'{hits.shape[0]} records; digests')
    dig, cnt = _per_doc(hits, N_DOCS)
    st = m.stats()
    del hits
    _log('done')
    yield {'processed': processed, 'ckb': ckb, 'corpus': corpus, 'm': m, 'd_arena': d_arena, 'd_off': d_off,
           'dig': dig, 'cnt': cnt, 'stats': st}
    m.close()
    del d_arena, d_off
    torch.cuda.empty_cache()


def _explain(b, docs):
    """Print the oracle's and the GPU's results of up to three documents."""
    from advanced_scrapper_amd.matcher import group_hits, records_from_tensor
    corpus, m = b['corpus'], b['m']
    names = b['ckb'].names
    for d in docs[:3]:
        m.scan(b['d_arena'], b['d_off'][2 * d:], 1)
        g = group_hits(records_from_tensor(m.hits_device()))
        want = oracle_pool.field_results(b['processed'], [corpus.text(d), corpus.title(d)], 2)
        for f in (0, 1):
            got = {names[p]: v for p, v in g.get(0, {}).get(f, {}).items()}
            w = want[f]
            print('doc', d, 'field', f, {n: (got.get(n), w.get(n)) for n in set(got) | set(w) if got.get(n) != w.get(n)})


def test_c3_ten_million_vs_oracle(c3_scan, golden):
    """Every document of config 3's 10M-article workload: per-document digests for 0..999 999, per-1000-document
    block digests for 1M..10M, against the CPU oracle."""
    from tests import corpus_digest as cd
    from tests.golden_data import HERE
    b = c3_scan
    dig, cnt = b['dig'], b['cnt']
    meta = json.load(open(os.path.join(HERE, 'c3_blocks.json')))
    z = np.load(os.path.join(HERE, 'c3_blocks.npz'))
    assert meta['n_docs'] == N_DOCS and meta['seed'] == SEED and meta['docs_per_block'] == BLOCK
    assert meta['all_blocks'], 'c3_blocks.npz does not pin every block'
    from advanced_scrapper_amd.synth import Corpus
    c = b['corpus']
    for k in (0, N_DOCS // SLICE - 1):              # the generator still makes the pinned documents
        lo = k * SLICE
        sub = Corpus(c.arena, c.off[2 * lo:2 * (lo + SLICE) + 1], c.flags[lo:lo + SLICE], lo, c.seed)
        assert cd.corpus_fingerprint(sub) == meta['slice_fingerprints'][k], f'slice {k} differs from the pinned corpus'
    # documents 0..999 999: per document
    c2 = np.load(os.path.join(HERE, 'c2_digests.npz'))
    bad = np.flatnonzero((dig[:SLICE] != c2['digest']) | (cnt[:SLICE] != c2['count'].astype(np.int64)))
    if len(bad):
        _explain(b, bad.tolist())
    assert not len(bad), f'{len(bad)} of the first 1M documents differ from the oracle; first: {bad[:20].tolist()}'
    # every 1000-document block
    with np.errstate(over='ignore'):
        bdig = dig.reshape(-1, BLOCK).sum(axis=1, dtype=np.uint64)
    bcnt = cnt.reshape(-1, BLOCK).sum(axis=1)
    blk = z['block'].astype(np.int64)
    assert np.array_equal(blk, np.arange(N_DOCS // BLOCK))
    badb = np.flatnonzero((bdig[blk] != z['digest']) | (bcnt[blk] != z['count'].astype(np.int64)))
    if len(badb):
        # name the differing documents of the first differing block: the oracle on that block, here
        lo = int(blk[badb[0]]) * BLOCK
        c = b['corpus']
        want = oracle_pool.field_results(b['processed'], [s for d in range(lo, lo + BLOCK)
                                                          for s in (c.text(d), c.title(d))])
        pid = {n: i for i, n in enumerate(b['ckb'].names)}
        rows = []
        for i in range(BLOCK):
            rows += cd.oracle_records(lo + i, [want[2 * i], want[2 * i + 1]], pid)
        a = np.asarray(rows, dtype=np.uint32).reshape(-1, 4).view(
            np.dtype([('doc', '<u4'), ('pattern', '<u4'), ('pos', '<u4'), ('field', '<u4')])).reshape(-1)
        wd, wc = cd.per_doc(a, BLOCK, lo)
        docs = (lo + np.flatnonzero((wd != dig[lo:lo + BLOCK]) | (wc != cnt[lo:lo + BLOCK]))).tolist()
        print('block', lo // BLOCK, 'differing documents', docs[:20])
        _explain(b, docs)
    assert not len(badb), f'{len(badb)} of {len(blk)} blocks differ from the oracle; first: {blk[badb[:20]].tolist()}'
    assert int(cnt.sum()) == int(c2['count'].astype(np.int64).sum()) + int(z['count'][SLICE // BLOCK:].astype(np.int64).sum())
    assert int(cnt.sum()) == meta['total_records']
    assert cd.total(dig) == meta['hits_digest']
    _log(f'10M documents pinned: {int(cnt.sum())} records, digest {cd.total(dig)}, stats {b["stats"]}')


def test_c3_one_shot_equals_ten_shards(c3_scan):
    """The 10M one-shot scan equals ten contiguous 1M-document scans (config 3's shards), per document."""
    from advanced_scrapper_amd.matcher import records_from_tensor
    from tests import corpus_digest as cd
    b = c3_scan
    m = b['m']
    for k in range(N_DOCS // SLICE):
        lo = k * SLICE
        m.scan(b['d_arena'], b['d_off'][2 * lo:], SLICE)
        rec = records_from_tensor(m.hits_device())     # shard-local document ids: rebase to global ones
        rec['doc'] += np.uint32(lo)
        d, c = cd.per_doc(rec, SLICE, lo)
        bad = np.flatnonzero((d != b['dig'][lo:lo + SLICE]) | (c != b['cnt'][lo:lo + SLICE]))
        assert not len(bad), f'shard {k}: {len(bad)} documents differ from the one-shot scan; first {(lo + bad[:10]).tolist()}'
