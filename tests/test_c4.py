"""Config 4: the ~50k-pattern synthetic knowledge base (advanced_scrapper_amd/synth_kb.py).

CPU tests pin the generators (digests recorded in tests/golden/c4_golden.json.gz)
and re-derive part of the fixture with the oracle; the GPU tests match the
whole fixture bit-exactly and run the oracle live on a second seeded corpus.
"""
import gzip
import json
import os
import random

import pytest

from tests import oracle_pool

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _fixture():
    with gzip.open(os.path.join(HERE, 'c4_golden.json.gz'), 'rt', encoding='utf-8') as fh:
        return json.load(fh)


def _inputs():
    import importlib.util
    spec = importlib.util.spec_from_file_location('make_c4_golden', os.path.join(HERE, 'make_c4_golden.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope='module')
def c4():
    mod = _inputs()
    kb, ckb, corpus = mod.inputs()
    return {'mod': mod, 'kb': kb, 'ckb': ckb, 'corpus': corpus, 'fx': _fixture()}


def _as_fixture(res):
    return sorted([k, list(v)] for k, v in res.items())


def test_c4_kb_shape(c4):
    """~50k active patterns, every name <= 64 code points, every class the reference has."""
    ckb = c4['ckb']
    assert 45_000 <= ckb.n_patterns <= 60_000
    assert max(len(n) for n in ckb.names) <= 64
    assert not any(ckb.invalid_regex)
    kb = c4['kb']
    from advanced_scrapper_amd.kb import classify_name
    classes = {classify_name(n) for t in kb.values() for a in t.values() for n in a}
    assert classes == {'U', 'F', 'X', 'S'}
    assert any(s or e for t in kb.values() for a in t.values() for (s, e) in a.values())
    assert any(any(ord(ch) > 127 for ch in n) for n in ckb.names)
    assert any('+' in n for n in ckb.names) and any('.' in n for n in ckb.names)


def test_c4_inputs_match_fixture(c4):
    """The seeded generators still produce the inputs the fixture was computed on."""
    d = c4['mod'].digests(c4['ckb'], c4['corpus'])
    fx = c4['fx']
    assert d['kb_names_sha256'] == fx['kb_names_sha256']
    assert d['arena_sha256'] == fx['arena_sha256']
    assert fx['n_patterns'] == c4['ckb'].n_patterns and fx['n_docs'] == c4['corpus'].n_docs


def test_c4_oracle_reproduces_fixture_sample(c4):
    """The oracle re-derives a sample of the committed fixture (titles of all docs, texts of a few)."""
    fx, corpus = c4['fx'], c4['corpus']
    titles = corpus.titles()
    got_i = oracle_pool.field_results(c4['kb'], titles, procs=min(8, os.cpu_count() or 1))
    for d in range(corpus.n_docs):
        assert _as_fixture(got_i[d]) == fx['docs'][d][1], d
    docs = [d for d in range(corpus.n_docs) if fx['docs'][d][0]][:4]
    got_t = oracle_pool.field_results(c4['kb'], [corpus.text(d) for d in docs], procs=4)
    for d, r in zip(docs, got_t):
        assert _as_fixture(r) == fx['docs'][d][0], d


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope='module')
def c4_gpu(c4):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.matcher import GpuMatcher
    return GpuMatcher(c4['ckb'])


def _gpu_fields(m, texts, titles):
    from advanced_scrapper_amd.matcher import group_hits
    g = group_hits(m.match_strings(texts, titles))
    names = m.ckb.names
    out = []
    for d in range(len(texts)):
        f = g.get(d, {})
        out.append(({names[p]: v for p, v in f.get(0, {}).items()}, {names[p]: v for p, v in f.get(1, {}).items()}))
    return out


@pytest.mark.gpu
def test_c4_gpu_matches_fixture(c4, c4_gpu):
    corpus, fx = c4['corpus'], c4['fx']
    got = _gpu_fields(c4_gpu, corpus.texts(), corpus.titles())
    bad = [d for d in range(corpus.n_docs)
           if _as_fixture(got[d][0]) != fx['docs'][d][0] or _as_fixture(got[d][1]) != fx['docs'][d][1]]
    for d in bad[:3]:
        print(d, _as_fixture(got[d][0]), fx['docs'][d][0], _as_fixture(got[d][1]), fx['docs'][d][1])
    assert not bad, f"config-4 GPU results differ from the fixture on docs {bad[:20]}"


@pytest.mark.gpu
def test_c4_gpu_vs_live_oracle(c4, c4_gpu):
    """A second seeded corpus plus near-miss / glued edits of KB names, checked against the oracle live."""
    from advanced_scrapper_amd import synth
    ckb = c4['ckb']
    names, kinds = synth.injectable_names(ckb)
    c = synth.generate(24, names, kinds, seed=77, doc_base=5000)
    texts, titles = c.texts(), c.titles()
    rng = random.Random(3)
    fz = [n for n, k in zip(ckb.names, ckb.classes) if k == 'F' and len(n) > 2]
    up = [n for n, k in zip(ckb.names, ckb.classes) if k == 'U']
    for _ in range(24):
        a, b = rng.choice(fz), rng.choice(fz)
        k = rng.randrange(len(a))
        texts.append(f"{a[:k]}{a[k + 1:]} and {b}x {rng.choice(up)}é{rng.choice(up)} {a}")
        titles.append(b[:-1])
    got = _gpu_fields(c4_gpu, texts, titles)
    want_t = oracle_pool.field_results(c4['kb'], texts)
    want_i = oracle_pool.field_results(c4['kb'], titles)
    bad = [d for d in range(len(texts)) if got[d][0] != want_t[d] or got[d][1] != want_i[d]]
    for d in bad[:3]:
        print(d, got[d], want_t[d], want_i[d])
    assert not bad, f"config-4 GPU results differ from the oracle on docs {bad[:20]}"


@pytest.mark.gpu
def test_c4_whole_corpus_vs_oracle_digests():
    """EVERY document of bench.py --workload kb50k's 1M-article corpus (config 4: the ~52k-name synthetic KB):
    the GPU's per-document record digest equals the CPU oracle's (tests/golden/c4_digests.npz, made in the
    build container by tests/golden/make_c2_digests.py --config 4), and so do the record count and the
    bench line's hits_digest."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    import bench
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher, background_sample, records_from_tensor
    from advanced_scrapper_amd.synth_kb import synthetic_kb
    from tests import corpus_digest as cd
    meta = json.load(open(os.path.join(HERE, 'c4_digests.json')))
    z = np.load(os.path.join(HERE, 'c4_digests.npz'))
    n, seed = meta['n_docs'], meta['seed']
    processed = synthetic_kb(2300, seed)
    ckb = compile_kb(processed)
    names, kinds = synth.injectable_names(ckb)
    corpus = synth.generate(n, names, kinds, seed=seed, doc_base=0)
    assert cd.corpus_fingerprint(corpus) == meta['corpus_fingerprint'], 'the generator no longer makes the pinned corpus'
    bg = synth.generate(2000, names, kinds, seed=seed + 7777, doc_base=0)
    m = GpuMatcher(ckb, 0, background_sample(bg.texts() + bg.titles()))
    d_arena, d_off = m.upload(corpus.arena, corpus.off)
    m.scan(d_arena, d_off, n)
    hits = m.hits_device().clone()
    rec = records_from_tensor(hits)
    dig, cnt = cd.per_doc(rec, n)
    bad = np.flatnonzero((dig != z['digest']) | (cnt != z['count'].astype(np.int64)))
    if len(bad):
        from advanced_scrapper_amd.matcher import group_hits
        g = group_hits(rec[np.isin(rec['doc'], bad[:3].astype(np.uint32))])
        want = oracle_pool.field_results(processed, [s for d in bad[:3].tolist()
                                                     for s in (corpus.text(d), corpus.title(d))], 3)
        for k, d in enumerate(bad[:3].tolist()):
            for f in (0, 1):
                got = {ckb.names[p]: v for p, v in g.get(d, {}).get(f, {}).items()}
                w = want[2 * k + f]
                print('doc', d, 'field', f, {x: (got.get(x), w.get(x)) for x in set(got) | set(w) if got.get(x) != w.get(x)})
    assert not len(bad), f'{len(bad)} of {n} documents differ from the oracle; first: {bad[:20].tolist()}'
    assert int(cnt.sum()) == meta['total_records']
    assert cd.total(dig) == meta['hits_digest'] == bench.hits_digest(hits)
    st = m.stats()
    assert st['big_docs'] > 1000 and st['deferred_item_caps'] == 0
    # the same corpus with no room in any epilogue workgroup's big-document queue (KW_TEST_BIGQ=0): every
    # all-ASCII big document takes the resolve kernel's big-document path instead (what a workgroup past its
    # 64 queued documents does at 10M), same records
    from advanced_scrapper_amd import _native
    import os as _os
    _os.environ['KW_TEST_BIGQ'] = '0'
    try:
        m.scan(d_arena, d_off, n)
        hits2 = m.hits_device()
        st2 = m.stats()
        routes = m.doc_routes(n)
    finally:
        del _os.environ['KW_TEST_BIGQ']
    dig2, cnt2 = cd.per_doc(records_from_tensor(hits2), n)
    bad2 = np.flatnonzero((dig2 != z['digest']) | (cnt2 != z['count'].astype(np.int64)))
    assert not len(bad2), f'KW_TEST_BIGQ=0: {len(bad2)} documents differ; first: {bad2[:20].tolist()}'
    # (big_docs counts both kernels' big documents)
    assert st2['deferred_item_caps'] == 0 and st2['deferred_docs'] == st['deferred_docs']
    assert st2['resolved_docs'] >= st['resolved_docs'] + st['big_docs'] // 2
    assert int((routes == _native.KW_ROUTE_RESOLVE).sum()) >= st2['resolved_docs'] - st['resolved_docs']
    m.close()


@pytest.mark.gpu
def test_c4_ten_million_vs_oracle():
    """Config 4 at its stated size: the ~52k-name KB against 10M articles in ONE kw_scan (~22.9 GB resident).
    Documents 0..999 999 per document against tests/golden/c4_digests.npz, and the strided 1000-document
    blocks beyond 1M that tests/golden/c4_blocks.npz pins (make_c2_digests.py --config 4 --strided 200
    --lo 1000000 --docs 10000000 --blocks c4_blocks, CPU oracle in the build container: 208 blocks, 2.3 % of
    the documents beyond 1M)."""
    import time
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher, background_sample, records_from_tensor
    from advanced_scrapper_amd.synth_kb import synthetic_kb
    from tests import corpus_digest as cd
    meta = json.load(open(os.path.join(HERE, 'c4_blocks.json')))
    z = np.load(os.path.join(HERE, 'c4_blocks.npz'))
    z1 = np.load(os.path.join(HERE, 'c4_digests.npz'))
    n, seed, blk = meta['n_docs'], meta['seed'], meta['docs_per_block']
    assert n == 10_000_000 and meta['config'] == 4
    processed = synthetic_kb(2300, seed)
    ckb = compile_kb(processed)
    names, kinds = synth.injectable_names(ckb)
    t0 = time.time()
    corpus = synth.generate(n, names, kinds, seed=seed, doc_base=0)
    bg = synth.generate(2000, names, kinds, seed=seed + 7777, doc_base=0)
    m = GpuMatcher(ckb, 0, background_sample(bg.texts() + bg.titles()))
    d_arena, d_off = m.upload(corpus.arena, corpus.off)
    m.scan(d_arena, d_off, n)
    hits = m.hits_device()
    print(f'c4 10M: {hits.shape[0]} records, {time.time() - t0:.1f} s, stats {m.stats()}', flush=True)
    dig, cnt = cd.per_doc(records_from_tensor(hits), n)
    del hits
    bad = np.flatnonzero((dig[:1_000_000] != z1['digest']) | (cnt[:1_000_000] != z1['count'].astype(np.int64)))
    assert not len(bad), f'{len(bad)} of the first 1M documents differ from the oracle; first: {bad[:20].tolist()}'
    with np.errstate(over='ignore'):
        bdig = dig.reshape(-1, blk).sum(axis=1, dtype=np.uint64)
    bcnt = cnt.reshape(-1, blk).sum(axis=1)
    sel = z['block'].astype(np.int64)
    beyond = sel[sel >= 1_000_000 // blk]
    assert len(beyond) >= 200
    badb = np.flatnonzero((bdig[sel] != z['digest']) | (bcnt[sel] != z['count'].astype(np.int64)))
    if len(badb):
        lo = int(sel[badb[0]]) * blk
        want = oracle_pool.field_results(processed, [s for d in range(lo, lo + blk)
                                                     for s in (corpus.text(d), corpus.title(d))])
        pid = {x: i for i, x in enumerate(ckb.names)}
        rows = []
        for i in range(blk):
            rows += cd.oracle_records(lo + i, [want[2 * i], want[2 * i + 1]], pid)
        a = np.asarray(rows, dtype=np.uint32).reshape(-1, 4).view(
            np.dtype([('doc', '<u4'), ('pattern', '<u4'), ('pos', '<u4'), ('field', '<u4')])).reshape(-1)
        wd, wc = cd.per_doc(a, blk, lo)
        print('block', lo // blk, 'differing documents',
              (lo + np.flatnonzero((wd != dig[lo:lo + blk]) | (wc != cnt[lo:lo + blk]))).tolist()[:20])
    assert not len(badb), f'{len(badb)} of {len(sel)} pinned blocks differ; first: {sel[badb[:10]].tolist()}'
    m.close()
