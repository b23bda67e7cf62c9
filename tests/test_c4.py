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
