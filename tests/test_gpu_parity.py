"""GPU parity: libkwmatch (HIP, gfx950) vs the CPU oracle and the reference's golden outputs.

Bar: bit-exact — the same (doc, field, name) set with the same code-point
positions as the oracle, the same ticker_matches dicts as the reference, and
byte-identical per-ticker CSV files.
"""
import io
import os
import random

import numpy as np
import pandas as pd
import pytest
from dateutil import parser

from tests import oracle_pool

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def env(golden):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    processed = golden.kb_processed()
    ckb = compile_kb(processed)
    return {'processed': processed, 'ckb': ckb, 'm': GpuMatcher(ckb)}


def _field_str(v):
    return str(v) if v else ""


def _golden_rows(golden):
    frame = golden.articles_frame()
    texts = [_field_str(v) for v in frame['article_text'].tolist()]
    titles = [_field_str(v) for v in frame['title'].tolist()]
    dates = [parser.parse(str(v)) if pd.notna(v) else None for v in frame['date_time'].tolist()]
    return texts, titles, dates


def _gpu_maps(m, texts, titles):
    from advanced_scrapper_amd.matcher import group_hits
    hits = m.match_strings(texts, titles)
    g = group_hits(hits)
    names = m.ckb.names
    out = []
    for d in range(len(texts)):
        f = g.get(d, {})
        out.append(({names[p]: v for p, v in f.get(0, {}).items()}, {names[p]: v for p, v in f.get(1, {}).items()}))
    return out


def _compare(processed, texts, titles, got):
    want_t = oracle_pool.field_results(processed, texts)
    want_i = oracle_pool.field_results(processed, titles)
    bad = []
    for d in range(len(texts)):
        if got[d][0] != want_t[d] or got[d][1] != want_i[d]:
            bad.append((d, sorted(set(got[d][0].items()) ^ set((k, tuple(v)) for k, v in want_t[d].items()))
                        if False else None))
            if len(bad) < 4:
                gt, wt = got[d][0], want_t[d]
                gi, wi = got[d][1], want_i[d]
                diff_t = {k: (gt.get(k), wt.get(k)) for k in set(gt) | set(wt) if gt.get(k) != wt.get(k)}
                diff_i = {k: (gi.get(k), wi.get(k)) for k in set(gi) | set(wi) if gi.get(k) != wi.get(k)}
                print(f"doc {d}: text diff {diff_t} title diff {diff_i}")
    return [b[0] for b in bad]


def test_golden_pattern_level(env, golden):
    texts, titles, _dates = _golden_rows(golden)
    got = _gpu_maps(env['m'], texts, titles)
    bad = _compare(env['processed'], texts, titles, got)
    assert not bad, f"GPU differs from the oracle on docs {bad[:20]}"


def test_golden_ticker_level(env, golden):
    from advanced_scrapper_amd.matcher import assemble_ticker_matches, group_hits
    texts, titles, dates = _golden_rows(golden)
    m = env['m']
    g = group_hits(m.match_strings(texts, titles))
    want = golden.matches()
    for d in range(len(texts)):
        got = assemble_ticker_matches(m.ckb, g.get(d, {}), dates[d])
        assert got == want[d], d
        assert list(got) == list(want[d]), d
        for t in got:
            assert list(got[t]['text']) == list(want[d][t]['text']), (d, t)
            assert list(got[t]['title']) == list(want[d][t]['title']), (d, t)


@pytest.mark.parametrize('native_cells', [True, False])
def test_dropin_process_chunk_csv_bytes(env, golden, tmp_path, monkeypatch, native_cells):
    """The drop-in driver writes byte-identical per-ticker CSVs (after the sort), with the JSON cells from
    libkwrows (checked to be the path taken) and with the Python assembly it falls back to."""
    from advanced_scrapper_amd import match_keywords as mk
    monkeypatch.chdir(tmp_path)
    native = mk.assemble_json_rows
    calls = []

    def cells(ckb, hits, dates):
        out = native(ckb, hits, dates) if native_cells else None
        calls.append(out is not None)
        return out
    monkeypatch.setattr(mk, 'assemble_json_rows', cells)
    os.makedirs('yahoo_ticker_matched_articles')
    processed = env['processed']
    for chunk in pd.read_csv(io.BytesIO(golden.articles_csv_bytes()), chunksize=golden.chunksize()):
        mk.process_chunk('yahoo', chunk, processed)
    for fn in os.listdir('yahoo_ticker_matched_articles'):
        mk.sort_matched_csv(f'yahoo_ticker_matched_articles/{fn}')
    want = golden.outputs()
    got = {fn: open(os.path.join('yahoo_ticker_matched_articles', fn), 'rb').read()
           for fn in os.listdir('yahoo_ticker_matched_articles')}
    assert sorted(got) == sorted(want)
    for fn in want:
        assert got[fn] == want[fn], fn
    assert calls and all(c == native_cells for c in calls)


@pytest.mark.parametrize('seed', [7, 11])
def test_random_corpus_vs_oracle(env, seed):
    from advanced_scrapper_amd import synth
    names, kinds = synth.injectable_names(env['ckb'])
    c = synth.generate(400, names, kinds, seed=seed, doc_base=seed * 1000)
    texts, titles = c.texts(), c.titles()
    got = _gpu_maps(env['m'], texts, titles)
    bad = _compare(env['processed'], texts, titles, got)
    assert not bad, f"seed {seed}: GPU differs from the oracle on docs {bad[:20]}"


def _adversarial_strings(ckb):
    rng = random.Random(5)
    fz = [n for n, c in zip(ckb.names, ckb.classes) if c == 'F' and n]
    up = [n for n, c in zip(ckb.names, ckb.classes) if c == 'U']
    texts, titles = [], []
    # empty fields, names as whole fields, names with one edit, glued uppercase names
    texts += ['', 'nan', 'a', 'é', '\n', '中文']
    titles += ['', '', 'nan', 'x', '', 'é']
    for n in rng.sample(fz, 60):
        texts.append(n)
        titles.append(n[1:] if len(n) > 1 else n)
        k = rng.randrange(len(n))
        texts.append(n[:k] + n[k + 1:])
        titles.append(n[:k] + 'x' + n[k:])
        texts.append('é ' * 40 + n[:k] + n[k + 1:] + ' ’' * 30)
        titles.append(n + ' ' + n)
    for n in rng.sample(up, 40):
        for glue in ('x', '_', '7', 'é', 'É', '中', '.', ' ', '+', '’'):
            texts.append(f"{glue}{n}{glue} {n}{glue}{n} {glue}{n}")
            titles.append(n + glue)
    long_na = ' '.join(rng.choice(fz) + rng.choice([' ', 'é ', '—', '\n']) for _ in range(400))
    texts.append(long_na)
    titles.append(long_na[:63])
    return texts, titles


def test_adversarial_strings_vs_oracle(env):
    texts, titles = _adversarial_strings(env['ckb'])
    got = _gpu_maps(env['m'], texts, titles)
    bad = _compare(env['processed'], texts, titles, got)
    assert not bad, f"GPU differs from the oracle on adversarial docs {bad[:20]}"


def test_batch_invariance_and_determinism(env):
    """Results of a doc do not depend on its batch or on the run (size-independent property)."""
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.matcher import group_hits
    names, kinds = synth.injectable_names(env['ckb'])
    c = synth.generate(3000, names, kinds, seed=99)
    m = env['m']
    d_arena, d_off = m.upload(c.arena, c.off)
    m.scan(d_arena, d_off, c.n_docs)
    full = np.sort(m.fetch(), order=['doc', 'field', 'pattern', 'pos'])
    m.scan(d_arena, d_off, c.n_docs)
    again = np.sort(m.fetch(), order=['doc', 'field', 'pattern', 'pos'])
    assert np.array_equal(full, again)
    half = c.n_docs // 2
    c2 = synth.generate(c.n_docs - half, names, kinds, seed=99, doc_base=half)
    a2, o2 = m.upload(c2.arena, c2.off)
    m.scan(a2, o2, c2.n_docs)
    tail = m.fetch()
    tail['doc'] += half
    tail = np.sort(tail, order=['doc', 'field', 'pattern', 'pos'])
    assert np.array_equal(full[full['doc'] >= half], tail)


_WILD_NAMES = ['x.yz.free', 'C.H. Robinson Worldwide', 'U.S. Smokeless Tobacco', '.zappos', 'ab.ab.ab',
               'é.éé.Zürich', 'E. I. du Pont de Nemours', 'Disney+ Hotstar', 'q..q..q..qq', 'Ab.c']


def test_wildcard_regex_names_vs_oracle():
    """'.'-wildcard names anchored in any literal run: positions, overlaps, edges, non-ASCII."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    processed = {'TK': {'name': {n: (None, None) for n in _WILD_NAMES}}}
    m = GpuMatcher(compile_kb(processed))
    rng = random.Random(17)
    subs = ['.', 'X', ' ', 'é', '中', '-', '\n']
    texts, titles = [], []
    for n in _WILD_NAMES:
        for _ in range(6):
            w = ''.join(rng.choice(subs) if ch == '.' else ch for ch in n)
            k = rng.randrange(len(n))
            texts.append(rng.choice(['', 'é', 'lorem ']) + w + w + ' ' + w[1:] + n[:k] + n[k + 1:] + w)
            titles.append(w + rng.choice(['', ' tail', 'é']))
    texts += ['ab.ab.ab.ab.ab', 'abXabXabXabXabXab', 'ab\nab.ab', 'q..q..q..qqq..q..q..qq', '.zappos' * 5]
    titles += ['ab.ab.ab', 'ab.ab.a', '', 'q..q..q..qq', 'zappos']
    got = _gpu_maps(m, texts, titles)
    bad = _compare(processed, texts, titles, got)
    assert not bad, f"GPU differs from the oracle on wildcard docs {bad[:20]}"


def test_regex_queue_overflow_rescans(monkeypatch):
    """A resolve wave whose regex-position queue overflows makes the host grow it and scan again."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    monkeypatch.setenv('KW_TEST_RX_CAP', '1')
    processed = {'TK': {'name': {n: (None, None) for n in _WILD_NAMES}}}
    m = GpuMatcher(compile_kb(processed))
    texts = [' '.join(_WILD_NAMES) + ' x' * k for k in range(40)]
    titles = [_WILD_NAMES[k % len(_WILD_NAMES)] for k in range(40)]
    got = _gpu_maps(m, texts, titles)
    bad = _compare(processed, texts, titles, got)
    assert not bad, f"GPU differs from the oracle after the regex-queue rescan on docs {bad[:20]}"
    assert m.stats()['regex_searches'] > 40


def _many_item_docs(ckb):
    """Fields around the fast path's item capacities (text 512, title 64: the epilogue kernel's LDS; beyond
    them the big-document epilogue up to 4096 / 512; 64 items of one name: the generic kernel)."""
    rng = random.Random(23)
    fz = [n for n, c in zip(ckb.names, ckb.classes) if c == 'F' and n and len(n) >= 4]
    up = [n for n, c in zip(ckb.names, ckb.classes) if c == 'U']
    texts, titles = [], []
    for na in ('', ' é'):
        one = rng.choice(up)
        for reps in (63, 64, 65, 80, 200):                 # one name: the > 64-items-per-name deferral
            texts.append(' '.join([one] * reps) + na)
            titles.append('t')
        for k in (60, 130, 300, 511, 520, 700, 1500):      # many names: below / above the text capacity
            texts.append(' , '.join(rng.choice(fz + up) for _ in range(k)) + na)
            titles.append(' '.join(rng.choice(up) for _ in range(k // 8)) + na)   # title capacity 64
        texts.append(' '.join(rng.choice(up) for _ in range(100)) + na)
        titles.append(' '.join(rng.choice(up) for _ in range(70)) + na)
    return texts, titles


def test_item_capacity_boundaries_vs_oracle(env):
    texts, titles = _many_item_docs(env['ckb'])
    got = _gpu_maps(env['m'], texts, titles)
    bad = _compare(env['processed'], texts, titles, got)
    assert not bad, f"GPU differs from the oracle on many-item docs {bad[:20]}"
    st = env['m'].stats()
    assert st['big_docs'] > 0          # the > 512-item all-ASCII texts took the big-document epilogue
    assert st['deferred_docs'] > 0     # > 64 items of one name: the generic kernel


def _nonascii_near_names(ckb):
    """Non-ASCII text fields (> 256 bytes) with near-miss fuzzy names and non-ASCII characters at every
    distance from them: inside the window family, just outside, at the field edges, plus regex-class
    names and uppercase names (code point positions after multi-byte characters)."""
    rng = random.Random(31)
    fz = [n for n, c in zip(ckb.names, ckb.classes) if c == 'F' and len(n) >= 11]
    up = [n for n, c in zip(ckb.names, ckb.classes) if c == 'U']
    words = ['market', 'shares', 'rose', 'the', 'company', 'said', 'on', 'Monday', 'analysts', 'quarter']
    na_chars = ['é', '’', '—', '中', '€', 'ß', '😀']
    texts, titles = [], []
    for i in range(160):
        n = rng.choice(fz)
        k = rng.randrange(len(n))
        near = n[:k] + n[k + 1:] if i % 3 else n[:k] + rng.choice('xyz') + n[k:]
        pre = ' '.join(rng.choice(words) for _ in range(rng.randrange(0, 60)))
        post = ' '.join(rng.choice(words) for _ in range(rng.randrange(0, 60)))
        gap = rng.choice([0, 1, 2, 3, 5, 8, 13, 40])
        c = rng.choice(na_chars)
        parts = [pre, ' ' * gap if i % 2 else '', near, ' ' * gap, post]
        t = ' '.join(parts)
        pos = rng.choice(['before', 'after', 'inside', 'start', 'end', 'far'])
        if pos == 'before':
            t = t.replace(near, c + ' ' * gap + near, 1)
        elif pos == 'after':
            t = t.replace(near, near + ' ' * gap + c, 1)
        elif pos == 'inside':
            j = rng.randrange(1, len(near))
            t = t.replace(near, near[:j] + c + near[j:], 1)
        elif pos == 'start':
            t = c + t
        elif pos == 'end':
            t = t + c
        else:
            t = c * 3 + ' ' + t + ' ' + c
        t += ' ' + ' '.join(rng.choice(up) for _ in range(3)) + ' ' + c
        while len(t.encode()) <= 300:
            t = rng.choice(words) + ' ' + t
        texts.append(t)
        titles.append(rng.choice(['', n, near, 'plain title']))
    return texts, titles


def test_nonascii_fields_in_scan_epilogue_vs_oracle(env):
    texts, titles = _nonascii_near_names(env['ckb'])
    got = _gpu_maps(env['m'], texts, titles)
    bad = _compare(env['processed'], texts, titles, got)
    assert not bad, f"GPU differs from the oracle on non-ASCII docs {bad[:20]}"


def test_nonascii_wildcard_and_regex_names_vs_oracle():
    """Regex-class names decided in non-ASCII fields go to the resolve kernel; literal ones stay."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    names = _WILD_NAMES + ['International Business Machines', 'Alphabet Incorporated Class', 'Nestlé Holdings AG']
    processed = {'TK': {'name': {n: (None, None) for n in names}}}
    m = GpuMatcher(compile_kb(processed))
    rng = random.Random(41)
    texts, titles = [], []
    for n in names:
        for c in ('é', '中', '’'):
            k = rng.randrange(len(n))
            filler = ' '.join(['lorem'] * 50)
            texts.append(f"{filler} {c} {n[:k] + n[k + 1:]} {filler} {n} {c}")
            texts.append(f"{c}{filler} {n[:k] + n[k + 1:]}{c} {filler}")
            titles += [n, c]
    got = _gpu_maps(m, texts, titles)
    bad = _compare(processed, texts, titles, got)
    assert not bad, f"GPU differs from the oracle on non-ASCII wildcard docs {bad[:20]}"


def _transcode_docs(ckb):
    """Documents built around the KB's non-ASCII fuzzy names, for the epilogue's transcoded view: exact
    occurrences, one-edit near misses (ASCII edits and the non-ASCII code point itself), edge windows (the
    name cut at the field start / end), short non-ASCII titles (the name, a part, a one-deletion variant, a
    <= 10 code point substring) and non-ASCII characters without markers sprinkled around them."""
    rng = random.Random(53)
    na = [n for n, c in zip(ckb.names, ckb.classes) if c == 'F' and any(ord(ch) > 127 for ch in n)]
    assert na
    words = ['market', 'shares', 'rose', 'the', 'company', 'said', 'on', 'Monday', 'analysts', 'quarter']
    other = ['中', '😀', 'Ω', 'ж', '€', '—', 'ß']
    texts, titles = [], []
    for i in range(240):
        n = na[i % len(na)]
        k = rng.randrange(len(n))
        edit = rng.choice(['exact', 'del', 'ins', 'del_na', 'swap_na'])
        v = n
        if edit == 'del':
            v = n[:k] + n[k + 1:]
        elif edit == 'ins':
            v = n[:k] + rng.choice('xyz') + n[k:]
        elif edit == 'del_na':
            v = ''.join(ch for ch in n if ord(ch) < 128)
        elif edit == 'swap_na':
            v = ''.join(rng.choice(other) if ord(ch) > 127 else ch for ch in n)
        filler = lambda: ' '.join(rng.choice(words + other) for _ in range(rng.randrange(5, 60)))
        shape = rng.choice(['mid', 'start', 'end', 'both'])
        if shape == 'mid':
            t = f"{filler()} {v} {filler()}"
        elif shape == 'start':
            t = f"{v[rng.randrange(1, 3):]} {filler()}"
        elif shape == 'end':
            t = f"{filler()} {v[:-rng.randrange(1, 3)]}"
        else:
            t = f"{v} {filler()} {v}"
        while len(t.encode()) <= 300:
            t = rng.choice(words) + ' ' + t
        texts.append(t)
        j = rng.randrange(len(n))
        titles.append(rng.choice([n, v, n[:j] + n[j + 1:], n[max(0, j - 6):j + 4], f"{n} {rng.choice(other)}",
                                  f"{rng.choice(other)} news", 'plain title']))
    return texts, titles


@pytest.mark.parametrize('mode', ['view', 'no_markers', 'no_room'])
def test_transcoded_view_vs_oracle(golden, monkeypatch, mode):
    """Non-ASCII documents on the epilogue's transcoded view (one byte per code point; the fuzzy names'
    non-ASCII code points as markers), and on the resolve kernel when the view cannot take them: names
    without markers (KW_TEST_TX_MARKERS=0: every non-ASCII name is PI_TXUNSAFE) or no room in the view."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import _native
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    if mode == 'no_markers':
        monkeypatch.setenv('KW_TEST_TX_MARKERS', '0')
    elif mode == 'no_room':
        monkeypatch.setenv('KW_TEST_TX_CAP', '16')
    processed = golden.kb_processed()
    m = GpuMatcher(compile_kb(processed))
    texts, titles = _transcode_docs(m.ckb)
    got = _gpu_maps(m, texts, titles)
    routes = m.doc_routes(len(texts))
    bad = _compare(processed, texts, titles, got)
    assert not bad, f"{mode}: GPU differs from the oracle on transcoded-view docs {bad[:20]}"
    n_tx = int((routes == _native.KW_ROUTE_TRANSCODE).sum())
    n_res = int((routes == _native.KW_ROUTE_RESOLVE).sum())
    if mode == 'view':
        assert n_tx > len(texts) // 2, (n_tx, n_res)
    elif mode == 'no_room':
        assert n_tx == 0 and n_res > 0, (n_tx, n_res)
    else:
        assert n_res > 0, (n_tx, n_res)


@pytest.mark.parametrize('case', ['invalid_regex', 'bad_date', 'int_dates'])
def test_dropin_error_paths_gpu(golden, tmp_path, monkeypatch, case):
    """process_chunk on the GPU writes exactly the rows the reference wrote before raising, and raises the
    same exception (tests/golden/make_error_golden.py ran the reference on these chunks)."""
    import time
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import match_keywords as mk
    monkeypatch.setenv('TZ', 'UTC')
    time.tzset()
    g = golden.error_cases()
    c = g['cases'][case]
    processed = golden.processed_from(g['kb_processed'])
    monkeypatch.chdir(tmp_path)
    os.makedirs('yahoo_ticker_matched_articles')
    raised = None
    try:
        for chunk in pd.read_csv(io.StringIO(c['articles_csv']), chunksize=g['chunksize']):
            mk.process_chunk('yahoo', chunk, processed)
    except Exception as exc:   # noqa: BLE001
        raised = type(exc).__name__
    assert raised == c['exception']
    got = {fn: open(os.path.join('yahoo_ticker_matched_articles', fn), encoding='utf-8').read()
           for fn in os.listdir('yahoo_ticker_matched_articles')}
    assert got == c['files']


@pytest.mark.parametrize('case', ['items_over_16384', 'non_ascii_over_65536_cps'])
def test_capacity_limits_grow_and_match_oracle(golden, case):
    """Fields past the generic kernel's initial buffers (more than 16 384 anchor occurrences in one field; a
    non-ASCII field of more than 65 536 code points) grow the buffers and rescan instead of failing, and give
    the oracle's result (a small KB keeps the oracle fast)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher, group_hits
    from oracle import kwmatch_oracle as orc
    processed = golden.processed_from(golden.error_cases()['kb_processed'])
    processed = {t: {a: {n: p for n, p in names.items() if n != 'Notepad++'} for a, names in attrs.items()}
                 for t, attrs in processed.items()}
    if case == 'items_over_16384':
        text = 'ACME Roadrunner Holdings ' * 9000 + 'Acme Rocket Skates.'
    else:
        text = 'é' * 70000 + ' ACME and Birdseed Deluxe; ' + 'ü' * 1000 + ' Wile E. Coyote'
    texts, titles = [text, 'RRN short', text[:5000]], ['ACME title', text[-3000:], 'nan']
    m = GpuMatcher(compile_kb(processed))
    g = group_hits(m.match_strings(texts, titles))
    st = m.stats()
    assert st['deferred_docs'] >= 1
    o = orc.Oracle(processed)
    for d in range(len(texts)):
        for f, s in ((0, texts[d]), (1, titles[d])):
            have = {m.ckb.names[p]: v for p, v in g.get(d, {}).get(f, {}).items()}
            assert have == o.field_results(s), (case, d, f)


def test_field_over_8mib_is_a_stated_limit():
    """A field beyond 8 MiB is the one capacity the device path does not take (23-bit item positions):
    kw_scan reports it by name instead of returning a wrong result."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import _native
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    processed = {'ACM': {'aliases': {'ACME': (None, None)}}}
    m = GpuMatcher(compile_kb(processed))
    with pytest.raises(_native.KwError, match='longer than 8388607 bytes'):
        m.match_strings(['x' * (9 << 20)], ['t'])


def test_fuzzy_name_over_64_code_points_is_rejected_with_the_reason():
    """Fuzzy names over 64 code points: rapidfuzz scores such needles with a heuristic this build does not
    restate, so kw_compile refuses the KB and says why, naming the name."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd import _native
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher
    long_name = 'Acme Consolidated Holdings of North American Widget Manufacturers Inc'   # 69 code points
    processed = {'ACM': {'aliases': {'ACME': (None, None), long_name: (None, None)}}}
    with pytest.raises(_native.KwError, match='matching-blocks heuristic') as ei:
        GpuMatcher(compile_kb(processed))
    assert long_name in str(ei.value)
