"""CPU tests of the host side: KB loading, classification, regex atoms, assembly, CSV egress, C-ABI."""
import io
import os
import random
import re
import subprocess

import numpy as np
import pandas as pd
import pytest
from dateutil import parser

from advanced_scrapper_amd import kb
from advanced_scrapper_amd.kb import compile_kb


# ------------------------------------------------------------------ KB loading (a1-a3)
def test_kb_loader_matches_reference(golden, tmp_path):
    order = golden.materialize_kb(str(tmp_path / 'ticker'))
    got = kb.read_and_process_json_files(str(tmp_path / 'ticker'), _listdir=lambda _p: order)
    want = golden.kb_processed()
    assert list(got) == list(want)
    for t in want:
        assert list(got[t]) == list(want[t])
        for a in want[t]:
            assert list(got[t][a].items()) == list(want[t][a].items()), (t, a)


def test_kb_loader_error_paths(tmp_path, capsys):
    d = tmp_path / 'kb'
    d.mkdir()
    (d / 'A_info.json').write_text('[{"ticker": "AAA", "country": ["United States"], "aliases": ["Aaa Corp"]}]')
    (d / 'B_info.json').write_text('[{"ticker": "BBB"}, {"ticker": "CCC"}]')       # KeyError: skipped
    (d / 'C_info.json').write_bytes('[{"ticker": "DDD", "aliases": ["Ca\xe9"]}]'.encode('latin1'))  # not utf-8
    (d / 'notes.txt').write_text('ignored')
    got = kb.read_and_process_json_files(str(d), _listdir=lambda p: sorted(os.listdir(p)))
    assert list(got) == ['AAA', 'DDD']
    assert 'Aaa Corp' in got['AAA']['aliases']
    # the reference's own messages (match_keywords.py:104,119): the KeyError file, then the utf-8 retry
    out = capsys.readouterr().out.splitlines()
    assert out[-2] == "处理文件 B_info.json 时出错: 'country'"
    assert out[-1] == 'UTF-8解码失败，尝试其他编码读取文件: C_info.json'


def test_extract_time_periods_rules():
    p = kb.extract_time_periods([
        'Steve Jobs (Start: 1997-09-16T00:00:00Z) (End: 2011-08-24T00:00:00Z)',
        'Steve Jobs (Start: 1976-04-01T00:00:00Z) (End: 1985-09-17T00:00:00Z)',
        'Tim Cook (Start: http://www.wikidata.org/.well-known/genid/abc)',
        'Plain Name',
        'Weird (End: not a date)',
    ])
    assert list(p) == ['Steve Jobs', 'Tim Cook', 'Plain Name', 'Weird']
    assert p['Steve Jobs'][0].year == 1976 and p['Steve Jobs'][1].year == 1985   # last wins, first position
    assert p['Tim Cook'] == (None, None)
    assert p['Plain Name'] == (None, None)
    assert kb.extract_time_periods('Solo') == {'Solo': (None, None)}


def test_is_within_period():
    d = parser.parse
    assert not kb.is_within_period(None, None, None)
    assert kb.is_within_period(d('2000-01-01'), None, None)
    assert kb.is_within_period(d('2000-01-01'), d('2000-01-01'), d('2000-01-01'))
    assert not kb.is_within_period(d('1999-12-31'), d('2000-01-01'), None)
    assert kb.is_within_period(d('2000-01-01T05:00:00+05:00'), d('2000-01-01'), None)
    assert not kb.is_within_period(d('2000-01-01T05:00:00+05:01'), d('2000-01-01'), None)


def test_classes_of_the_golden_kb(golden):
    from collections import Counter
    names = {}
    for _t, attrs in golden.kb_processed().items():
        for _a, ns in attrs.items():
            for n in ns:
                names[n] = kb.classify_name(n)
    c = Counter(names.values())
    assert c == Counter({'F': 2209, 'U': 253, 'S': 127, 'X': 4})
    ckb = compile_kb(golden.kb_processed())
    assert ckb.n_patterns == 2462
    assert ckb.classes[:253] == ['U'] * 253
    lens = [len(n) for n in ckb.names[253:]]
    assert lens == sorted(lens, reverse=True)
    assert max(lens) <= 64


# ------------------------------------------------------------------ regex atoms
def _atoms_finditer(atoms, s):
    """Python mirror of the device matcher (kwmatch_kernels.hpp rx_match + rx_positions)."""
    def match_at(st):
        stack = []
        a, pos = 0, st
        while True:
            fail = False
            if a == len(atoms):
                return pos
            op, val, lo, hi = atoms[a]
            ok = lambda c: (c == chr(val)) if op == 0 else (c != '\n')
            if lo == 1 and hi == 1:
                if pos < len(s) and ok(s[pos]):
                    pos += 1
                    a += 1
                    continue
                fail = True
            else:
                k = 0
                while (hi < 0 or k < hi) and pos + k < len(s) and ok(s[pos + k]):
                    k += 1
                if k < lo:
                    fail = True
                else:
                    stack.append([a, pos, k])
                    pos += k
                    a += 1
                    continue
            if fail:
                while stack:
                    t = stack[-1]
                    if t[2] > atoms[t[0]][2]:
                        t[2] -= 1
                        pos = t[1] + t[2]
                        a = t[0] + 1
                        break
                    stack.pop()
                else:
                    return -1
    out, last = [], 0
    for st in range(len(s)):
        e = match_at(st)
        if e >= 0 and st >= last:
            out.append(st)
            last = e if e > st else st + 1
    return out


def test_regex_atoms_match_python_re(golden):
    rng = random.Random(3)
    names = [n for n in compile_kb(golden.kb_processed()).names if kb.regex_atoms(n) not in (None, 'invalid')]
    extra = ['ab+c', 'a.?b', 'x*yz', 'E*Trade', 'Guess?', 'a{2,3}b', '(foo)bar', 'C.+D']
    for name in names + extra:
        atoms = kb.regex_atoms(name)
        alphabet = list(set(name.replace('\\', ''))) + ['\n', 'y', 'Z']
        for _ in range(40):
            s = ''.join(rng.choice(alphabet) for _ in range(rng.randint(0, 30)))
            if rng.random() < 0.5:
                s = s[:5] + name.replace('(', '').replace(')', '') + s[5:]
            want = [m.start() for m in re.finditer(name, s)]
            assert _atoms_finditer(atoms, s) == want, (name, s)


def test_regex_atoms_dot_fast_path_and_parallel_compile():
    """The '.'-only fast path equals the sre_parse walk, and the parallel regex parse equals the serial one
    (config-4 KB: ~52k names)."""
    from advanced_scrapper_amd.synth_kb import synthetic_kb
    processed = synthetic_kb(600, 11)
    serial = compile_kb(processed, workers=1)
    dots = [n for n in serial.names if set(n) & kb._META == {'.'}]
    assert len(dots) > 100
    for name in dots + ['.', 'a.b', '..', 'é.ü']:
        assert kb.regex_atoms(name) == kb.regex_atoms_sre(name), name
    old = kb.PAR_MIN_REGEX
    kb.PAR_MIN_REGEX = 1
    try:
        par = compile_kb(processed, workers=2)
    finally:
        kb.PAR_MIN_REGEX = old
    assert par.names == serial.names and par.invalid_regex == serial.invalid_regex
    assert np.array_equal(par.rx_atoms, serial.rx_atoms) and np.array_equal(par.rx_off, serial.rx_off)


def test_regex_atoms_classification():
    assert kb.regex_atoms('Apple Inc') is None
    assert kb.regex_atoms('C++') == 'invalid'
    assert kb.regex_atoms('Disney+ Hotstar')[5] == (0, ord('y'), 1, -1)
    with pytest.raises(kb.UnsupportedPattern):
        kb.regex_atoms('[24]7.ai')
    with pytest.raises(kb.UnsupportedPattern):
        kb.regex_atoms('A|B')


# ------------------------------------------------------------------ assembly (a10) from oracle field results
def test_assembly_reproduces_reference_dicts(golden):
    """Host expansion of per-(field, name) results == the reference's ticker_matches."""
    from advanced_scrapper_amd.matcher import assemble_ticker_matches
    from tests import oracle_pool
    processed = golden.kb_processed()
    ckb = compile_kb(processed)
    pid = {n: i for i, n in enumerate(ckb.names)}
    frame = golden.articles_frame()
    texts = [str(v) if v else "" for v in frame['article_text'].tolist()]
    titles = [str(v) if v else "" for v in frame['title'].tolist()]
    dates = [parser.parse(str(v)) if pd.notna(v) else None for v in frame['date_time'].tolist()]
    ft = oracle_pool.field_results(processed, texts, procs=8)
    fi = oracle_pool.field_results(processed, titles, procs=8)
    want = golden.matches()
    for d in range(len(texts)):
        fields = {0: {pid[n]: v for n, v in ft[d].items()}, 1: {pid[n]: v for n, v in fi[d].items()}}
        got = assemble_ticker_matches(ckb, fields, dates[d])
        assert got == want[d], d
        assert list(got) == list(want[d])
        for t in got:
            assert list(got[t]['text']) == list(want[d][t]['text'])
            assert list(got[t]['title']) == list(want[d][t]['title'])


# ------------------------------------------------------------------ CSV egress (a11, a12)
def test_csv_egress_bytes(golden, tmp_path, monkeypatch):
    """Rows built from the golden matches and written/sorted by the drop-in == reference files."""
    from advanced_scrapper_amd import match_keywords as mk
    monkeypatch.chdir(tmp_path)
    os.makedirs('yahoo_ticker_matched_articles')
    want_m = golden.matches()
    start = 0
    for chunk in pd.read_csv(io.BytesIO(golden.articles_csv_bytes()), chunksize=golden.chunksize()):
        by_ticker = {}
        for i in range(len(chunk)):
            for ticker, matched in want_m[start + i].items():
                by_ticker.setdefault(ticker, []).append(mk._csv_row(matched, chunk.iloc[i]))
        for ticker, rows in by_ticker.items():
            mk._append_rows('yahoo', ticker, rows)
        start += len(chunk)
    for fn in os.listdir('yahoo_ticker_matched_articles'):
        mk.sort_matched_csv(f'yahoo_ticker_matched_articles/{fn}')
    want = golden.outputs()
    got = sorted(os.listdir('yahoo_ticker_matched_articles'))
    assert got == sorted(want)
    for fn in want:
        with open(os.path.join('yahoo_ticker_matched_articles', fn), 'rb') as fh:
            assert fh.read() == want[fn], fn


def test_csv_egress_chunk_rows_bytes(golden, tmp_path, monkeypatch):
    """The chunk-level egress (_chunk_rows: column lists, one date parse) == reference files after sort."""
    from dateutil import parser as dparser
    from advanced_scrapper_amd import match_keywords as mk
    monkeypatch.chdir(tmp_path)
    os.makedirs('yahoo_ticker_matched_articles')
    want_m = golden.matches()
    start = 0
    for chunk in pd.read_csv(io.BytesIO(golden.articles_csv_bytes()), chunksize=golden.chunksize()):
        results = want_m[start:start + len(chunk)]
        dates = [dparser.parse(str(v)) if pd.notna(v) else None for v in chunk['date_time'].tolist()]
        by_ticker, err = mk._chunk_rows(chunk, results, dates)
        assert err is None
        for ticker, rows in by_ticker.items():
            mk._append_rows('yahoo', ticker, rows)
        start += len(chunk)
    for fn in os.listdir('yahoo_ticker_matched_articles'):
        mk.sort_matched_csv(f'yahoo_ticker_matched_articles/{fn}')
    want = golden.outputs()
    assert sorted(os.listdir('yahoo_ticker_matched_articles')) == sorted(want)
    for fn in want:
        with open(os.path.join('yahoo_ticker_matched_articles', fn), 'rb') as fh:
            assert fh.read() == want[fn], fn


def test_egress_append_rows_equals_pandas_per_row(tmp_path):
    """egress.append_rows == one pd.DataFrame([row]).to_csv(mode='a') per row (match_keywords.py:145-146),
    byte for byte, over quotes, commas, CR/LF, empty strings, unicode, NaN/None, ints, and the cell types
    that take the pandas fallback (floats, bools)."""
    import numpy as np
    from advanced_scrapper_amd import egress
    cols = ('time_unix', 'date_time', 'text_matches', 'title', 'url')
    rng = np.random.default_rng(7)
    atoms = ['', 'a', 'x,y', 'say "hi"', 'line\nbreak', 'cr\rlf\r\n', 'cr\ronly', 'tab\t', '\x1c', ' lead', 'trail ', 'é中文', '"',
             float('nan'), None, 0, -17, np.int64(1700000000), 2 ** 70, 1.5, np.float64(2.25), True, 'NA']
    rows = []
    for _ in range(400):
        rows.append(tuple(atoms[int(rng.integers(len(atoms)))] for _ in cols))
    rows.append(tuple('' for _ in cols))
    got, want = str(tmp_path / 'got.csv'), str(tmp_path / 'want.csv')
    for k in range(0, len(rows), 37):       # several appends, header only on the first
        egress.append_rows(got, cols, rows[k:k + 37])
    for r in rows:
        pd.DataFrame([dict(zip(cols, r))]).to_csv(want, mode='a', index=False, header=not os.path.exists(want))
    assert open(got, 'rb').read() == open(want, 'rb').read()
    # a NUL cell: pandas' writer raises, and so does append_rows (the rows before it are written first)
    bad = ('a', 'b\0c', 'x', 'y', 'z')
    with pytest.raises(Exception) as want_exc:
        pd.DataFrame([dict(zip(cols, bad))]).to_csv(str(tmp_path / 'w2.csv'), index=False)
    with pytest.raises(type(want_exc.value)):
        egress.append_rows(str(tmp_path / 'g2.csv'), cols, [('1', '2', '3', '4', '5'), bad])
    assert open(str(tmp_path / 'g2.csv'), 'rb').read() == b'time_unix,date_time,text_matches,title,url\n1,2,3,4,5\n'


def test_parse_date_equals_dateutil():
    """dates.parse_date == dateutil.parser.parse on the dataset layout (random valid stamps) and on
    edge strings (invalid fields, leap days, other layouts), including raising the same exception type."""
    import numpy as np
    from dateutil import parser as dparser
    from advanced_scrapper_amd.dates import parse_date
    rng = np.random.default_rng(11)
    cases = []
    for _ in range(3000):
        y, mo, d = int(rng.integers(900, 2100)), int(rng.integers(0, 14)), int(rng.integers(0, 33))
        hh, mi, ss = int(rng.integers(0, 26)), int(rng.integers(0, 62)), int(rng.integers(0, 62))
        sep = ' ' if rng.random() < 0.8 else 'T'
        cases.append(f'{y:04d}-{mo:02d}-{d:02d}{sep}{hh:02d}:{mi:02d}:{ss:02d}')
    cases += ['2024-02-29 00:00:00', '2023-02-29 00:00:00', '1900-02-29 12:00:00', '2000-02-29 23:59:59',
              '2020-13-01 00:00:00', '2020-01-13 00:00:00', '2020-12-31 24:00:00', '0999-01-01 00:00:00',
              '2020-01-02 03:04:05.123', '2020-01-02 03:04:05Z', '2020-01-02 03:04:05+02:00', ' 2020-01-02 03:04:05',
              '2020-01-02 03:04:05 ', '2020/01/02 03:04:05', 'Jan 2 2020', '2020-01-02', 'nan', '', '12']
    for s in cases:
        try:
            want = dparser.parse(s)
        except Exception as exc:   # noqa: BLE001
            with pytest.raises(type(exc)):
                parse_date(s)
            continue
        got = parse_date(s)
        assert got == want and got.tzinfo == want.tzinfo, s


def test_period_us_equals_is_within_period():
    """kb.period_us/epoch_us integer bounds decide exactly like is_within_period (match_keywords.py:17-37)
    for naive and offset-aware dates, open bounds, equal bounds and microsecond neighbours."""
    from datetime import datetime, timedelta, timezone
    from advanced_scrapper_amd.kb import epoch_us, is_within_period, period_us
    rng = random.Random(5)

    def rnd():
        d = datetime(rng.randint(1, 9999), rng.randint(1, 12), rng.randint(1, 28), rng.randint(0, 23),
                     rng.randint(0, 59), rng.randint(0, 59), rng.choice([0, 1, 999999, rng.randint(0, 999999)]))
        if rng.random() < 0.4:
            try:
                d = d.replace(tzinfo=timezone(timedelta(minutes=rng.randint(-900, 900))))
                d - datetime(1970, 1, 1, tzinfo=timezone.utc)
            except OverflowError:
                d = d.replace(tzinfo=None)
        return d

    for _ in range(5000):
        a = rnd()
        lo = None if rng.random() < 0.2 else (a if rng.random() < 0.1 else rnd())
        hi = None if rng.random() < 0.2 else (a + timedelta(microseconds=rng.choice([-1, 0, 1])) if
                                              rng.random() < 0.2 and a.year < 9999 else rnd())
        lo_us, hi_us = period_us(lo, hi)
        assert (lo_us <= epoch_us(a) <= hi_us) == is_within_period(a, lo, hi), (a, lo, hi)


def test_native_json_rows_equal_python_assembly(golden):
    """rows.assemble_json_rows (csrc/kwrows.c) == group_hits + assemble_ticker_matches + json.dumps on seeded
    random hit records over the golden KB and articles (periods, both fields, position-less matches)."""
    import json
    from dateutil import parser as dparser
    from advanced_scrapper_amd import _native
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import assemble_ticker_matches, group_hits
    from advanced_scrapper_amd.rows import assemble_json_rows
    ckb = compile_kb(golden.kb_processed())
    frame = pd.read_csv(io.BytesIO(golden.articles_csv_bytes()))
    dates = [dparser.parse(str(v)) if pd.notna(v) else None for v in frame['date_time'].tolist()]
    valid = [p for p in range(len(ckb.names)) if not ckb.invalid_regex[p]]
    rng = np.random.default_rng(3)
    recs = []
    for d in range(len(frame)):
        for _ in range(int(rng.integers(0, 6))):
            p, f, k = valid[int(rng.integers(len(valid)))], int(rng.integers(2)), int(rng.integers(0, 4))
            if k == 0:
                recs.append((d, p, _native.KW_NOPOS, f))
            for q in rng.choice(5000, size=k, replace=False):
                recs.append((d, p, int(q), f))
    hits = np.array(recs, dtype=_native.HIT_DTYPE)
    rng.shuffle(hits)
    got = assemble_json_rows(ckb, hits, dates)
    want = [(d, t, json.dumps(m['text']), json.dumps(m['title']))
            for d, fields in sorted(group_hits(hits).items())
            for t, m in assemble_ticker_matches(ckb, fields, dates[d]).items()]
    assert len(want) > 500 and got == want


def test_append_to_csv_single_row(tmp_path, monkeypatch):
    from advanced_scrapper_amd import match_keywords as mk
    monkeypatch.chdir(tmp_path)
    os.makedirs('src_ticker_matched_articles')
    art = pd.Series({'date_time': '2020-01-02 03:04:05', 'title': float('nan'), 'url': 'u,1', 'source': 's',
                     'source_url': 'su', 'article_text': 'He said "hi"\nand left é'})
    mk.append_to_csv('src', 'AAPL', {'text': {'Apple': [0]}, 'title': {}}, art)
    mk.append_to_csv('src', 'AAPL', {'text': {'Andrés': []}, 'title': {'X': [1, 2]}}, art)
    data = open('src_ticker_matched_articles/AAPL_match.csv', encoding='utf-8').read()
    assert data.count('time_unix') == 1
    assert '"{""Andr\\u00e9s"": []}"' in data
    assert '1577934245' in data


# ------------------------------------------------------------------ C-ABI boundary
def _header_functions():
    inc = os.path.join(os.path.dirname(__file__), '..', 'include')
    hdr = ''.join(open(os.path.join(inc, f)).read() for f in sorted(os.listdir(inc)) if f.endswith('.h'))
    return sorted(set(re.findall(r'^\s*(?:int|const char \*)\s*\*?(kw_\w+|dedup_urls)\s*\(', hdr, re.M)))


def test_library_exports_every_header_symbol():
    from advanced_scrapper_amd import _native
    L = _native.lib()
    funcs = _header_functions()
    assert funcs, 'no functions parsed from the header'
    assert sorted(_native.EXPORTS) == funcs
    for f in funcs:
        assert hasattr(L, f), f
    out = subprocess.run(['nm', '-D', '--defined-only', _native.LIB_PATH], capture_output=True, text=True).stdout
    for f in funcs:
        assert re.search(rf'\bT {f}\b', out), f


def test_compile_rejects_unsupported_without_gpu():
    """kw_compile validates before touching the device."""
    import ctypes
    from advanced_scrapper_amd import _native
    L = _native.lib()
    names = ['X' * 70]
    b = np.frombuffer(names[0].encode(), dtype=np.uint8).copy()
    off = np.array([0, len(b)], dtype=np.int64)
    cls = np.array([ord('F')], dtype=np.uint8)
    h = ctypes.c_void_p()
    rc = L.kw_compile(_native.ptr(b), _native.ptr(off), _native.ptr(cls), 1, None, None,
                      _native.ptr(kb.word_bitmap()), None, 0, 0, ctypes.byref(h))
    assert rc == _native.KW_EUNSUPPORTED
    assert b'64' in L.kw_last_error(h)
    L.kw_destroy(h)


# ------------------------------------------------------------------ synthetic corpus
def test_synth_is_shard_invariant(golden):
    from advanced_scrapper_amd import synth
    ckb = compile_kb(golden.kb_processed())
    names, kinds = synth.injectable_names(ckb)
    a = synth.generate(300, names, kinds, seed=5)
    b = synth.generate(100, names, kinds, seed=5, doc_base=200)
    for i in range(100):
        assert a.text(200 + i) == b.text(i)
        assert a.title(200 + i) == b.title(i)
    c = synth.generate(300, names, kinds, seed=5)
    assert np.array_equal(a.arena, c.arena) and np.array_equal(a.off, c.off)
    assert 1500 < a.n_bytes / a.n_docs < 3500


# ------------------------------------------------------------------ error paths (match_keywords.py:152, :131, :178)
@pytest.mark.parametrize('case', ['invalid_regex', 'bad_date', 'int_dates'])
def test_dropin_error_paths_write_reference_partial_output(golden, tmp_path, monkeypatch, case):
    """When a chunk raises mid-way, the drop-in writes exactly the rows the reference wrote before raising
    and raises the same exception (tests/golden/make_error_golden.py ran the reference); the scan is the
    oracle stand-in (tests/oracle_matcher.py), everything above it is the product path."""
    import time
    from advanced_scrapper_amd import match_keywords as mk
    from tests.oracle_matcher import OracleMatcher
    monkeypatch.setenv('TZ', 'UTC')
    time.tzset()
    g = golden.error_cases()
    c = g['cases'][case]
    processed = golden.processed_from(g['kb_processed'])
    monkeypatch.chdir(tmp_path)
    os.makedirs('yahoo_ticker_matched_articles')
    m = OracleMatcher(processed)
    raised = None
    try:
        for chunk in pd.read_csv(io.StringIO(c['articles_csv']), chunksize=g['chunksize']):
            mk._write_chunk('yahoo', chunk, processed, m)
    except Exception as exc:   # noqa: BLE001
        raised = type(exc).__name__
    assert raised == c['exception']
    got = {fn: open(os.path.join('yahoo_ticker_matched_articles', fn), encoding='utf-8').read()
           for fn in os.listdir('yahoo_ticker_matched_articles')}
    assert got == c['files']


def test_egress_fast_path_probe(monkeypatch, tmp_path):
    """The fast CSV line writer is checked against the interpreter's csv writer at import; with the check
    failing, append_rows still writes the writer's bytes (every row through csv.writer)."""
    from advanced_scrapper_amd import egress
    assert egress._FAST_OK
    rows = [('a\rb', 1, 'x,y'), ('', 'q"t', 'é')]
    p1, p2 = tmp_path / 'a.csv', tmp_path / 'b.csv'
    egress.append_rows(str(p1), ('c1', 'c2', 'c3'), rows)
    monkeypatch.setattr(egress, '_FAST_OK', False)
    egress.append_rows(str(p2), ('c1', 'c2', 'c3'), rows)
    assert p1.read_bytes() == p2.read_bytes()


def _run_main(tmp_path, csv_bytes, chunksize, force_reread=False, monkeypatch=None):
    """match_keywords.run over csv_bytes in a fresh directory (the scan by the oracle stand-in); returns
    {file: bytes}.  force_reread: every output file takes the reference's re-read + sort."""
    import time
    from advanced_scrapper_amd import egress
    from advanced_scrapper_amd import match_keywords as mk
    from tests import golden_data
    from tests.oracle_matcher import OracleMatcher
    work = tmp_path / ('reread' if force_reread else 'indexed')
    work.mkdir()
    (work / 'articles.csv').write_bytes(csv_bytes)
    monkeypatch.setenv('TZ', 'UTC')
    time.tzset()
    monkeypatch.chdir(work)
    processed = golden_data.kb_processed()
    monkeypatch.setattr(mk, 'read_and_process_json_files', lambda _d: processed)
    calls = {'finish': 0}
    real = egress.RunFiles.finish

    def finish(self, name):
        if force_reread:
            return False
        ok = real(self, name)
        calls['finish'] += ok
        return ok
    monkeypatch.setattr(egress.RunFiles, 'finish', finish)
    args = mk._parse(['--info-dir', 'unused', '--articles', str(work / 'articles.csv'), '--chunksize', str(chunksize)])
    assert mk.run(args, 0, 1, None, None, matcher=OracleMatcher(processed)) == 0
    out = work / 'yahoo_ticker_matched_articles'
    return {fn: (out / fn).read_bytes() for fn in sorted(os.listdir(out))}, calls['finish']


def test_indexed_sort_equals_reread_on_shuffled_rows_with_ties(golden, tmp_path, monkeypatch):
    """The run index's sort (no re-read) writes the bytes of the reference's re-read + quicksort + rewrite,
    on rows out of time order with repeated timestamps (the unstable sort's tie order)."""
    import io
    import pandas as pd
    frame = golden.articles_frame()
    rng = np.random.default_rng(7)
    frame = frame.iloc[rng.permutation(len(frame))].reset_index(drop=True)
    frame.loc[frame.index % 5 == 0, 'date_time'] = '2016-03-04 05:06:07'     # ties across many articles
    data = frame.to_csv(index=False).encode('utf-8')
    fast, n_fast = _run_main(tmp_path, data, 150, monkeypatch=monkeypatch)
    slow, _ = _run_main(tmp_path, data, 150, force_reread=True, monkeypatch=monkeypatch)
    assert n_fast > 0 and sorted(fast) == sorted(slow)
    for fn in slow:
        assert fast[fn] == slow[fn], fn


def test_indexed_sort_declines_numeric_only_block(golden, tmp_path, monkeypatch):
    """A pandas read block (shrunk to 4 rows here) whose title cells all look numeric would be re-read as
    numbers: the index declines and the file takes the re-read path, with the same bytes as a forced re-read."""
    from advanced_scrapper_amd import egress
    monkeypatch.setattr(egress, 'PANDAS_BLOCK_ROWS', 4)
    frame = golden.articles_frame().iloc[500:600].reset_index(drop=True)
    frame['title'] = [f'{k}.50' if k % 7 else 'Apple Inc. AAPL' for k in range(len(frame))]
    data = frame.to_csv(index=False).encode('utf-8')
    fast, _ = _run_main(tmp_path, data, 40, monkeypatch=monkeypatch)
    slow, _ = _run_main(tmp_path, data, 40, force_reread=True, monkeypatch=monkeypatch)
    assert sorted(fast) == sorted(slow)
    for fn in slow:
        assert fast[fn] == slow[fn], fn


def test_native_sort_defers_numeric_looking_block(tmp_path):
    """pandas' low-memory reader infers types per 65 536-row block: a block whose title cells all look
    numeric ('007') would come back re-rendered ('7'), so the native sort must hand such a file to the
    pandas path, while the same rows with one text title per block stay native."""
    from advanced_scrapper_amd import egress
    from advanced_scrapper_amd import match_keywords as mk
    n = egress.PANDAS_BLOCK_ROWS + 10
    head = 'time_unix,date_time,text_matches,title_matches,title,url,source,source_url,article_text\n'

    def write(path, titles):
        with open(path, 'w') as fh:
            fh.write(head)
            for i, t in enumerate(titles):
                fh.write(f'{n - i},d{i},"{{}}","{{}}",{t},u{i},s,su,text {i}\n')

    bad = tmp_path / 'bad.csv'
    write(bad, ['007'] * egress.PANDAS_BLOCK_ROWS + ['abc'] * 10)
    assert mk._sort_native(str(bad)) is False
    good = tmp_path / 'good.csv'
    write(good, ['abc'] + ['007'] * (egress.PANDAS_BLOCK_ROWS - 1) + ['abc'] + ['007'] * 9)
    assert mk._sort_native(str(good)) is True


def test_threaded_json_rows_equal_serial(golden, monkeypatch):
    """kwrows_assemble_mt (hit records cut at document boundaries, slices assembled apart, concatenated) gives
    the serial kwrows_assemble's rows, tickers and JSON text on a large synthetic hit set."""
    from datetime import datetime, timedelta
    from advanced_scrapper_amd import _native
    from advanced_scrapper_amd import rows as R
    from advanced_scrapper_amd.kb import compile_kb
    ckb = compile_kb(golden.kb_processed())
    rng = np.random.default_rng(5)
    n_docs, n = 3000, 40000
    doc = np.sort(rng.integers(0, n_docs, n)).astype(np.uint32)
    pat = rng.integers(0, ckb.n_patterns, n).astype(np.uint32)
    pos = np.where(rng.random(n) < 0.2, 0xFFFFFFFF, rng.integers(0, 5000, n)).astype(np.uint32)
    fld = rng.integers(0, 2, n).astype(np.uint32)
    hits = np.zeros(n, dtype=_native.HIT_DTYPE)
    hits['doc'], hits['pattern'], hits['pos'], hits['field'] = doc, pat, pos, fld
    valid = np.array([not x for x in ckb.invalid_regex])
    hits = hits[valid[hits['pattern']]]
    base = datetime(1980, 1, 1)
    dates = [None if d % 97 == 0 else base + timedelta(seconds=int(d) * 470000) for d in range(n_docs)]
    monkeypatch.setenv('KW_HOST_THREADS', '1')
    one = R.assemble_json_raw(ckb, hits, dates)
    monkeypatch.setenv('KW_HOST_THREADS', '6')
    six = R.assemble_json_raw(ckb, hits, dates)
    assert one is not None and len(one[0]) > 10000
    for a, b in zip(one, six):
        assert np.array_equal(a, b)


def test_word_bitmap_is_cpython_word_class():
    """kb.word_bitmap (re's \\w over every code point) == chr(c).isalnum() or c == '_' for all of 0..0x10FFFF."""
    from advanced_scrapper_amd import kb
    flags = np.fromiter((chr(c).isalnum() for c in range(0x110000)), dtype=bool, count=0x110000)
    flags[0x5F] = True
    assert np.array_equal(kb.word_bitmap(), np.packbits(flags, bitorder='little').view(np.uint32))
