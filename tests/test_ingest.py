"""Native CSV ingest and output sort (csrc/kwcsv.c) against pandas.

The reference reads the article CSV with pd.read_csv(chunksize=20000) (match_keywords.py:230) and
re-reads, sorts and rewrites every per-ticker file (:195-217).  The native paths must give pandas'
values and bytes: NA strings (quoted or not), blank lines, CR / CRLF / LF record ends, embedded
newlines and doubled quotes, per-chunk dtype inference (handed back to pandas), quicksort ties.
"""
import io
import math
import os
import shutil

import numpy as np
import pandas as pd
import pytest

ATOMS = ['', 'a', 'x,y', 'say "hi"', 'line\nbreak', 'cr\rlf\r\n', 'cr\ronly', 'tab\t', ' lead', 'trail ', 'é中文',
         '"', 'NA', 'null', 'None', 'nan', 'N/A', '#N/A', '12', '1.5', '-3e4', 'True', 'inf', ' 7 ', '""', "it's",
         'ab"c']
COLS = ['article_text', 'title', 'date_time', 'url', 'source', 'source_url']


def _cell(rng):
    return ''.join(ATOMS[rng.integers(len(ATOMS))] for _ in range(int(rng.integers(1, 4))))


def _same(a, b):
    return len(a) == len(b) and all((isinstance(x, float) and math.isnan(x) and isinstance(y, float) and
                                     math.isnan(y)) or x == y for x, y in zip(a, b))


@pytest.mark.parametrize('seed0', [0, 100])
def test_chunks_equal_pandas(seed0):
    from advanced_scrapper_amd import ingest
    from advanced_scrapper_amd.matcher import field_str, pack_fields
    native = 0
    for seed in range(seed0, seed0 + 100):
        rng = np.random.default_rng(seed)
        n = int(rng.integers(1, 40))
        rows = [{c: _cell(rng) for c in COLS} for _ in range(n)]
        if seed % 7 == 0:   # a numeric-only column: pandas infers a number dtype -> its own chunk
            for r in rows:
                r['title'] = str(rng.integers(0, 99))
        buf = io.StringIO()
        pd.DataFrame(rows).to_csv(buf, index=False, lineterminator='\r\n' if seed % 5 == 0 else '\n')
        data = buf.getvalue().encode('utf-8')
        if seed % 3 == 0:
            data = data.replace(b'\n', b'\n\n   \n', 2)   # blank and blanks-only lines are skipped
        cs = int(rng.integers(1, 15))
        want = list(pd.read_csv(io.BytesIO(data), chunksize=cs))
        got = list(ingest.read_chunks_bytes(data, cs))
        assert len(want) == len(got), seed
        for w, g in zip(want, got):
            if isinstance(g, ingest.NativeChunk):
                native += 1
                f = g.frame()
                assert list(w.index) == list(f.index), seed
                for c in COLS:
                    assert _same(w[c].tolist(), f[c].tolist()), (seed, c)
                ar, off = g.arena()
                ar2, off2 = pack_fields([field_str(v) for v in w['article_text'].tolist()],
                                        [field_str(v) for v in w['title'].tolist()])
                assert np.array_equal(off, off2) and bytes(ar[:off[-1]]) == bytes(ar2[:off2[-1]]), seed
            else:
                assert list(w.columns) == list(g.columns) and w.equals(g), seed
    assert native > 50


def test_golden_articles_native(golden):
    from advanced_scrapper_amd import ingest
    data = golden.articles_csv_bytes()
    cs = golden.chunksize()
    want = list(pd.read_csv(io.BytesIO(data), chunksize=cs))
    got = list(ingest.read_chunks_bytes(data, cs))
    assert all(isinstance(g, ingest.NativeChunk) for g in got)
    for w, g in zip(want, got):
        f = g.frame()
        for c in COLS:
            assert _same(w[c].tolist(), f[c].tolist()), c


def _pandas_sort(path):
    frame = pd.read_csv(path)
    ordered = frame.sort_values('time_unix', ascending=True)
    ordered['time_unix'] = ordered['time_unix'].astype(int)
    ordered.to_csv(path, index=False)


@pytest.mark.parametrize('seed0', [0, 50])
def test_sort_native_equals_pandas(tmp_path, seed0):
    """The native rewrite == pandas' re-read + quicksort + to_csv, byte for byte (ties in time_unix, NA
    strings in text cells, quoting, numeric-only columns handed to pandas)."""
    from advanced_scrapper_amd import egress
    from advanced_scrapper_amd import match_keywords as mk
    cols = ('time_unix', 'date_time', 'text_matches', 'title_matches', 'title', 'url', 'source', 'source_url',
            'article_text')
    taken = 0
    for seed in range(seed0, seed0 + 50):
        rng = np.random.default_rng(seed)
        n = int(rng.integers(1, 60))
        atoms = [a for a in ATOMS if '\r' not in a]
        rows = []
        for _ in range(n):
            t = int(rng.integers(0, 6)) * 1000 + (0 if seed % 2 else int(rng.integers(0, 10**6)))
            rows.append((t, '2020-01-01 00:00:00', '{"A": [1]}', '{}') +
                        tuple(''.join(atoms[rng.integers(len(atoms))] for _ in range(2)) for _ in range(5)))
        if seed % 9 == 0:
            rows = [r[:4] + (str(i),) + r[5:] for i, r in enumerate(rows)]   # numeric-only title column
        p1, p2 = tmp_path / f'a{seed}.csv', tmp_path / f'b{seed}.csv'
        egress.append_rows(str(p1), cols, rows)
        shutil.copy(p1, p2)
        before = p1.read_bytes()
        native = mk._sort_native(str(p1))
        taken += native
        _pandas_sort(str(p2))
        if not native:
            assert p1.read_bytes() == before, seed      # declined: untouched, the pandas path sorts it
            mk.sort_matched_csv(str(p1))
        assert p1.read_bytes() == p2.read_bytes(), (seed, native)
    assert taken > 25


@pytest.mark.parametrize('threads', ['1', '3', '7'])
def test_threaded_tokenizer_equals_pandas(monkeypatch, threads):
    """kwcsv_parse_mt over several threads (row ranges tokenized apart, then compacted) gives pandas' cells,
    the single-thread arena and the same chunk decisions, on chunks large enough to split."""
    from advanced_scrapper_amd import ingest
    from advanced_scrapper_amd.matcher import field_str, pack_fields
    monkeypatch.setenv('KW_HOST_THREADS', threads)
    atoms = [a for a in ATOMS if '\r' not in a]   # (an unquoted lone CR ends a record: pandas' own chunks)
    for seed in (3, 4):
        rng = np.random.default_rng(seed)
        rows = [{c: ''.join(atoms[rng.integers(len(atoms))] for _ in range(int(rng.integers(1, 4)))) for c in COLS}
                for _ in range(700)]
        buf = io.StringIO()
        pd.DataFrame(rows).to_csv(buf, index=False, lineterminator='\r\n' if seed % 2 else '\n')
        data = buf.getvalue().encode('utf-8').replace(b'\n', b'\n\n  \n', 5)
        want = list(pd.read_csv(io.BytesIO(data), chunksize=500))
        got = list(ingest.read_chunks_bytes(data, 500))
        assert len(want) == len(got)
        assert all(isinstance(g, ingest.NativeChunk) for g in got)
        for w, g in zip(want, got):
            f = g.frame()
            for c in COLS:
                assert _same(w[c].tolist(), f[c].tolist()), (seed, c)
            ar, off = g.arena()
            ar2, off2 = pack_fields([field_str(v) for v in w['article_text'].tolist()],
                                    [field_str(v) for v in w['title'].tolist()])
            assert np.array_equal(off, off2) and bytes(ar[:off[-1]]) == bytes(ar2[:off2[-1]]), seed


def test_native_dates_equal_parse_date(monkeypatch):
    """NativeChunk.dates (kwcsv_dates + dateutil for the other layouts) == [parse_date(str(v)) if notna(v) else
    None] row by row, stopping at the same row with the same exception; epoch_us_arrays == kb.epoch_us."""
    import time
    from advanced_scrapper_amd import ingest
    from advanced_scrapper_amd.dates import parse_date
    from advanced_scrapper_amd.kb import epoch_us
    monkeypatch.setenv('TZ', 'UTC')
    time.tzset()
    cells = ['2020-02-29 12:34:56', '2021-02-29 12:34:56', '1999-12-31T23:59:59', '0999-01-01 00:00:00',
             '1000-01-01 00:00:00', '9999-12-31 23:59:59', '2020-13-01 00:00:00', '2020-01-01 24:00:00',
             '2020-01-01 00:00', '2020-01-01 00:00:00.5', '２０２０-01-01 00:00:00', 'June 5 2020 10:00',
             '2020-06-05 10:00:00+02:00', '', 'NA', '1900-02-29 00:00:00', '2000-02-29 00:00:00', '2024-06-01 00:60:00']
    rows = [{'article_text': 'a', 'title': 't', 'date_time': d, 'url': 'u', 'source': 's', 'source_url': 'x'}
            for d in cells]
    buf = io.StringIO()
    pd.DataFrame(rows).to_csv(buf, index=False)
    data = buf.getvalue().encode('utf-8')
    (chunk,) = list(ingest.read_chunks_bytes(data, 100))
    assert isinstance(chunk, ingest.NativeChunk)
    vals = pd.read_csv(io.BytesIO(data))['date_time'].tolist()
    want, want_exc = [], None
    for v in vals:
        try:
            want.append(parse_date(str(v)) if pd.notna(v) else None)
        except Exception as exc:   # noqa: BLE001
            want_exc = exc
            break
    got, exc = chunk.dates()
    assert type(exc) is type(want_exc) and str(exc) == str(want_exc)
    assert list(got) == want and len(got) == len(want)
    us, ok = got.epoch_us_arrays()
    assert ok.tolist() == [d is not None for d in want]
    assert [int(u) for u, d in zip(us, want) if d is not None] == [epoch_us(d) for d in want if d is not None]
    rows_ = [i for i, d in enumerate(want) if d is not None]
    assert got.utc_stamps(rows_)[0].tolist() == [int(want[i].timestamp()) for i in rows_]
    monkeypatch.setenv('TZ', 'America/New_York')
    time.tzset()
    try:
        assert got.utc_stamps(rows_) is None        # a zone with transitions: the caller calls timestamp()
    finally:
        monkeypatch.setenv('TZ', 'UTC')
        time.tzset()


@pytest.mark.parametrize('threads', [1, 5])
def test_threaded_emitter_equals_serial(threads):
    """kwcsv_emit_mt (articles rendered in parallel, row offsets by prefix sum, rows in parallel) writes the
    serial kwcsv_emit's bytes, line offsets and cell flags (NA cells, quoting, '\\r', negative stamps)."""
    from advanced_scrapper_amd import egress, ingest
    from advanced_scrapper_amd.ingest import _p
    L = egress._csv_lib()
    rng = np.random.default_rng(11)
    rows = [{c: _cell(rng) for c in COLS} for _ in range(900)]
    buf = io.StringIO()
    pd.DataFrame(rows).to_csv(buf, index=False, lineterminator='\r\n')
    (chunk,) = [g for g in ingest.read_chunks_bytes(buf.getvalue().encode('utf-8'), 1000)]
    assert isinstance(chunk, ingest.NativeChunk)
    c = chunk.cells
    cols = np.asarray([chunk.col[k] for k in ('date_time', 'title', 'url', 'source', 'source_url', 'article_text')],
                      dtype=np.int32)
    n = 2500
    rd = np.sort(rng.integers(0, len(chunk), n)).astype(np.int32)
    rd = rd[np.argsort(rng.integers(0, 40, n), kind='stable')]          # ticker-grouped order
    rs = rng.integers(-2**40, 2**40, n).astype(np.int64)
    js = [('{"A": [%d]}' % k if k % 3 else '{}') + ('"\r' if k % 17 == 0 else '') + ('"x", ' * (k % 50))
          for k in range(2 * n)]                                        # long quoted cells too
    jbuf = np.frombuffer(''.join(js).encode(), dtype=np.uint8).copy()
    joff = np.zeros(2 * n + 1, dtype=np.int64)
    joff[1:] = np.cumsum([len(j) for j in js])
    j3 = np.empty(3 * n, dtype=np.int64)
    j3[0::3], j3[1::3], j3[2::3] = joff[0:-1:2], joff[1::2], joff[2::2]
    cap = 64 << 20
    o1, l1, f1 = np.empty(cap, np.uint8), np.empty(n + 1, np.int64), np.empty(n, np.uint32)
    assert L.kwcsv_emit(_p(c.buf), _p(c.off), _p(c.flags), c.ncols, _p(cols), _p(rd), _p(rs), n, _p(jbuf), _p(j3),
                        _p(o1), cap, _p(l1), _p(f1)) == 0
    art = np.empty(int(L.kwcsv_emit_art_bytes(_p(c.off), c.ncols, _p(cols), _p(rd), n)), np.uint8)
    o2, l2, f2 = np.empty(cap, np.uint8), np.empty(n + 1, np.int64), np.empty(n, np.uint32)
    assert L.kwcsv_emit_mt(_p(c.buf), _p(c.off), _p(c.flags), c.ncols, _p(cols), _p(rd), _p(rs), n, _p(jbuf),
                           _p(j3), _p(o2), cap, _p(l2), _p(f2), _p(art), threads) == 0
    assert np.array_equal(l1, l2) and np.array_equal(f1, f2)
    assert bytes(o1[:l1[-1]]) == bytes(o2[:l2[-1]])
    small = np.empty(16, np.uint8)           # too small: -1 and the bytes needed
    assert L.kwcsv_emit_mt(_p(c.buf), _p(c.off), _p(c.flags), c.ncols, _p(cols), _p(rd), _p(rs), n, _p(jbuf),
                           _p(j3), _p(small), 16, _p(l2), _p(f2), _p(art), threads) == -1
    assert l2[-1] == l1[-1]
