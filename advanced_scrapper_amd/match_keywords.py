"""Drop-in replacement of the reference's ``match_keywords.py`` (MI355X build).

Same public functions, arguments, side effects and CSV schema as
match_keywords.py:17-246 of lwowlwowl/advanced_scrapper:

* ``is_within_period``, ``extract_time_periods``, ``process_json_data``,
  ``read_and_process_json_files``   (re-exported from :mod:`.kb`)
* ``append_to_csv(source_name, ticker, matched_names, article)``   :128-146
* ``process_chunk(source_name, chunk, processed_data)``            :148-192
* ``sort_matched_csv(file_path)``                                  :195-217
* ``main()`` / ``python -m advanced_scrapper_amd.match_keywords``   :220-246

What changes is where the per-article x per-name loop runs: ``process_chunk``
packs the chunk's ``article_text``/``title`` strings into one byte arena, and
the hand-written HIP kernels of libkwmatch compute every
(article, field, name) result on the GPU.  The host then applies the period
filter, builds the same ``ticker_matches`` dicts and appends the same rows.
``process_chunk`` runs in-process (forking after HIP initialisation is
unsafe), one call per chunk instead of one per CPU sub-chunk.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
from typing import Dict, List, Optional

import numpy as np
import pandas as pd
from dateutil import parser

from . import egress, ingest
from .ingest import NativeChunk, ShardChunk
from .dates import parse_date
from .kb import (ATTRIBUTES, compile_kb, extract_time_periods, is_within_period,  # noqa: F401 (re-export)
                 process_json_data, read_and_process_json_files)
from .rows import assemble_json_raw, assemble_json_rows
from .matcher import (GpuMatcher, assemble_ticker_matches, background_sample, field_str, group_hits,  # noqa: F401
                      pack_fields, records_from_tensor)

OUTPUT_COLUMNS = ('time_unix', 'date_time', 'text_matches', 'title_matches', 'title', 'url', 'source',
                  'source_url', 'article_text')


def _output_dir(source_name):
    return f'{source_name}_ticker_matched_articles'


def _output_path(source_name, ticker):
    return f'{_output_dir(source_name)}/{ticker}_match.csv'


# the per-ticker files of the current run() and their rows' index (egress.RunFiles), None outside run()
_RUN: Optional[egress.RunFiles] = None


def _csv_row(matched_names, article):
    """One output row (match_keywords.py:131-144)."""
    stamp = int(parser.parse(article['date_time']).timestamp())
    return {
        'time_unix': stamp,
        'date_time': article['date_time'],
        'text_matches': json.dumps(matched_names['text']),
        'title_matches': json.dumps(matched_names['title']),
        'title': article['title'],
        'url': article['url'],
        'source': article['source'],
        'source_url': article['source_url'],
        'article_text': article['article_text'],
    }


def append_to_csv(source_name, ticker, matched_names, article):
    """Append one matched article to ``{source}_ticker_matched_articles/{ticker}_match.csv``."""
    _append_rows(source_name, ticker, [_csv_row(matched_names, article)])


def _append_rows(source_name, ticker, rows):
    """Append row dicts (or value tuples in ``OUTPUT_COLUMNS`` order), one reference append per row."""
    values = (tuple(r[c] for c in OUTPUT_COLUMNS) if isinstance(r, dict) else r for r in rows)
    if _RUN is not None:
        _RUN.note_other(f'{ticker}_match.csv')
    egress.append_rows(_output_path(source_name, ticker), OUTPUT_COLUMNS, values)


def _chunk_rows(chunk, results, dates):
    """Output rows of a matched chunk grouped by ticker, from ``ticker_matches`` dicts (see :func:`_cell_rows`)."""
    cells = [(i, t, json.dumps(m['text']), json.dumps(m['title'])) for i, tm in enumerate(results)
             for t, m in tm.items()]
    return _cell_rows(chunk, cells, dates)[:2]


def _cell_rows(chunk, cells, dates):
    """Output rows grouped by ticker, in article order (value tuples, OUTPUT_COLUMNS order), and the
    exception of the first row whose cells raise (``None`` if none does).

    ``cells`` = ``(row index, ticker, text_matches JSON, title_matches JSON)`` in article then ticker order
    (rows.assemble_json_rows, or json.dumps of ``ticker_matches``).  Each row equals ``_csv_row(matched,
    chunk.iloc[i])``: the cells are read from column lists (one ``tolist`` per column instead of one ``iloc``
    per row) and ``time_unix`` reuses the article's period-filter parse (match_keywords.py:152 parses
    ``str(date_time)``, :131 parses ``date_time``; the two agree when the cell is a ``str``, otherwise :131's
    own call runs).  A chunk without an object column (``iloc`` would upcast its ints to floats) takes the
    ``iloc`` path.  When a row's ``time_unix`` raises (the reference raises in that article's first
    ``append_to_csv``, :131-132), the rows of the articles before it are kept and the exception returned.
    The third value is the failing row's index (``None`` if no row raises).
    """
    rows_by_ticker: Dict[str, list] = {}
    if not cells:
        return rows_by_ticker, None, None
    if isinstance(chunk, NativeChunk):
        # the native tokenizer's chunk (all six columns object-typed): only matched rows are decoded
        last, stamp, tail, raw = -1, None, None, None
        for i, ticker, tj, tt in cells:
            if i != last:
                raw = chunk.value(i, 'date_time')
                try:
                    stamp = int((dates[i] if isinstance(raw, str) else parser.parse(raw)).timestamp())
                except Exception as exc:   # noqa: BLE001
                    return rows_by_ticker, exc, i
                tail = tuple(chunk.value(i, c) for c in ('title', 'url', 'source', 'source_url', 'article_text'))
                last = i
            rows_by_ticker.setdefault(ticker, []).append((stamp, raw, tj, tt) + tail)
        return rows_by_ticker, None, None
    if not any(dt == object for dt in chunk.dtypes):
        last, stamp, row = -1, None, None
        for i, ticker, tj, tt in cells:
            row = chunk.iloc[i]
            try:
                stamp = int(parser.parse(row['date_time']).timestamp())
            except Exception as exc:   # noqa: BLE001 - the reference's own exception, re-raised by the caller
                return rows_by_ticker, exc, i
            rows_by_ticker.setdefault(ticker, []).append(
                (stamp, row['date_time'], tj, tt, row['title'], row['url'], row['source'], row['source_url'],
                 row['article_text']))
        return rows_by_ticker, None, None
    cols = {c: chunk[c].tolist() for c in ('date_time', 'title', 'url', 'source', 'source_url', 'article_text')}
    last, stamp, tail = -1, None, None
    for i, ticker, tj, tt in cells:
        if i != last:
            raw = cols['date_time'][i]
            try:
                stamp = int((dates[i] if isinstance(raw, str) else parser.parse(raw)).timestamp())
            except Exception as exc:   # noqa: BLE001
                return rows_by_ticker, exc, i
            tail = (cols['title'][i], cols['url'][i], cols['source'][i], cols['source_url'][i],
                    cols['article_text'][i])
            last = i
        rows_by_ticker.setdefault(ticker, []).append((stamp, raw, tj, tt) + tail)
    return rows_by_ticker, None, None


# --------------------------------------------------------------------- matcher cache
_MATCHERS: Dict[tuple, GpuMatcher] = {}


def _kb_fingerprint(processed_data) -> str:
    h = hashlib.sha1()
    for ticker, attrs in processed_data.items():
        h.update(repr(ticker).encode())
        for attr, names in attrs.items():
            h.update(repr(attr).encode())
            for name, period in names.items():
                h.update(repr((name, period)).encode())
    return h.hexdigest()


def get_matcher(processed_data, device: Optional[int] = None, sample_texts=None) -> GpuMatcher:
    """Compile (once) the knowledge base into a libkwmatch handle.

    ``sample_texts`` (the first chunk's articles) tunes the anchor choice to
    the corpus; results do not depend on it.
    """
    key = (id(processed_data), _kb_fingerprint(processed_data), device)
    m = _MATCHERS.get(key)
    if m is None:
        bg = background_sample(sample_texts) if sample_texts else None
        m = GpuMatcher(compile_kb(processed_data), device, bg)
        _MATCHERS.clear()
        _MATCHERS[key] = m
    return m


# --------------------------------------------------------------------- process_chunk
def match_chunk(chunk, processed_data, matcher: Optional[GpuMatcher] = None):
    """``ticker_matches`` of every row of ``chunk`` and the parse error, if any (see :func:`_match`)."""
    results, error, _ = _match(chunk, processed_data, matcher)
    return results, error


def _match(chunk, processed_data, matcher: Optional[GpuMatcher] = None):
    """``ticker_matches`` of every row of ``chunk`` (list aligned with the rows), the error, the dates."""
    hits, error, dates, matcher = _match_hits(chunk, processed_data, matcher)
    results, err_asm = _results(matcher, hits, dates)
    if err_asm is not None:
        raise err_asm
    return results, error, dates


def _results(matcher, hits, dates):
    """``ticker_matches`` per row; stops at the first row whose assembly raises (an in-period fuzzy name
    whose regex does not compile: the reference's ``re.error`` at :178) and returns the rows before it
    with that exception."""
    results: List[dict] = [{} for _ in range(len(dates))]
    if hits is not None and len(hits):
        for doc, fields in group_hits(hits).items():      # ascending document order
            try:
                results[doc] = assemble_ticker_matches(matcher.ckb, fields, dates[doc])
            except Exception as exc:   # noqa: BLE001 - raised after the earlier rows are written
                return results[:doc], exc
    return results, None


def _dates(values):
    """``dateutil.parse(str(v)) if notna(v) else None`` per row (match_keywords.py:152) up to the first row
    that raises; returns the dates and that exception (or ``None``)."""
    dates: List = []
    for v in values:
        try:
            dates.append(parse_date(str(v)) if pd.notna(v) else None)
        except Exception as exc:   # match_keywords.py:152 raises here for this row
            return dates, exc
    return dates, None


def _prepare(chunk):
    """The reference's per-row field prep (match_keywords.py:150-152) of a whole chunk: texts, titles, the
    dates of the rows before the first unparseable ``date_time``, and that parse error (or ``None``)."""
    texts = [field_str(v) for v in chunk['article_text'].tolist()]
    titles = [field_str(v) for v in chunk['title'].tolist()]
    dates, error = _dates(chunk['date_time'].tolist())
    return texts, titles, dates, error


def _match_hits(chunk, processed_data, matcher: Optional[GpuMatcher] = None):
    """Device hit records of ``chunk``'s rows, the parse error (if any), the parsed dates and the matcher.

    Raises the reference's exceptions: a row whose ``date_time`` does not parse
    raises after the rows before it were matched (the returned ``error`` lets
    ``process_chunk`` write those rows first, as the reference's row loop does).
    """
    if len(chunk) == 0:
        return None, None, [], matcher
    texts, titles, dates, error = _prepare(chunk)
    n_ok = len(dates)
    matcher = matcher or get_matcher(processed_data, sample_texts=texts[:n_ok])
    hits = matcher.match_strings(texts[:n_ok], titles[:n_ok]) if n_ok else None
    return hits, error, dates, matcher


def _hit_rows(chunk, matcher, hits, dates, error):
    """The output rows of a matched chunk grouped by ticker, up to its first failing article, with that
    article's exception and row (``None, None`` if none fails).  In the reference's row order a row fails
    when its ``date_time`` does not parse (:152, row ``len(dates)``), its assembly raises (``re.error``,
    :178) or its output cells raise (:131); the rows of the articles before it are written."""
    cells = assemble_json_rows(matcher.ckb, hits, dates) if hits is not None else None
    asm_row = None
    if cells is None:
        results, err_asm = _results(matcher, hits, dates)
        if err_asm is not None:
            asm_row = len(results)
        cells = [(i, t, json.dumps(m['text']), json.dumps(m['title'])) for i, tm in enumerate(results)
                 for t, m in tm.items()]
    else:
        err_asm = None
    by_ticker, err_rows, row = _cell_rows(chunk, cells, dates)
    for exc, r in ((err_rows, row), (err_asm, asm_row), (error, len(dates))):
        if exc is not None:
            return by_ticker, exc, r
    return by_ticker, None, None


def _native_rows(chunk, matcher, hits, dates, error):
    """The rows of a native chunk rendered in C (egress.render_native: JSON cells from rows.assemble_json_raw,
    the other cells straight from the tokenized chunk), up to its first failing article, with that article's
    exception and row (as :func:`_hit_rows`); ``None`` when only the Python path can answer."""
    if not isinstance(chunk, NativeChunk) or hits is None:
        return None
    raw = assemble_json_raw(matcher.ckb, hits, dates)
    if raw is None:
        return None
    row_doc = raw[0]
    stamps = np.zeros(max(len(dates), 1), dtype=np.int64)
    exc, row = None, None
    docs = np.unique(row_doc)
    fast = dates.utc_stamps(docs) if hasattr(dates, 'utc_stamps') else None
    if fast is not None:                       # a UTC process: naive dates' timestamp() = their epoch seconds
        st, k, e = fast
        stamps[docs[:k]] = st[:k]
        if e is not None:                      # that article's append raises in the reference: rows before it
            exc, row = e, int(docs[k])
    else:
        for d in docs.tolist():                # time_unix = int(parse(date_time).timestamp()), :131-132
            try:
                stamps[d] = int(dates[d].timestamp())
            except Exception as e:   # noqa: BLE001 - that article's append raises in the reference
                exc, row = e, d
                break
    if exc is not None:
        k = int(np.searchsorted(row_doc, row))   # rows are in document order
        raw = (raw[0][:k], raw[1][:k], raw[2], raw[3][:2 * k + 1])
    rendered = egress.render_native(chunk, raw, stamps, matcher.ckb.tickers)
    if rendered is None:
        return None
    if exc is None and error is not None:
        exc, row = error, len(dates)
    return rendered, exc, row


def _append_hits(source_name, chunk, matcher, hits, dates, error):
    """Append the rows of a matched chunk up to its first failing article; returns that article's exception
    and row (``None, None`` if none fails, see :func:`_hit_rows`)."""
    nat = _native_rows(chunk, matcher, hits, dates, error)
    if nat is not None:
        rendered, exc, row = nat
        egress.append_rendered(_output_dir(source_name), rendered, _RUN)
        return exc, row
    by_ticker, exc, row = _hit_rows(chunk, matcher, hits, dates, error)
    for ticker, rows in by_ticker.items():
        _append_rows(source_name, ticker, rows)
    return exc, row


def _write_hits(source_name, chunk, matcher, hits, dates, error):
    """Append the rows of a matched chunk, then raise its first error (see :func:`_hit_rows`)."""
    exc, _row = _append_hits(source_name, chunk, matcher, hits, dates, error)
    if exc is not None:
        raise exc


def _write_chunk(source_name, chunk, processed_data, matcher: Optional[GpuMatcher] = None):
    """Match ``chunk`` and append its rows; the JSON cells come from libkwrows (rows.py), or from the
    Python assembly when only it can decide (offset-less timezones, a non-compiling in-period name)."""
    hits, error, dates, matcher = _match_hits(chunk, processed_data, matcher)
    _write_hits(source_name, chunk, matcher, hits, dates, error)
    return matcher


def shard_rows(texts, titles, n_rows: int, rank: int, world: int):
    """Contiguous, byte-balanced row range [lo, hi) of ``rank`` over the first ``n_rows`` rows."""
    from .dist import byte_balanced_ranges
    off = np.zeros(2 * n_rows + 1, dtype=np.int64)
    if n_rows:
        lens = np.fromiter((len(s.encode('utf-8', 'surrogatepass')) for i in range(n_rows)
                            for s in (texts[i], titles[i])), dtype=np.int64, count=2 * n_rows)
        np.cumsum(lens, out=off[1:])
    return byte_balanced_ranges(off, world)[rank]


def _write_chunk_sharded(source_name, chunk, processed_data, matcher, exchange):
    """``process_chunk`` over ``exchange.world`` GPUs (the reference's Pool over sub-chunks,
    match_keywords.py:231-238): every rank matches its byte-balanced row range of the chunk, the hit
    records move to rank 0 (RCCL), and rank 0 -- the single writer -- appends the rows in article order.
    Rank 0's first failing row (a date, assembly or output-cell error) reaches every rank by a MIN
    all-reduce before anyone raises, so all ranks leave the chunk together: rank 0 raises the reference's
    exception, the others the same date error (every rank parsed the dates) or :class:`ShardError`."""
    if len(chunk) == 0:
        return matcher
    texts, titles, dates, error = _prepare(chunk)
    n_ok = len(dates)
    matcher = matcher or get_matcher(processed_data, sample_texts=texts[:n_ok])
    lo, hi = shard_rows(texts, titles, n_ok, exchange.rank, exchange.world)
    local = matcher.match_device(texts[lo:hi], titles[lo:hi])
    allh = exchange.gather(local, lo)
    never = np.iinfo(np.int64).max
    exc, row = None, None
    if exchange.rank == 0:
        hits = records_from_tensor(allh) if n_ok else None
        try:
            exc, row = _append_hits(source_name, chunk, matcher, hits, dates, error)
        except Exception as e:   # noqa: BLE001 - an unexpected writer error still releases the other ranks
            exc, row = e, -1
    first = int(exchange.allreduce_min([row if exc is not None else never])[0])
    if first != never:
        if exc is not None:
            raise exc
        if error is not None and first == n_ok:
            raise error
        raise ShardError(f'process_chunk stopped at row {first} of a chunk (on rank 0)')
    return matcher


def _native_sample(chunk: NativeChunk, limit: int = 4000):
    """The first rows' article texts (the anchor statistics' sample; speed only)."""
    col = chunk.col['article_text']
    return [field_str(chunk.cells.value(i, col)) for i in range(min(len(chunk), limit))]


def _native_match(chunk: NativeChunk, processed_data, matcher, exchange=None):
    """Hits of a natively read chunk: the arena is packed in C from the tokenized cells (no per-row
    ``str``); with an exchange, this rank matches its byte-balanced row range and rank 0 gets all."""
    from .dist import byte_balanced_ranges
    dates, error = chunk.dates()
    n_ok = len(dates)
    matcher = matcher or get_matcher(processed_data, sample_texts=_native_sample(chunk))
    if n_ok == 0:
        return None, dates, error, matcher
    arena, off = chunk.arena()
    off = off[:2 * n_ok + 1]
    if exchange is None:
        matcher.scan_host(arena, off, n_ok)          # libkwmatch's own device buffers: no torch in this path
        return matcher.fetch_host(), dates, error, matcher
    lo, hi = byte_balanced_ranges(off, exchange.world)[exchange.rank]
    d_arena, d_off = matcher.upload(arena, off)
    matcher.scan(d_arena, d_off[2 * lo:], hi - lo)
    allh = exchange.gather(matcher.hits_device(), lo)
    return (records_from_tensor(allh) if exchange.rank == 0 else None), dates, error, matcher


def _write_native(source_name, chunk: NativeChunk, processed_data, matcher, exchange=None):
    hits, dates, error, matcher = _native_match(chunk, processed_data, matcher, exchange)
    if exchange is None or exchange.rank == 0:
        _write_hits(source_name, chunk, matcher, hits, dates, error)
    elif error is not None:
        raise error
    return matcher


class ShardError(RuntimeError):
    """Raised on the ranks of ``--gpus N`` that did not hold the failing row of a chunk (its rank raises
    the reference's own exception)."""


def _write_shard(source_name, chunk: ShardChunk, processed_data, matcher, exchange):
    """``--gpus N`` with sharded host work: this rank parses the dates, packs and uploads the arena, scans,
    builds the JSON cells and the output rows of ITS byte-balanced share of the chunk only
    (ingest.read_chunks_sharded).  The chunk's first failing row is agreed on by a MIN all-reduce, and the
    ranks append their rows in rank order (= article order: shares are contiguous) up to it, one rank at a
    time, so every per-ticker file receives the rows in the order the reference's loop appends them."""
    dates, error = chunk.dates()
    n_ok = len(dates)
    hits = None
    if n_ok:
        arena, off = chunk.arena()
        d_arena, d_off = matcher.upload(arena, off[:2 * n_ok + 1])
        matcher.scan(d_arena, d_off, n_ok)
        hits = matcher.fetch()
    nat = _native_rows(chunk, matcher, hits, dates, error)
    if nat is not None:
        rendered, exc, row = nat
        by_ticker = None
    else:
        by_ticker, exc, row = _hit_rows(chunk, matcher, hits, dates, error)
    never = np.iinfo(np.int64).max
    # one MIN all-reduce: the chunk's first failing row, each rank's first row, and which ranks have rows
    # to append (0 = rows); a rank whose share starts after the failing row writes nothing
    w = exchange.world
    v = np.full(1 + 2 * w, never, dtype=np.int64)
    v[0] = chunk.lo + row if exc is not None else never
    v[1 + exchange.rank] = chunk.lo
    v[1 + w:] = 1
    v[1 + w + exchange.rank] = 0 if (rendered if by_ticker is None else by_ticker) else 1
    agreed = exchange.allreduce_min(v)
    first = int(agreed[0])
    writers = [r for r in range(w) if agreed[1 + w + r] == 0 and agreed[1 + r] <= first]
    for k, r in enumerate(writers):          # rank order = article order; a barrier only between writers
        if r == exchange.rank:
            if by_ticker is None:
                egress.append_rendered(_output_dir(source_name), rendered, _RUN, (chunk.chunk_index0, r))
            else:
                for ticker, rows in by_ticker.items():
                    _append_rows(source_name, ticker, rows)
        if k + 1 < len(writers):
            exchange.barrier()
    if first != never:
        if exc is not None and chunk.lo + row == first:
            raise exc
        raise ShardError(f'process_chunk stopped at row {chunk.chunk_index0 + first} of the articles (on another rank)')
    return matcher


def process_chunk(source_name, chunk, processed_data):
    """Match every row of ``chunk`` and append the per-ticker CSV rows (match_keywords.py:148-192)."""
    _write_chunk(source_name, chunk, processed_data)


# --------------------------------------------------------------------- sort
def _sort_native(file_path) -> bool:
    """sort_matched_csv's re-read, sort and rewrite without pandas when the result is provably the same
    bytes (§8(f)2); ``False`` (file untouched) hands the file to the pandas path.

    pandas' re-read (match_keywords.py:198) keeps a column ``object`` when a cell proves it text, reads an
    all-NA column as NaN, and makes ``time_unix`` int64 when every cell is a plain integer; NA strings
    become NaN, which to_csv writes as an empty cell.  ``sort_values('time_unix')`` with the default
    kind is ``np.argsort(kind='quicksort')`` on those integers (pandas' nargsort without NaNs), so ties
    keep pandas' (unstable) order.  A record whose cells are already in the writer's QUOTE_MINIMAL form,
    with no NA cell and a canonical integer, is copied as it stands; the others are rendered again.
    """
    from .ingest import CANON, NA, TEXT, parse_all
    with open(file_path, 'rb') as fh:
        data = fh.read()
    parsed = parse_all(data)
    if parsed is None:
        return False
    names, cells, span = parsed
    if 'time_unix' not in names:
        return False
    n, nc = cells.nrows, cells.ncols
    ti = names.index('time_unix')
    fl = cells.flags.reshape(n, nc)
    # pandas' low-memory reader infers each column's type per block of rows: every block must keep every
    # non-time column text (a witness) or all-NA, or a numeric-looking block would be re-rendered by pandas
    for b0 in range(0, n, egress.PANDAS_BLOCK_ROWS):
        blk = fl[b0:b0 + egress.PANDAS_BLOCK_ROWS]
        for c in range(nc):
            if c != ti and not ((blk[:, c] & TEXT).any() or (blk[:, c] & NA).all()):
                return False
    raw = [bytes(cells._mv[cells.off[r * nc + ti]:cells.off[r * nc + ti + 1]]) for r in range(n)]
    if n and (fl[:, ti] & (NA | TEXT)).any():
        return False
    try:
        ints = [int(x) for x in raw]
    except ValueError:
        return False
    if any(v >= (1 << 63) or v < -(1 << 63) for v in ints):
        return False
    order = np.argsort(np.asarray(ints, dtype=np.int64), kind='quicksort')
    plain = (fl & CANON).all(axis=1) & ~(fl & NA).any(axis=1) if n else np.zeros(0, bool)
    lines = [egress._join(list(names)).encode('utf-8')]
    nl = os.linesep.encode()
    for r in order.tolist():
        if plain[r] and str(ints[r]).encode() == raw[r]:
            lines.append(data[span[r, 0]:span[r, 1]] + nl)
        else:
            vals = [str(ints[r]) if c == ti else ('' if fl[r, c] & NA else cells.value(r, c)) for c in range(nc)]
            line = egress._join(vals)
            if line is None:
                return False
            lines.append(line.encode('utf-8'))
    with open(file_path, 'wb') as fh:
        fh.write(b''.join(lines))
    return True


def sort_matched_csv(file_path):
    """Re-read, sort by ``time_unix`` (pandas default quicksort) and rewrite (match_keywords.py:195-217)."""
    try:
        if _sort_native(file_path):
            print(f"Sorted and saved: {file_path}")
            return
        frame = pd.read_csv(file_path)
        if 'time_unix' not in frame.columns:
            frame['date_time'] = frame['date_time'].apply(parser.parse)
            frame['time_unix'] = frame['date_time'].apply(lambda d: int(d.timestamp()))
        ordered = frame.sort_values('time_unix', ascending=True)
        ordered['time_unix'] = ordered['time_unix'].astype(int)
        ordered.to_csv(file_path, index=False)
        print(f"Sorted and saved: {file_path}")
    except Exception as exc:  # noqa: BLE001 - mirrors the reference
        print(f"Error processing {file_path}: {str(exc)}")


# --------------------------------------------------------------------- CLI
def _parse(argv):
    ap = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    ap.add_argument('--source', default='yahoo')
    ap.add_argument('--info-dir', default='info/Icahn_filter')
    ap.add_argument('--articles', default='datasets/yahoo_articles_all_20250605.csv')
    ap.add_argument('--chunksize', type=int, default=20000)
    ap.add_argument('--device', type=int, default=None, help='single GPU: the HIP device (default: current)')
    ap.add_argument('--gpus', type=int, default=1,
                    help='GPUs of this node; N > 1 starts one rank per GPU (torch.distributed.run) that '
                         'matches a byte-balanced share of every chunk, rank 0 writes')
    return ap.parse_args(argv)


def main(argv=None):
    """The reference's ``__main__`` (match_keywords.py:220-246) with its constants as defaults."""
    args = _parse(argv)
    world_env = os.environ.get('WORLD_SIZE')
    if world_env is None and args.gpus > 1:
        # one process per GPU, started before this process touches the GPU
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(('127.0.0.1', 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
               '--master-addr', '127.0.0.1', f'--master-port={port}', '-m', 'advanced_scrapper_amd.match_keywords']
        cmd += list(argv if argv is not None else sys.argv[1:])
        return subprocess.call(cmd)
    if world_env is not None and int(world_env) != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world_env}')
    if args.gpus > 1:
        from . import dist
        rank, world, local = dist.init('nccl')
        return run(args, rank, world, local, 'nccl')
    return run(args, 0, 1, args.device, None)


def _prefetch(chunks, depth: int = 1):
    """Yield the items of ``chunks`` while a background thread already produces the next ``depth`` of them
    (the next chunk's tokenizing overlaps this chunk's matching and writing: the native ingest runs in C
    with the GIL released).  Order and exceptions are the producer's."""
    import queue
    import threading
    q: queue.Queue = queue.Queue(maxsize=depth)
    stop = threading.Event()
    done = object()

    def put(x) -> bool:
        """Queue x unless the consumer has left (stop set): never blocks past its exit."""
        while not stop.is_set():
            try:
                q.put(x, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def produce():
        try:
            for item in chunks:
                if not put((item, None)):
                    return
            put((done, None))
        except BaseException as exc:   # noqa: BLE001 - re-raised in the consumer, in order
            put((done, exc))

    th = threading.Thread(target=produce, name='kw-ingest', daemon=True)
    th.start()
    try:
        while True:
            item, exc = q.get()
            if item is done:
                if exc is not None:
                    raise exc
                return
            yield item
    finally:
        stop.set()
        th.join(timeout=5)


def _warm_device(device):
    """Start the HIP runtime and create the device context on a background thread (libkwmatch's
    kw_device_init, in C with the GIL released: the runtime's start-up costs a fixed fraction of a second)
    while the KB loads and the first chunk is tokenized."""
    import threading

    def warm():
        try:
            from . import _native
            _native.lib().kw_device_init(0 if device is None else int(device))
        except Exception:   # noqa: BLE001 - the matcher's own initialisation reports any error
            pass

    th = threading.Thread(target=warm, name='kw-device-init', daemon=True)
    th.start()
    return th


def run(args, rank: int, world: int, device, backend, matcher=None):
    """The driver loop on one rank: read the chunks, match (sharded over the ranks when world > 1), write,
    then sort every output file (match_keywords.py:226-246)."""
    global _RUN
    warm = _warm_device(device) if (world == 1 and matcher is None) else None
    processed = read_and_process_json_files(args.info_dir)
    out_dir = f'{args.source}_ticker_matched_articles'
    if rank == 0:
        os.makedirs(out_dir, exist_ok=True)
    if world > 1:
        from .dist import Exchange
        exchange = Exchange(rank, world, device, backend)
        os.makedirs(out_dir, exist_ok=True)
        exchange.barrier()
        try:
            return _run_sharded(args, processed, exchange, device, out_dir, matcher)
        finally:
            exchange.close()
    _RUN = egress.RunFiles(out_dir)
    try:
        # the native tokenizer (ingest.py), chunk by chunk, with pandas' own chunks where it cannot be exact;
        # the next chunk is read while this one is matched and written
        for chunk in _prefetch(ingest.read_chunks(args.articles, args.chunksize)):
            if warm is not None:
                warm.join()
                warm = None
            if isinstance(chunk, NativeChunk):
                if matcher is None:
                    matcher = get_matcher(processed, device, _native_sample(chunk))
                matcher = _write_native(args.source, chunk, processed, matcher)
                continue
            if matcher is None:
                matcher = get_matcher(processed, device, [field_str(v) for v in chunk['article_text'].tolist()])
            matcher = _write_chunk(args.source, chunk, processed, matcher)
        print("All matched CSV files have been processed.")
        for name in os.listdir(out_dir):
            # the files this run created are sorted from their write index (no re-read when already in
            # time order); the others take the reference's re-read, sort and rewrite
            if _RUN.finish(name):
                print(f"Sorted and saved: {out_dir}/{name}")
            else:
                sort_matched_csv(f"{out_dir}/{name}")
        print("All matched CSV files have been sorted by date and time.")
    finally:
        _RUN = None
    return 0


def _run_sharded(args, processed, exchange, device, out_dir, matcher=None):
    """``--gpus N``: every rank reads its byte-balanced share of each chunk (ingest.read_chunks_sharded),
    matches and writes it (rank order per chunk); then the ranks sort disjoint sets of the output files.
    A chunk pandas must parse (the native tokenizer cannot prove its dtypes) is parsed whole by every rank,
    matched in shares and written by rank 0.  Every rank indexes the rows it appends (egress.RunFiles, keyed
    by chunk and rank); each file's index meets at the rank that sorts it, so the files this run created are
    sorted from the index, without the reference's re-read (match_keywords.py:243-244)."""
    global _RUN
    rank, world = exchange.rank, exchange.world
    _RUN = egress.RunFiles(out_dir)          # every rank lists the directory before any rank writes
    try:
        for chunk in ingest.read_chunks_sharded(args.articles, args.chunksize, rank, world, exchange.allreduce_min):
            if isinstance(chunk, ShardChunk):
                if matcher is None:
                    matcher = get_matcher(processed, device, _native_sample(chunk))
                matcher = _write_shard(args.source, chunk, processed, matcher, exchange)
                continue
            if matcher is None:
                matcher = get_matcher(processed, device, [field_str(v) for v in chunk['article_text'].tolist()])
            matcher = _write_chunk_sharded(args.source, chunk, processed, matcher, exchange)
        exchange.barrier()
        if rank == 0:
            print("All matched CSV files have been processed.")
        names = sorted(os.listdir(out_dir))
        mine = names[rank::world]             # the final pass over the files, split over the ranks
        parts = exchange.exchange_objects([(_RUN.export(names[r::world]), sorted(_RUN.other))
                                           for r in range(world)])
        for src, (exported, other) in enumerate(parts):
            if src != rank:
                _RUN.absorb(exported, other)
        for name in mine:
            if _RUN.finish(name):
                print(f"Sorted and saved: {out_dir}/{name}")
            else:
                sort_matched_csv(f"{out_dir}/{name}")
        exchange.barrier()
    finally:
        _RUN = None
    if rank == 0:
        print("All matched CSV files have been sorted by date and time.")
    return 0


if __name__ == '__main__':
    sys.exit(main())
