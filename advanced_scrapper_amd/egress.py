"""Per-ticker CSV egress, byte-identical to the reference's row-at-a-time pandas appends.

The reference writes every (article, ticker) match with
``pd.DataFrame([row]).to_csv(path, mode='a', index=False, header=...)``
(match_keywords.py:128-146): one single-row frame per output row, so each
column's dtype is inferred from that one value.  pandas writes such a frame
through the stdlib ``csv`` writer (QUOTE_MINIMAL, ``"`` quote char, doubled
quotes, ``os.linesep`` line ends) after rendering each cell:

* ``str``                          -> the string itself
* ``int`` / numpy integer          -> ``str(int(v))``
* ``None`` / float NaN             -> ``''`` (``na_rep``)

Those are the only cell types a matched row of a read_csv chunk normally
holds (text columns, the ``time_unix`` int, NaN for missing cells).  Any
other cell (a non-NaN float, a bool, a timestamp ...) sends its row through
the reference's own pandas call, so the bytes are identical by construction.

What changes is the cost per row: no DataFrame per row, no ``chunk.iloc``
per (article, ticker), no second ``dateutil`` parse per row (the article's
date was already parsed once for the period filter, match_keywords.py:152),
and one file open per ticker per chunk instead of one per row.
"""
from __future__ import annotations

import csv
import io
import math
import numbers
import os
from typing import Iterable, List, Sequence

import numpy as np
import pandas as pd


def _cell(v):
    """pandas' rendering of a one-value column, or ``None`` when the fast path does not cover ``v``."""
    if isinstance(v, str):
        return v
    if v is None:
        return ''
    if isinstance(v, (bool, np.bool_)):
        return None
    if isinstance(v, (numbers.Integral, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)) and math.isnan(v):
        return ''
    return None


def _pandas_row_bytes(columns: Sequence[str], values: Sequence, header: bool) -> str:
    """The reference's own call for one row (match_keywords.py:145-146), rendered to a string."""
    buf = io.StringIO()
    pd.DataFrame([dict(zip(columns, values))]).to_csv(buf, index=False, header=header)
    return buf.getvalue()


def append_rows(path: str, columns: Sequence[str], rows: Iterable[Sequence]) -> int:
    """Append ``rows`` (value tuples in ``columns`` order) to ``path``; header iff the file is new.

    Equivalent, byte for byte, to one ``pd.DataFrame([dict(zip(columns, r))]).to_csv(path, mode='a',
    index=False, header=not os.path.exists(path))`` per row, in order.  Returns the rows written.
    """
    header = not os.path.exists(path)
    n = 0
    lines: List[str] = []
    # newline='' so the csv writer's os.linesep terminator reaches the file unchanged (pandas does the same)
    with open(path, 'a', newline='', encoding='utf-8') as fh:
        w = csv.writer(fh, lineterminator=os.linesep, delimiter=',', quotechar='"',
                       quoting=csv.QUOTE_MINIMAL, doublequote=True, escapechar=None)
        head = _join(list(columns)) if header and _FAST_OK else None
        for values in rows:
            line = _line(values) if _FAST_OK else None
            if line is None or (header and head is None):
                if lines:
                    fh.write(''.join(lines))
                    lines.clear()
                cells: List = [_cell(v) for v in values]
                if any(c is None for c in cells):
                    fh.write(_pandas_row_bytes(columns, values, header))
                else:
                    if header:
                        w.writerow(columns)
                    w.writerow(cells)
            else:
                if header:
                    lines.append(head)
                lines.append(line)
            header = False
            n += 1
        if lines:
            fh.write(''.join(lines))
    return n


_LINESEP = os.linesep
_QUOTE_TRIGGERS = tuple(dict.fromkeys((',', '"') + tuple(os.linesep)))


def _line(values: Sequence):
    """``_join`` of the rendered cells in one pass (``None`` when a cell needs the pandas or writer path)."""
    if not _NL_ONLY:
        cells = [_cell(v) for v in values]
        return None if any(c is None for c in cells) else _join(cells)
    out = []
    for v in values:
        if type(v) is not str:
            v = _cell(v)
            if v is None:
                return None
        if '\0' in v:
            return None
        if ',' in v or '"' in v or '\n' in v:
            v = '"' + v.replace('"', '""') + '"'
        out.append(v)
    if len(out) == 1 and out[0] == '':
        out[0] = '""'
    return ','.join(out) + '\n'


_NL_ONLY = os.linesep == '\n'


def _fast_path_agrees() -> bool:
    """True iff ``_line`` / ``_join`` write what this interpreter's ``csv`` writer writes (the QUOTE_MINIMAL
    rule they hard-code is CPython 3.10's) on probe rows: CR-only, LF, CRLF, tab, quotes, commas, empty
    cells, a lone empty cell, non-ASCII.  When they disagree every row goes through the writer."""
    probes = [('a', 'b'), ('cr\ronly', 'x'), ('lf\nx', 'y'), ('crlf\r\n', 'z'), ('t\tab', ''), ('say "hi"', 'q'),
              ('x,y', 'c'), ('', ''), ('',), (' lead', 'trail '), ('é中', '\x1c'), (1, 'int')]
    for row in probes:
        buf = io.StringIO()
        csv.writer(buf, lineterminator=os.linesep, delimiter=',', quotechar='"', quoting=csv.QUOTE_MINIMAL,
                   doublequote=True, escapechar=None).writerow([_cell(v) for v in row])
        if _line(row) != buf.getvalue() or _join([_cell(v) for v in row]) != buf.getvalue():
            return False
    return True



def _join(cells: Sequence[str]):
    """One CSV line as the ``csv`` writer above writes it (QUOTE_MINIMAL), or ``None`` for a cell it
    rejects (a NUL character: that row goes through the writer itself, which raises as pandas does).

    Python 3.10's writer quotes a field iff it holds the delimiter, the quote char or a character of the
    line terminator (``\\r`` alone is not quoted when the terminator is ``\\n``), and doubles embedded
    quotes; a lone empty field is written ``""``.  Scanning and joining whole ``str`` objects avoids the
    writer's per-character UCS-4 copy, which made it the slowest step of the write path.
    """
    out = []
    for c in cells:
        if '\0' in c:
            return None
        for q in _QUOTE_TRIGGERS:
            if q in c:
                c = '"' + c.replace('"', '""') + '"'
                break
        out.append(c)
    if len(out) == 1 and out[0] == '':
        out[0] = '""'
    return ','.join(out) + _LINESEP


_FAST_OK = _fast_path_agrees()


# --------------------------------------------------------------------- native rows, no final re-read
_CSV_LIB = None


def _csv_lib():
    global _CSV_LIB
    if _CSV_LIB is None:
        import ctypes
        from .ingest import _lib
        L = _lib()
        P, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.kwcsv_emit.restype = i64
        L.kwcsv_emit.argtypes = [P, P, P, i32, P, P, P, i64, P, P, P, i64, P, P]
        L.kwcsv_emit_mt.restype = i64
        L.kwcsv_emit_mt.argtypes = [P, P, P, i32, P, P, P, i64, P, P, P, i64, P, P, P, i32]
        L.kwcsv_emit_art_bytes.restype = i64
        L.kwcsv_emit_art_bytes.argtypes = [P, i32, P, P, i64]
        _CSV_LIB = L
    return _CSV_LIB


_HEADER_COLUMNS = ('time_unix', 'date_time', 'text_matches', 'title_matches', 'title', 'url', 'source',
                   'source_url', 'article_text')
PANDAS_BLOCK_ROWS = 65536   # pandas' low_memory reader infers dtypes per block of rows (2^20 // 9 columns -> 2^16)
_F_WITNESS = 0xFF
_F_NA_SHIFT = 8
_F_CR = 1 << 16


class RunFiles:
    """The per-ticker files ONE run creates (none existed when it started), indexed as they are written: each
    row's time_unix, line length and cell flags (kwcsv_emit).  At the end the reference's re-read + sort +
    rewrite (match_keywords.py:195-217) is decided from the index: when pandas' re-read provably yields the
    written values (every non-time column of every 65 536-row block keeps a text witness or is all NaN, no
    cell holds a lone '\\r'), the sorted file is the written records in ``np.argsort(time_unix,
    kind='quicksort')`` order -- the records already in that order (ascending, no ties) mean no rewrite at
    all.  Other files (pre-existing ones, those a row went to by another path) take sort_matched_csv.

    Under ``--gpus N`` every rank appends its share of each chunk in rank order: each append is keyed
    ``(chunk's first row, rank)``, the ranks' indexes of a file meet at the rank that sorts it
    (:meth:`export` / :meth:`absorb`), and the key order is the file's row order."""

    def __init__(self, out_dir: str):
        self.out_dir = out_dir
        self.pre = set(os.listdir(out_dir)) if os.path.isdir(out_dir) else set()
        self.files = {}          # name -> [[(key, stamps, lengths, flags), ...], header bytes]
        self.other = set()       # names written by another path

    def owned(self, name: str) -> bool:
        return name not in self.pre and name not in self.other

    def note_other(self, name: str):
        self.other.add(name)
        self.files.pop(name, None)

    def add(self, name: str, stamps, lengths, flags, header: bytes, key=(0, 0)):
        f = self.files.get(name)
        if f is None:
            f = self.files[name] = [[], header]
        f[0].append((key, stamps, lengths, flags))

    def export(self, names) -> dict:
        """The index entries of ``names`` (those this run indexed), to be absorbed by another rank."""
        return {n: self.files[n] for n in names if n in self.files}

    def absorb(self, exported: dict, other=()):
        """Merge another rank's exported entries (and the names it wrote by another path)."""
        for n in other:
            self.note_other(n)
        for n, (entries, header) in exported.items():
            if n in self.other:
                continue
            f = self.files.get(n)
            if f is None:
                f = self.files[n] = [[], header]
            f[0].extend(entries)

    def finish(self, name: str) -> bool:
        """Sort one indexed file as the reference's sort_matched_csv does; False = not decidable here."""
        if not self.owned(name) or name not in self.files:
            return False
        entries, header = self.files[name]
        entries = sorted(entries, key=lambda e: e[0])     # stable: one process's appends keep their order
        stamps = np.concatenate([e[1] for e in entries])
        lens = np.concatenate([e[2] for e in entries])
        flags = np.concatenate([e[3] for e in entries])
        n = len(stamps)
        if n == 0 or (flags & _F_CR).any():
            return False
        for b0 in range(0, n, PANDAS_BLOCK_ROWS):
            blk = flags[b0:b0 + PANDAS_BLOCK_ROWS]
            wit = np.bitwise_or.reduce(blk & _F_WITNESS)
            na_all = np.bitwise_and.reduce(blk >> _F_NA_SHIFT) & 0xFF
            if (wit | na_all) != 0xFF:
                return False
        path = os.path.join(self.out_dir, name)
        if os.path.getsize(path) != len(header) + int(lens.sum()):
            return False                                  # the index does not describe the file
        if n > 1 and not (np.diff(stamps) > 0).all():
            order = np.argsort(stamps, kind='quicksort')
            if not (order == np.arange(n)).all():
                with open(path, 'rb') as fh:
                    data = fh.read()
                ends = len(header) + np.cumsum(lens)
                starts = ends - lens
                mv = memoryview(data)
                body = b''.join([mv[s:e] for s, e in zip(starts[order].tolist(), ends[order].tolist())])
                with open(path, 'wb') as fh:
                    fh.write(data[:len(header)])
                    fh.write(body)
        return True


_EMIT_BUF = [np.zeros(0, dtype=np.uint8), np.zeros(0, dtype=np.uint8)]


def _scratch(k: int, cap: int) -> np.ndarray:
    """Scratch buffer k of the emitter, kept across chunks (k = 1: the articles' rendered cells)."""
    if len(_EMIT_BUF[k]) < cap:
        _EMIT_BUF[k] = np.empty(cap + cap // 4, dtype=np.uint8)
    return _EMIT_BUF[k]


def _emit_buffer(cap: int) -> np.ndarray:
    """The emitter's output buffer, kept across chunks (a fresh 100+ MB buffer per chunk costs its page faults):
    render_native's views are valid until its next call, and every caller writes them out before that."""
    if len(_EMIT_BUF[0]) < cap:
        _EMIT_BUF[0] = np.empty(cap + cap // 4, dtype=np.uint8)
    return _EMIT_BUF[0]


def render_native(chunk, raw_rows, stamps_by_doc, tickers):
    """The rows of a native chunk (``raw_rows`` = rows.assemble_json_raw's arrays, document order, KB ticker
    order) rendered by the C emitter into one buffer, grouped by ticker file: a list of 6-tuples (file name,
    line bytes, time_unix[], line lengths[], cell flags[], document ids[]) in KB ticker order, rows in article
    order within each (document ids[] = each row's article in the chunk).
    ``stamps_by_doc[d]`` = article d's time_unix.  ``None`` when the emitter cannot reproduce the writer (a
    NUL cell, a platform line end other than "\n"): the caller takes the per-row path."""
    from .ingest import _p
    row_doc, row_ti, jbuf, joff = raw_rows
    n = len(row_doc)
    if n == 0:
        return []
    if not (_FAST_OK and _NL_ONLY):
        return None
    order = np.argsort(row_ti, kind='stable')
    rd = np.ascontiguousarray(row_doc[order], dtype=np.int32)
    rs = np.ascontiguousarray(stamps_by_doc[rd], dtype=np.int64)
    j3 = np.empty(3 * n, dtype=np.int64)
    j3[0::3] = joff[2 * order]
    j3[1::3] = joff[2 * order + 1]
    j3[2::3] = joff[2 * order + 2]
    c = chunk.cells
    cols = np.asarray([chunk.col[k] for k in ('date_time', 'title', 'url', 'source', 'source_url', 'article_text')],
                      dtype=np.int32)
    jb = jbuf if len(jbuf) else np.zeros(1, np.uint8)
    line_off = np.empty(n + 1, dtype=np.int64)
    flags = np.empty(n, dtype=np.uint32)
    L = _csv_lib()
    art = _scratch(1, int(L.kwcsv_emit_art_bytes(_p(c.off), c.ncols, _p(cols), _p(rd), n)))
    from .ingest import host_threads
    cap = len(_EMIT_BUF[0])
    rc = -1
    for _ in range(2):      # -1: out too small, line_off[n] = the bytes the rows need
        out = _emit_buffer(cap)
        rc = L.kwcsv_emit_mt(_p(c.buf), _p(c.off), _p(c.flags), c.ncols, _p(cols), _p(rd), _p(rs), n, _p(jb), _p(j3),
                             _p(out), len(out), _p(line_off), _p(flags), _p(art), host_threads())
        if rc != -1:
            break
        cap = int(line_off[n])
    if rc != 0:
        return None
    ti = row_ti[order]
    cuts = np.flatnonzero(np.r_[True, ti[1:] != ti[:-1], True]).tolist()
    mv = memoryview(out)
    return [(f'{tickers[ti[a]]}_match.csv', mv[line_off[a]:line_off[b]], rs[a:b], np.diff(line_off[a:b + 1]),
             flags[a:b], rd[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]


def header_bytes() -> bytes:
    return _join(list(_HEADER_COLUMNS)).encode('utf-8')


_POOL = None


def _write_pool():
    """Host threads for the per-ticker appends (file writes release the GIL)."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        from .ingest import host_threads
        _POOL = ThreadPoolExecutor(max_workers=min(8, host_threads()), thread_name_prefix='kw-egress')
    return _POOL


def _append_file(path: str, header: bytes, data) -> None:
    new = not os.path.exists(path)
    with open(path, 'ab') as fh:
        if new:
            fh.write(header)
        fh.write(data)


def append_rendered(out_dir: str, rendered, run_files: 'RunFiles' = None, key=(0, 0)):
    """Append rendered rows (render_native) to their files, the header first in a new file; the run index
    records the rows of the files this run owns (under ``key``, see RunFiles).  Each file is written by one
    thread (the files of a chunk are distinct), so every file receives its rows in order."""
    header = header_bytes()
    if len(rendered) > 4:
        jobs = [_write_pool().submit(_append_file, os.path.join(out_dir, r[0]), header, r[1]) for r in rendered]
        for j in jobs:
            j.result()
    else:
        for r in rendered:
            _append_file(os.path.join(out_dir, r[0]), header, r[1])
    if run_files is not None:
        for name, data, stamps, lens, flags, _docs in rendered:
            if run_files.owned(name):
                run_files.add(name, stamps, lens, flags, header, key)
