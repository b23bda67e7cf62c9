"""Article ingest without pandas on the hot path (reference match_keywords.py:230, :150-152).

``read_chunks(path, chunksize)`` yields the article CSV in ``chunksize``-row chunks, like
``pd.read_csv(path, chunksize=...)``.  Each chunk is tokenized by the C tokenizer (csrc/kwcsv.c,
``lib/libkwcsv.so``) into unescaped cell bytes, offsets and per-cell flags; the matcher's byte arena
(text then title of every row, NaN -> ``"nan"``) is packed in C straight from the cells, and the host
only decodes the cells it needs as Python ``str`` (dates of every row, the output cells of matched
rows).  A chunk comes back as a :class:`NativeChunk` when the tokenizer's result provably equals
pandas' for the six columns the path reads -- every record has the header's field count, no
malformed quoting, valid UTF-8, and each needed column holds a cell that keeps it dtype ``object``
(pandas infers dtypes per chunk) -- and otherwise as the ``pandas.DataFrame`` pandas itself parses
from the same bytes, so every consumer sees pandas' values.
"""
from __future__ import annotations

import ctypes
import io
import math
import os
from typing import Iterator, List, Optional, Sequence, Union

import numpy as np
import pandas as pd

NEEDED = ('article_text', 'title', 'date_time', 'url', 'source', 'source_url')
QUOTED, NA, TEXT, CANON = 1, 2, 4, 8

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib', 'libkwcsv.so')
        if not os.path.exists(path):
            raise RuntimeError(f'{path} is missing: run __graft_entry__.build()')
        L = ctypes.CDLL(path)
        P, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.kwcsv_parse.restype = i64
        L.kwcsv_parse.argtypes = [P, i64, i64, i64, i32, P, P, i32, P, i64, P, P, P, P]
        L.kwcsv_pack.restype = i64
        L.kwcsv_pack.argtypes = [P, P, P, i64, i32, i32, i32, P, i64, P]
        L.kwcsv_utf8_ok.restype = i32
        L.kwcsv_utf8_ok.argtypes = [P, P, P, i64, i32, i32]
        L.kwcsv_records.restype = i64
        L.kwcsv_records.argtypes = [P, i64, i64, i64, i32, P]
        L.kwcsv_parse_mt.restype = i64
        L.kwcsv_parse_mt.argtypes = [P, i64, P, i64, i32, P, P, i32, P, P, P, i32]
        L.kwcsv_utf8_ok_mt.restype = None
        L.kwcsv_utf8_ok_mt.argtypes = [P, P, P, i64, i32, P, i32, P, i32]
        L.kwcsv_pack_mt.restype = i64
        L.kwcsv_pack_mt.argtypes = [P, P, P, i64, i32, i32, i32, P, i64, P, i32]
        L.kwcsv_dates.restype = None
        L.kwcsv_dates.argtypes = [P, P, P, i64, i32, i32, P, P, i32]
        _LIB = L
    return _LIB


def host_threads() -> int:
    """Host threads of the native ingest / egress: the CPUs this process may use (affinity), at most 16, or
    ``KW_HOST_THREADS``."""
    env = os.environ.get('KW_HOST_THREADS')
    if env:
        return max(1, int(env))
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    return max(1, min(16, n))


def _na_table():
    """pandas' own default NA strings (the parser's STR_NA_VALUES) as one byte buffer + offsets."""
    from pandas._libs.parsers import STR_NA_VALUES
    vals = sorted(v.encode('utf-8') for v in STR_NA_VALUES)
    off = np.zeros(len(vals) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(v) for v in vals])
    return np.frombuffer(b''.join(vals) or b'\0', dtype=np.uint8).copy(), off, len(vals)


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


class Cells:
    """Tokenized records of one chunk: cell c of row r is ``buf[off[r*ncols+c]:off[r*ncols+c+1]]``."""

    def __init__(self, buf: np.ndarray, off: np.ndarray, flags: np.ndarray, nrows: int, ncols: int):
        self.buf, self.off, self.flags, self.nrows, self.ncols = buf, off, flags, nrows, ncols
        self._mv = memoryview(buf)

    def value(self, r: int, c: int):
        """The cell as pandas gives it in an object column: ``str``, or NaN for an NA string."""
        k = r * self.ncols + c
        if self.flags[k] & NA:
            return math.nan
        return bytes(self._mv[self.off[k]:self.off[k + 1]]).decode('utf-8')

    def column(self, c: int) -> List:
        off = self.off.tolist()
        fl = self.flags.tolist()
        mv, n = self._mv, self.ncols
        out = []
        for r in range(self.nrows):
            k = r * n + c
            out.append(math.nan if fl[k] & NA else bytes(mv[off[k]:off[k + 1]]).decode('utf-8'))
        return out


class NativeChunk:
    """One chunk read by the native tokenizer (the columns the path reads, decoded on demand)."""

    def __init__(self, cells: Cells, columns: Sequence[str], index0: int):
        self.cells = cells
        self.columns = list(columns)
        self.col = {c: i for i, c in enumerate(self.columns)}
        self.index0 = index0          # row number of the chunk's first row in the file (pandas' index)
        self._cache = {}

    def __len__(self):
        return self.cells.nrows

    def column_list(self, name: str) -> List:
        v = self._cache.get(name)
        if v is None:
            v = self._cache[name] = self.cells.column(self.col[name])
        return v

    def value(self, r: int, name: str):
        v = self._cache.get(name)
        return v[r] if v is not None else self.cells.value(r, self.col[name])

    def arena(self, pad: int = 64):
        """The matcher's arena and 2n+1 offsets (text, title per row; NaN -> "nan")."""
        c = self.cells
        n = c.nrows
        cap = int(c.off[-1]) + 3 * 2 * n + pad
        arena = np.empty(cap, dtype=np.uint8)
        off = np.zeros(2 * n + 1, dtype=np.int64)
        got = _lib().kwcsv_pack_mt(_p(c.buf), _p(c.off), _p(c.flags), n, c.ncols, self.col['article_text'],
                                   self.col['title'], _p(arena), cap - pad, _p(off), host_threads())
        if got < 0:
            raise RuntimeError('kwcsv_pack: arena too small')
        arena[got:got + pad] = 0
        return arena[:got + pad], off

    def dates(self):
        """The reference's per-row ``dateutil.parse(str(v)) if notna(v) else None`` (match_keywords.py:152) of
        the ``date_time`` column up to the first row that raises: (:class:`dates.Dates`, that exception or
        ``None``).  Cells of the dataset's layout are parsed in C (kwcsv_dates), the others by
        dates.parse_date (dateutil)."""
        from .dates import Dates, parse_date
        c = self.cells
        n = c.nrows
        us = np.empty(max(n, 1), dtype=np.int64)
        kind = np.empty(max(n, 1), dtype=np.uint8)
        _lib().kwcsv_dates(_p(c.buf), _p(c.off), _p(c.flags), n, c.ncols, self.col['date_time'], _p(us), _p(kind),
                           host_threads())
        slow = {}
        for r in np.flatnonzero(kind[:n] == 0).tolist():
            try:
                slow[r] = parse_date(str(self.value(r, 'date_time')))
            except Exception as exc:   # noqa: BLE001 - match_keywords.py:152 raises here for this row
                return Dates(us[:r], kind[:r], {k: v for k, v in slow.items() if k < r}), exc
        return Dates(us[:n], kind[:n], slow), None

    def frame(self) -> pd.DataFrame:
        """The chunk as pandas would give it (object columns; for the drop-in process_chunk API)."""
        data = {name: self.column_list(name) for name in self.columns}
        return pd.DataFrame(data, index=pd.RangeIndex(self.index0, self.index0 + len(self)))


def _split_header(buf: bytes):
    """Header fields and the byte position after the header record (simple unquoted or quoted names)."""
    nl = buf.find(b'\n')
    cr = buf.find(b'\r', 0, nl if nl >= 0 else len(buf))    # only within the first line (not the whole file)
    ends = [k for k in (nl, cr) if k >= 0]
    end = min(ends) if ends else len(buf)
    head = bytes(buf[:end]).decode('utf-8')
    pos = end
    if buf[pos:pos + 2] == b'\r\n':
        pos += 2
    elif pos < len(buf):
        pos += 1
    import csv
    names = next(csv.reader([head])) if head else []
    return names, head, pos


def _map(path: str):
    """The file's bytes, memory-mapped read-only (ranks of one node share the page cache; nothing is copied)."""
    import mmap
    with open(path, 'rb') as fh:
        if os.fstat(fh.fileno()).st_size == 0:
            return b''
        return mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)


def read_chunks(path: str, chunksize: int) -> Iterator[Union[NativeChunk, pd.DataFrame]]:
    """Chunks of the article CSV: :class:`NativeChunk` where the fast path equals pandas, else the
    ``DataFrame`` pandas parses from the same rows (see the module doc)."""
    yield from read_chunks_bytes(_map(path), chunksize, path)


def _pandas_rows(data, pos: int, end: int, index0: int, head_end: int) -> pd.DataFrame:
    """pandas on exactly the records in data[pos:end) (dtype inference is per chunk): the header + these bytes."""
    frame = pd.read_csv(io.BytesIO(bytes(data[:head_end]) + bytes(data[pos:end])))
    frame.index = pd.RangeIndex(index0, index0 + len(frame))
    return frame


def _pandas_rest(data, pos: int, chunksize: int, index0: int, head_end: int):
    """A record the tokenizer does not reproduce: pandas takes the rest of the file, chunk by chunk."""
    tail = bytes(data[:head_end]) + bytes(data[pos:])
    for frame in pd.read_csv(io.BytesIO(tail), chunksize=chunksize):
        frame.index = pd.RangeIndex(index0, index0 + len(frame))
        index0 += len(frame)
        yield frame


def _header_ok(names) -> bool:
    return len(names) > 0 and len(set(names)) == len(names) and all(n in names for n in NEEDED)


_NA = None


def _tokenize(buf: np.ndarray, starts: np.ndarray, ncols: int):
    """kwcsv_parse_mt of the records whose starts kwcsv_records found (``starts`` = rows + 1 entries, the last
    = the position after the last record) -> Cells, or None when a record is not reproduced exactly."""
    global _NA
    if _NA is None:
        _NA = _na_table()
    na_buf, na_off, n_na = _NA
    rows = len(starts) - 1
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    out = np.empty(int(starts[-1] - starts[0]) + 16, dtype=np.uint8)     # a record's cells take at most its bytes
    coff = np.empty(rows * ncols + 1, dtype=np.int64)
    cfl = np.empty(max(rows * ncols, 1), dtype=np.uint8)
    got = _lib().kwcsv_parse_mt(_p(buf), len(buf), _p(starts), rows, ncols, _p(na_buf), _p(na_off), n_na, _p(out),
                                _p(coff), _p(cfl), host_threads())
    if got != rows:
        return None
    return Cells(out, coff[:rows * ncols + 1], cfl[:rows * ncols], int(rows), ncols)


def _native_flags(cells: Cells, need_idx) -> np.ndarray:
    """Per needed column: [no text witness among these rows, invalid UTF-8 among them] (0 / 1)."""
    n, nc = cells.nrows, cells.ncols
    fl = cells.flags.reshape(n, nc) if n else np.zeros((0, nc), np.uint8)
    cols = np.asarray(need_idx, dtype=np.int32)
    ok = np.zeros(len(cols), dtype=np.int32)
    _lib().kwcsv_utf8_ok_mt(_p(cells.buf), _p(cells.off), _p(cells.flags), n, nc, _p(cols), len(cols), _p(ok),
                            host_threads())
    out = np.zeros(2 * len(need_idx), dtype=np.int64)
    for k, c in enumerate(need_idx):
        out[2 * k] = 0 if (n and (fl[:, c] & TEXT).any()) else 1
        out[2 * k + 1] = 0 if ok[k] else 1
    return out


def read_chunks_bytes(data, chunksize: int, path: Optional[str] = None) -> Iterator[Union[NativeChunk, pd.DataFrame]]:
    names, head, pos = _split_header(data)
    ncols = len(names)
    if not _header_ok(names):
        yield from pd.read_csv(io.BytesIO(bytes(data)) if path is None else path, chunksize=chunksize)
        return
    need_idx = [names.index(n) for n in NEEDED]
    buf = np.frombuffer(data, dtype=np.uint8)
    head_end = pos
    L = _lib()
    index0 = 0
    starts = np.empty(chunksize + 1, dtype=np.int64)
    while pos < len(data):
        rows = L.kwcsv_records(_p(buf), len(buf), pos, chunksize, ncols, _p(starts))
        if rows == 0:
            break
        if rows < 0:
            yield from _pandas_rest(data, pos, chunksize, index0, head_end)
            return
        end = int(starts[rows])
        cells = _tokenize(buf, starts[:rows + 1], ncols)
        if cells is None:
            yield from _pandas_rest(data, pos, chunksize, index0, head_end)
            return
        if not _native_flags(cells, need_idx).any():
            yield NativeChunk(cells, names, index0)
        else:
            yield _pandas_rows(data, pos, end, index0, head_end)
        index0 += int(rows)
        pos = end


class ShardChunk(NativeChunk):
    """This rank's byte-balanced share [lo, hi) of one chunk's rows (``--gpus N``): its cells only; the chunk
    has ``chunk_rows`` rows starting at file row ``chunk_index0``."""

    def __init__(self, cells: Cells, columns, chunk_index0: int, lo: int, hi: int, chunk_rows: int):
        super().__init__(cells, columns, chunk_index0 + lo)
        self.chunk_index0, self.lo, self.hi, self.chunk_rows = chunk_index0, lo, hi, chunk_rows


def balanced_cuts(starts: np.ndarray, world: int):
    """Contiguous row ranges of ~equal record bytes (starts = rows + 1 record start offsets)."""
    n = len(starts) - 1
    total = float(starts[-1] - starts[0])
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(starts[1:], starts[0] + total * r / world, side='left')) + 1)
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def read_chunks_sharded(path: str, chunksize: int, rank: int, world: int, allreduce_min
                        ) -> Iterator[Union[ShardChunk, pd.DataFrame]]:
    """The ``--gpus N`` reader: every rank memory-maps the file and finds each chunk's record boundaries
    (kwcsv_records, no cell copies), then tokenizes only its own byte-balanced share of the chunk's
    records.  Whether the chunk equals pandas' (a text witness in each needed column, valid UTF-8) is
    decided over the whole chunk by ``allreduce_min`` (an element-wise MIN of small int64 vectors over the
    ranks).  Every rank gets the same sequence: a :class:`ShardChunk` (its rows) per native chunk, the
    whole chunk as pandas' DataFrame otherwise."""
    data = _map(path)
    names, head, pos = _split_header(data)
    ncols = len(names)
    if not _header_ok(names):
        yield from pd.read_csv(path, chunksize=chunksize)
        return
    need_idx = [names.index(n) for n in NEEDED]
    buf = np.frombuffer(data, dtype=np.uint8)
    head_end = pos
    L = _lib()
    index0 = 0
    starts = np.empty(chunksize + 1, dtype=np.int64)
    while pos < len(data):
        rows = L.kwcsv_records(_p(buf), len(buf), pos, chunksize, ncols, _p(starts))
        if rows == 0:
            break
        if rows < 0:
            yield from _pandas_rest(data, pos, chunksize, index0, head_end)
            return
        rows = int(rows)
        end = int(starts[rows])
        lo, hi = balanced_cuts(starts[:rows + 1], world)[rank]
        if hi > lo:
            # the share's last record ends where the next share's first begins (blank lines are skipped)
            tok = _tokenize(buf, starts[lo:hi + 1], ncols)
        else:   # no rows on this rank: nothing to witness, nothing invalid
            tok = Cells(np.zeros(16, np.uint8), np.zeros(1, np.int64), np.zeros(1, np.uint8), 0, ncols)
        local = np.zeros(2 * len(need_idx) + 1, dtype=np.int64)
        if tok is None:
            local[-1] = 1
        else:
            local[:-1] = _native_flags(tok, need_idx)
        # witness: some rank has one (MIN of "no witness" = 0); UTF-8 and tokenizing: every rank is fine
        # (MIN of the negated flags, i.e. MAX of the failures, through -x)
        red = allreduce_min(np.concatenate([local[0:-1:2], -local[1:-1:2], -local[-1:]]))
        k = len(need_idx)
        native = not red[:k].any() and not (red[k:] < 0).any()
        if native:
            yield ShardChunk(tok, names, index0, lo, hi, rows)
        else:
            yield _pandas_rows(data, pos, end, index0, head_end)
        index0 += rows
        pos = end


def parse_all(data: bytes):
    """Every record of a whole CSV file: (column names, Cells, record byte spans [n, 2]) or ``None``
    when the tokenizer cannot reproduce pandas' split of the file (the caller falls back to pandas)."""
    names, _head, pos = _split_header(data)
    ncols = len(names)
    if ncols == 0 or len(set(names)) != ncols:
        return None
    na_buf, na_off, n_na = _na_table()
    buf = np.frombuffer(data, dtype=np.uint8)
    # records <= terminators + 1; cells <= bytes
    max_rows = data.count(b'\n') + data.count(b'\r') + 1
    out = np.empty(len(data) + 16, dtype=np.uint8)
    coff = np.empty(max_rows * ncols + 1, dtype=np.int64)
    cfl = np.empty(max(max_rows * ncols, 1), dtype=np.uint8)
    span = np.empty(2 * max_rows + 2, dtype=np.int64)
    newpos = ctypes.c_int64(pos)
    rows = _lib().kwcsv_parse(_p(buf), len(data), pos, max_rows, ncols, _p(na_buf), _p(na_off), n_na, _p(out),
                              len(data) + 16, _p(coff), _p(cfl), ctypes.byref(newpos), _p(span))
    if rows < 0 or newpos.value != len(data):
        return None
    cells = Cells(out, coff[:rows * ncols + 1], cfl[:rows * ncols], int(rows), ncols)
    return names, cells, span[:2 * rows].reshape(-1, 2)
