"""Output rows' ``text_matches`` / ``title_matches`` cells built in C from the device hit records.

``assemble_json_rows`` is the write path's form of ``group_hits`` + ``assemble_ticker_matches`` +
``json.dumps`` (match_keywords.py:159-187, :137-138): it returns, in document order and KB ticker order,
``(doc, ticker, text_json, title_json)`` for every (article, ticker) the reference writes a row for.  The
C routine (csrc/kwrows.c, ``lib/libkwrows.so``) applies the period filter on integer epoch-µs bounds
(``kb.period_us``) and writes the JSON text exactly as ``json.dumps`` does.  It returns ``None`` when only
the Python path can answer: a date or period bound without a UTC offset, or an in-period name whose regex
does not compile (the Python path raises the reference's ``re.error``).
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from .kb import CompiledKB, epoch_us

_LIB = None
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib', 'libkwrows.so')
        if not os.path.exists(path):
            raise RuntimeError(f'{path} is missing: run __graft_entry__.build()')
        lib = ctypes.CDLL(path)
        P = ctypes.c_void_p
        lib.kwrows_assemble.restype = ctypes.c_int64
        lib.kwrows_assemble.argtypes = [P, ctypes.c_int64, P, P, ctypes.c_int64, P, P, P, P, P, P, P, P,
                                        ctypes.c_int32, P, P, ctypes.c_int64, P, P, ctypes.c_int64]
        lib.kwrows_assemble_mt.restype = ctypes.c_int64
        lib.kwrows_assemble_mt.argtypes = [P, ctypes.c_int64, P, P, ctypes.c_int64, P, P, P, P, P, P, P, P,
                                           ctypes.c_int32, P, P, ctypes.c_int64, P, P, ctypes.c_int64, P, ctypes.c_int32]
        _LIB = lib
    return _LIB


def _kb_tables(ckb: CompiledKB):
    """Occurrence CSR + JSON keys of a compiled KB (built once per KB), or ``None`` (see module doc)."""
    cached = ckb.__dict__.get('_rows_tables', False)
    if cached is not False:
        return cached
    occ = ckb.occurrences_us()
    if occ is None:
        ckb.__dict__['_rows_tables'] = None
        return None
    flat = [o for lst in occ for o in lst]
    off = np.zeros(len(occ) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(lst) for lst in occ])
    ti = np.array([o[0] for o in flat], dtype=np.int32)
    rank = np.array([o[1] for o in flat], dtype=np.int32)
    lo = np.array([max(o[2], _I64_MIN) for o in flat], dtype=np.int64)
    hi = np.array([min(o[3], _I64_MAX) for o in flat], dtype=np.int64)
    keys = [json.dumps(n).encode('ascii') for n in ckb.names]
    key_off = np.zeros(len(keys) + 1, dtype=np.int64)
    key_off[1:] = np.cumsum([len(k) for k in keys])
    key_buf = np.frombuffer(b''.join(keys) or b'\0', dtype=np.uint8).copy()
    invalid = np.array(ckb.invalid_regex, dtype=np.uint8)
    tables = (off, ti, rank, lo, hi, invalid, key_buf, key_off)
    ckb.__dict__['_rows_tables'] = tables
    return tables


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def assemble_json_rows(ckb: CompiledKB, hits: np.ndarray, dates: Sequence) -> Optional[List[Tuple[int, str, str, str]]]:
    """``[(doc, ticker, text_json, title_json), ...]`` of one chunk, or ``None`` (use the Python path)."""
    raw = assemble_json_raw(ckb, hits, dates)
    if raw is None:
        return None
    row_doc, row_ti, buf, off = raw
    n = len(row_doc)
    text = buf.tobytes().decode('ascii')
    oo = off.tolist()
    tickers = ckb.tickers
    return [(int(row_doc[r]), tickers[row_ti[r]], text[oo[2 * r]:oo[2 * r + 1]], text[oo[2 * r + 1]:oo[2 * r + 2]])
            for r in range(n)]


def assemble_json_raw(ckb: CompiledKB, hits: np.ndarray, dates: Sequence):
    """The rows of :func:`assemble_json_rows` as arrays: (row_doc int32[n], row_ti int32[n] (KB ticker
    index), JSON bytes uint8, offsets int64[2n + 1]: row r's text_matches then title_matches), or ``None``."""
    tables = _kb_tables(ckb)
    if tables is None:
        return None
    n_docs = len(dates)
    if len(hits) == 0 or n_docs == 0:
        return (np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, np.uint8), np.zeros(1, np.int64))
    try:
        if hasattr(dates, 'epoch_us_arrays'):            # dates.Dates: integer forms without datetimes
            date_us, date_ok = dates.epoch_us_arrays()
        else:
            date_us = np.zeros(n_docs, dtype=np.int64)
            date_ok = np.zeros(n_docs, dtype=np.uint8)
            for i, d in enumerate(dates):
                if d is not None:
                    date_us[i] = epoch_us(d)
                    date_ok[i] = 1
    except TypeError:
        return None
    h = np.ascontiguousarray(hits[np.lexsort((hits['pos'], hits['pattern'], hits['field'], hits['doc']))])
    assert h.dtype == _native.HIT_DTYPE
    off, ti, rank, lo, hi, invalid, key_buf, key_off = tables
    from .ingest import host_threads
    row_cap = max(1024, len(h) + len(h) // 2)
    out_cap = max(1 << 16, 48 * len(h))
    need = np.zeros(2, dtype=np.int64)
    for _attempt in range(2):      # -1: the rows / text need more room than guessed (need = the exact sizes)
        row_doc = np.empty(row_cap, dtype=np.int32)
        row_ti = np.empty(row_cap, dtype=np.int32)
        out = np.empty(out_cap, dtype=np.uint8)
        out_off = np.empty(2 * row_cap + 1, dtype=np.int64)
        n = _lib().kwrows_assemble_mt(_ptr(h), len(h), _ptr(date_us), _ptr(date_ok), n_docs, _ptr(off), _ptr(ti),
                                      _ptr(rank), _ptr(lo), _ptr(hi), _ptr(invalid), _ptr(key_buf), _ptr(key_off),
                                      len(ckb.tickers), _ptr(row_doc), _ptr(row_ti), row_cap, _ptr(out),
                                      _ptr(out_off), out_cap, _ptr(need), host_threads())
        if n == -2:
            return None
        if n == -3:
            raise MemoryError('kwrows_assemble: allocation failed')
        if n == -1:
            row_cap, out_cap = int(need[0]) + 1, int(need[1]) + 1
            continue
        break
    else:
        raise RuntimeError('kwrows_assemble: output kept overflowing')
    return row_doc[:n], row_ti[:n], out[:out_off[2 * n]], out_off[:2 * n + 1]
