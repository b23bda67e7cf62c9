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
