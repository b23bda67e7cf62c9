"""Article date parsing for the period filter and ``time_unix`` (match_keywords.py:131,152).

The reference calls ``dateutil.parser.parse(str(date_time))`` once per article
(:152) and again per output row (:131): tens of microseconds each, which at
GPU scan rates is the host's largest per-article cost.  The scraped dataset's
``date_time`` cells are ``YYYY-MM-DD HH:MM:SS``; for a
string of exactly that shape (``T`` or space between date and time) whose
fields form a valid date and time, dateutil returns the naive
``datetime(Y, M, D, h, m, s)``, which is what the fast path builds.  Every
other string — other layouts, fractional seconds, zones, out-of-range fields,
years below 1000 — goes to dateutil itself, so results (and exceptions) are
dateutil's by construction.
"""
from __future__ import annotations

import re
from datetime import datetime, timedelta

from dateutil import parser as _dparser

_ISO = re.compile(r'(\d{4})-(\d{2})-(\d{2})[ T](\d{2}):(\d{2}):(\d{2})')
_DAYS = (31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31)


def parse_date(s: str) -> datetime:
    """``dateutil.parser.parse(s)`` for a ``str``, with the dataset's layout parsed directly."""
    m = _ISO.fullmatch(s)
    if m is not None:
        y, mo, d, hh, mi, ss = (int(x) for x in m.groups())
        if y >= 1000 and 1 <= mo <= 12 and hh < 24 and mi < 60 and ss < 60:
            dim = 29 if mo == 2 and y % 4 == 0 and (y % 100 != 0 or y % 400 == 0) else _DAYS[mo - 1]
            if 1 <= d <= dim:
                return datetime(y, mo, d, hh, mi, ss)
    return _dparser.parse(s)


_EPOCH_NAIVE = datetime(1970, 1, 1)


class Dates:
    """The parsed article dates of a native chunk's rows (ingest.NativeChunk.dates): a sequence of naive
    ``datetime`` / ``None`` / dateutil results like the list ``[parse_date(str(v)) if notna(v) else None]``,
    held as arrays for the rows of the dataset's layout (kind 1: epoch µs, naive read as UTC; kind 2: None)
    and as objects for the others (kind 0: ``slow[row]``, dateutil's result).  ``epoch_us_arrays`` and
    ``utc_stamps`` give the write path integer forms without building a ``datetime`` per row."""

    __slots__ = ('us', 'kind', 'slow')

    def __init__(self, us, kind, slow):
        self.us, self.kind, self.slow = us, kind, slow

    def __len__(self):
        return len(self.kind)

    def __getitem__(self, i):
        k = self.kind[i]
        if k == 1:
            return _EPOCH_NAIVE + timedelta(microseconds=int(self.us[i]))
        if k == 2:
            return None
        return self.slow[int(i)]

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def epoch_us_arrays(self):
        """(epoch µs int64[n], has-date uint8[n]) as kb.epoch_us gives them (naive = UTC); raises TypeError
        for a date whose tzinfo has no UTC offset, as epoch_us does."""
        from .kb import epoch_us
        import numpy as np
        us = np.array(self.us, dtype=np.int64, copy=True)
        ok = (self.kind != 2).astype(np.uint8)
        for r, d in self.slow.items():
            us[r] = epoch_us(d)
        return us, ok

    def utc_stamps(self, rows):
        """``(stamps, k, exc)``: ``int(d.timestamp())`` of the given rows' dates when the process's local time
        zone is UTC (a naive datetime's timestamp() reads it in local time, match_keywords.py:131-132), else
        ``None``.  Rows of the dataset's layout take their epoch seconds; the others call timestamp(), and the
        first of them that raises (e.g. a year-1 date) stops there: ``k`` is its index in ``rows`` and ``exc``
        the exception (``k = len(rows)``, ``exc = None`` when none raises; ``stamps[:k]`` are valid)."""
        import numpy as np
        if not local_zone_is_utc():
            return None
        rows = np.asarray(rows, dtype=np.int64)
        out = self.us[rows] // 1000000
        for j in np.flatnonzero(self.kind[rows] != 1).tolist():
            try:
                out[j] = int(self[int(rows[j])].timestamp())
            except Exception as exc:   # noqa: BLE001 - the reference's append_to_csv raises here (:131-132)
                return out, j, exc
        return out, len(rows), None


def local_zone_is_utc() -> bool:
    """The process's local time zone is UTC without transitions (``time.timezone == time.altzone == 0``, no
    DST, zone name UTC/UCT/GMT): then a naive datetime's ``timestamp()`` equals its epoch seconds read as UTC.
    Checked on every call (TZ may change with ``time.tzset``)."""
    import time
    return (time.timezone == 0 and time.altzone == 0 and not time.daylight and
            time.tzname[0] in ('UTC', 'UCT', 'GMT', 'Etc/UTC', 'Universal', 'Zulu'))
