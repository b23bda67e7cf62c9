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
from datetime import datetime

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
