"""ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker (or as the timed CPU port).  The
product (advanced_scrapper_amd/) never imports it.

CPU restatement of the reference's per-article matching (lwowlwowl/
advanced_scrapper match_keywords.py), written independently of the product:

* ``in_period``            <- is_within_period, match_keywords.py:17-37
* ``name_class``           <- the branch taken at :165-174
* ``field_results``        <- :155-156, :165-180 for one string
                              (``\\b`` literal via CPython ``re``; the fuzzy
                              decision via oracle/partial_ratio.c; positions via
                              ``re.finditer(name, s)``)
* ``ticker_matches``       <- :149-187 for one article

Parity status: pinned against tests/golden/ (fixtures produced by running the
reference's own match_keywords.py in the build container, see
tests/golden/make_golden.py) for everything except rapidfuzz, whose
partial_ratio is restated from its published algorithm (oracle/partial_ratio.c;
"parity unpinned" at that boundary).
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
from typing import Dict, List, Optional, Sequence

import numpy as np
from dateutil.tz import tzutc

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'build', 'libkworacle.so')

_LIB = None


def build() -> str:
    """Compile oracle/partial_ratio.c (make)."""
    subprocess.run(['make', '-s', '-C', HERE], check=True)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        for fn in (L.pr_score_brute, L.pr_score_fast):
            fn.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int]
            fn.restype = ctypes.c_double
        L.pr_decide.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int]
        L.pr_decide.restype = ctypes.c_int
        L.pr_decide_many.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int, vp]
        L.pr_decide_many.restype = None
        _LIB = L
    return _LIB


def _cps(s: str) -> np.ndarray:
    return np.frombuffer(s.encode('utf-32-le', 'surrogatepass'), dtype=np.uint32)


def partial_ratio_score(s1: str, s2: str, brute: bool = False) -> float:
    """rapidfuzz.fuzz.partial_ratio(s1, s2) restated (float score)."""
    a, b = _cps(s1), _cps(s2)
    f = lib().pr_score_brute if brute else lib().pr_score_fast
    return f(a.ctypes.data, len(a), b.ctypes.data, len(b))


def partial_ratio_gt95(s1: str, s2: str) -> bool:
    a, b = _cps(s1), _cps(s2)
    return bool(lib().pr_decide(a.ctypes.data, len(a), b.ctypes.data, len(b)))


class NameSet:
    """Fuzzy-class names packed once for pr_decide_many."""

    def __init__(self, names: Sequence[str]):
        self.names = list(names)
        arrs = [_cps(n) for n in self.names]
        self.off = np.zeros(len(arrs) + 1, dtype=np.int64)
        np.cumsum([len(a) for a in arrs], out=self.off[1:])
        self.cps = np.concatenate(arrs) if arrs else np.zeros(1, np.uint32)
        if self.cps.size == 0:
            self.cps = np.zeros(1, np.uint32)

    def decide(self, text: str) -> np.ndarray:
        t = _cps(text)
        out = np.zeros(len(self.names), dtype=np.uint8)
        tt = t if t.size else np.zeros(1, np.uint32)
        lib().pr_decide_many(tt.ctypes.data, len(t), self.cps.ctypes.data, self.off.ctypes.data, len(self.names),
                             out.ctypes.data)
        return out.astype(bool)


# ------------------------------------------------------------------ reference rules
def in_period(article_date, start, end) -> bool:
    """match_keywords.py:17-37."""
    if article_date is None:
        return False
    z = tzutc()
    a = article_date if article_date.tzinfo is not None else article_date.replace(tzinfo=z)
    s = None if not start else (start if start.tzinfo is not None else start.replace(tzinfo=z))
    e = None if not end else (end if end.tzinfo is not None else end.replace(tzinfo=z))
    if s is not None and e is not None:
        return s <= a <= e
    if s is not None:
        return s <= a
    if e is not None:
        return a <= e
    return True


def name_class(name: str) -> str:
    """'U' (\\b literal), 'X'/'S' (never match) or 'F' (fuzzy) — match_keywords.py:165-174."""
    if name.isupper():
        return 'U' if len(name) > 1 else 'X'
    if name.islower() and name.replace(' ', '').isalpha():
        return 'S'
    return 'F'


def upper_positions(name: str, s: str) -> List[int]:
    # the pattern is the escaped literal between two \b: no match without the literal as a substring
    if name not in s:
        return []
    return [m.start() for m in re.finditer(r'\b' + re.escape(name) + r'\b', s)]


def regex_positions(name: str, s: str) -> List[int]:
    return [m.start() for m in re.finditer(name, s)]


class Oracle:
    """Per-string results for every active name of a processed KB dict."""

    def __init__(self, processed_data: Dict):
        self.processed = processed_data
        seen = {}
        for _t, attrs in processed_data.items():
            for _a, names in attrs.items():
                for name in names:
                    if name not in seen:
                        seen[name] = name_class(name)
        self.upper = [n for n, c in seen.items() if c == 'U']
        self.fuzzy = [n for n, c in seen.items() if c == 'F']
        self.fset = NameSet(self.fuzzy)

    def field_results(self, s: str) -> Dict[str, Optional[List[int]]]:
        """name -> positions for every name whose branch adds a key for string s.

        U names appear only with a non-empty position list (:170-173); fuzzy
        names appear whenever partial_ratio > 95, possibly with [] (:177-180).
        """
        out: Dict[str, List[int]] = {}
        for n in self.upper:
            pos = upper_positions(n, s)
            if pos:
                out[n] = pos
        dec = self.fset.decide(s)
        for n, d in zip(self.fuzzy, dec):
            if d:
                out[n] = regex_positions(n, s)
        return out

    def ticker_matches(self, article_text: str, title: str, article_date) -> Dict:
        """match_keywords.py:149-187 for one article (strings already str()-ed)."""
        if article_date is None:
            return {}
        text_r = self.field_results(article_text)
        title_r = self.field_results(title)
        result = {}
        for ticker, attrs in self.processed.items():
            tm, ti = {}, {}
            for _attr, names in attrs.items():
                for name, (start, end) in names.items():
                    # the period test only decides names that matched a field; skipping it for the others
                    # changes nothing (it has no side effects and cannot raise on aware/naive datetimes)
                    if name not in text_r and name not in title_r:
                        continue
                    if not in_period(article_date, start, end):
                        continue
                    if name in text_r:
                        tm[name] = text_r[name]
                    if name in title_r:
                        ti[name] = title_r[name]
            if tm or ti:
                result[ticker] = {'text': tm, 'title': ti}
        return result
