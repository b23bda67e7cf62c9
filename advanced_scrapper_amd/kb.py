"""Knowledge-base loading, name classification and pattern compilation.

Host side of the matching path.  The loaders restate the reference's
knowledge-base functions with the same names, arguments, ordering rules and
error behaviour:

* ``extract_time_periods``        match_keywords.py:40-65
* ``process_json_data``           match_keywords.py:68-87
* ``read_and_process_json_files`` match_keywords.py:90-120
* ``is_within_period``            match_keywords.py:17-37

``compile_kb`` then turns the loaded dict into the pattern table handed to
``kw_compile`` (include/kwmatch.h): every distinct name of the two classes
that can ever match (match_keywords.py:165-174) becomes one pattern, and every
(ticker, attribute, name) occurrence is kept on the host for the period
filter and the per-ticker dict assembly (match_keywords.py:159-187).
"""
from __future__ import annotations

import json
import os
import re
from dataclasses import dataclass, field
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
from dateutil import parser as _dtparser
from dateutil.tz import tzutc

try:  # Python <= 3.10
    import sre_constants as _sre_c
    import sre_parse as _sre_p
except ImportError:  # pragma: no cover - Python >= 3.11
    from re import _constants as _sre_c  # type: ignore
    from re import _parser as _sre_p  # type: ignore

# Attribute order of one company record (match_keywords.py:76-85).
ATTRIBUTES = ('id_label', 'ticker', 'aliases', 'products', 'subsidiaries',
              'owned_entities', 'ceos', 'board_members')

# The reference prints every ticker and the whole merged dict while loading
# (match_keywords.py:73, :86, :92).  Off by default; set True for identical
# stdout.
PRINT_LIKE_REFERENCE = False


# --------------------------------------------------------------------- a5
def is_within_period(article_date, start_date, end_date):
    """Inclusive period test (match_keywords.py:17-37).

    A missing article date never matches; naive datetimes are taken as UTC;
    a missing bound is open.
    """
    if article_date is None:
        return False
    utc = tzutc()

    def aware(d):
        return d.replace(tzinfo=utc) if d.tzinfo is None else d

    a = aware(article_date)
    lo = aware(start_date) if start_date else None
    hi = aware(end_date) if end_date else None
    if lo is not None and hi is not None:
        return lo <= a <= hi
    if lo is not None:
        return lo <= a
    if hi is not None:
        return a <= hi
    return True


_EPOCH = datetime(1970, 1, 1, tzinfo=tzutc())
_OPEN_LO, _OPEN_HI = -(1 << 63), 1 << 63


def epoch_us(d) -> int:
    """The instant ``is_within_period`` compares, as integer microseconds since 1970 (naive = UTC).

    Exact for every datetime (timedelta arithmetic is integral), so ``lo <= a <= hi`` on these integers
    equals the aware-datetime comparison of match_keywords.py:31-37.  Raises ``TypeError`` for a tzinfo
    whose ``utcoffset`` is ``None`` (the reference's comparison raises for it too).
    """
    if d.tzinfo is None:
        d = d.replace(tzinfo=_EPOCH.tzinfo)
    td = d - _EPOCH
    return (td.days * 86400 + td.seconds) * 1000000 + td.microseconds


def period_us(start_date, end_date) -> Tuple[int, int]:
    """(lo, hi) integer bounds of one KB period; a missing (falsy) bound is open (match_keywords.py:26-30)."""
    return (epoch_us(start_date) if start_date else _OPEN_LO, epoch_us(end_date) if end_date else _OPEN_HI)


# --------------------------------------------------------------------- a1
def _period_bound(part: str, tag: str):
    text = part.replace(tag, "").replace("T00:00:00Z)", "").strip()
    try:
        return _dtparser.parse(text)
    except (ValueError, _dtparser.ParserError):
        return None


def extract_time_periods(names):
    """Ordered ``{name: (start, end)}`` from the KB strings (match_keywords.py:40-65).

    ``"Name (Start: 2001-01-01T00:00:00Z) (End: ...)"`` -> ``name``; a repeated
    name keeps its first position and takes the last period.
    """
    periods = {}
    if isinstance(names, str):
        names = [names]
    for entry in names:
        head, *tail = entry.split(" (")
        start = end = None
        for part in tail:
            if 'Start:' in part:
                start = _period_bound(part, "Start:")
            elif 'End:' in part:
                end = _period_bound(part, "End:")
        periods[head.strip()] = (start, end)
    return periods


# --------------------------------------------------------------------- a2
def process_json_data(json_data):
    """Per-ticker attribute dicts of one KB file (match_keywords.py:68-87).

    A company is kept when the file holds a single record or when
    ``'United States'`` is in its ``country``; a repeated ticker overwrites
    the earlier value but keeps its first position.
    """
    result = {}
    single = len(json_data) <= 1
    for company in json_data:
        if (not single and 'United States' in company['country']) or single:
            ticker = company['ticker']
            if PRINT_LIKE_REFERENCE:
                print(ticker)
            result[ticker] = {attr: extract_time_periods(company.get(attr, [])) for attr in ATTRIBUTES}
    if PRINT_LIKE_REFERENCE:
        print(result)
    return result


# --------------------------------------------------------------------- a3
def _load_kb_file(path: str, encoding: str):
    with open(path, 'r', encoding=encoding) as fh:
        return process_json_data(json.load(fh))


def read_and_process_json_files(folder_path, _listdir=None):
    """Merge every ``*.json`` KB file of ``folder_path`` (match_keywords.py:90-120).

    Files are visited in ``os.listdir`` order (``_listdir`` lets tests pin the
    order a fixture recorded).  Decoding falls back utf-8 -> gbk -> latin1;
    a file that still fails is reported and skipped, exactly as the reference
    does (including its quirk that an error other than UnicodeDecodeError
    during the gbk attempt propagates).
    """
    merged = {}
    if PRINT_LIKE_REFERENCE:
        print(folder_path)
    names = (_listdir or os.listdir)(folder_path)
    for filename in names:
        if not filename.endswith('.json'):
            continue
        path = os.path.join(folder_path, filename)
        try:
            merged.update(_load_kb_file(path, 'utf-8'))
        except UnicodeDecodeError:
            print(f"UTF-8解码失败，尝试其他编码读取文件: {filename}")   # ref :104
            try:
                merged.update(_load_kb_file(path, 'gbk'))
            except UnicodeDecodeError:
                try:
                    merged.update(_load_kb_file(path, 'latin1'))
                except Exception as exc:  # noqa: BLE001 - mirrors the reference
                    print(f"无法读取文件 {filename}: {exc}")   # ref :117
        except Exception as exc:  # noqa: BLE001 - mirrors the reference
            print(f"处理文件 {filename} 时出错: {exc}")   # ref :119
    return merged


# --------------------------------------------------------------------- a4
CLASS_UPPER = 'U'      # isupper and len > 1: \b literal search       (:165-173)
CLASS_SINGLE = 'X'     # isupper and len <= 1: never matches           (:166)
CLASS_LOWER = 'S'      # islower and alpha after removing spaces: never (:174)
CLASS_FUZZY = 'F'      # everything else: partial_ratio > 95           (:174-180)


def classify_name(name: str) -> str:
    """The branch match_keywords.py:165-174 takes for ``name``."""
    if name.isupper():
        return CLASS_UPPER if len(name) > 1 else CLASS_SINGLE
    if name.islower() and name.replace(' ', '').isalpha():
        return CLASS_LOWER
    return CLASS_FUZZY


# --------------------------------------------------------------------- regex atoms
_META = set('.^$*+?{}[]\\|()')
_DOT = {'.'}
RX_LIT, RX_ANY = 0, 1


class UnsupportedPattern(NotImplementedError):
    """A fuzzy-class name whose regex uses constructs the GPU matcher lacks."""


def regex_atoms(name: str):
    """Atom program for ``re.finditer(name, s)`` (match_keywords.py:178,180).

    Returns ``None`` when the name has no regex metacharacter (literal search),
    ``'invalid'`` when ``re.compile(name)`` raises (the reference then raises
    ``re.error`` the first time the name fuzzy-matches), or a list of
    ``(op, value, min, max)`` atoms.  Supported: literals, ``.``, greedy
    ``? * + {m,n}`` on a single literal or ``.``, and unquantified groups.
    Anything else raises :class:`UnsupportedPattern`.
    """
    meta = _META & set(name)
    if not meta:
        return None
    if meta == _DOT:
        # only '.': every other character is a literal (the sre_parse walk gives the same atoms, ~50x slower)
        return [(RX_ANY, 0, 1, 1) if ch == '.' else (RX_LIT, ord(ch), 1, 1) for ch in name]
    return regex_atoms_sre(name)


def regex_atoms_sre(name: str):
    """regex_atoms through sre_parse (any name with a metacharacter)."""
    try:
        parsed = _sre_p.parse(name)
    except re.error:
        return 'invalid'
    atoms: List[Tuple[int, int, int, int]] = []

    def single(op, av):
        if op is _sre_c.LITERAL:
            return (RX_LIT, int(av))
        if op is _sre_c.ANY:
            return (RX_ANY, 0)
        return None

    def walk(items):
        for op, av in items:
            s = single(op, av)
            if s is not None:
                atoms.append((s[0], s[1], 1, 1))
                continue
            if op is _sre_c.MAX_REPEAT:
                lo, hi, sub = av
                sub = list(sub)
                if len(sub) == 1:
                    s = single(*sub[0])
                    if s is not None:
                        hi_v = -1 if hi == _sre_c.MAXREPEAT else int(hi)
                        atoms.append((s[0], s[1], int(lo), hi_v))
                        continue
            if op is _sre_c.SUBPATTERN:
                _group, add_flags, del_flags, sub = av
                if not add_flags and not del_flags:
                    walk(sub)
                    continue
            raise UnsupportedPattern(f"regex construct {op} in KB name {name!r} is not supported by the GPU matcher")

    walk(parsed)
    if sum(a[2] for a in atoms) == 0:
        raise UnsupportedPattern(f"KB name {name!r} can match the empty string")
    return atoms


# --------------------------------------------------------------------- word table
_WORD_BITMAP: Optional[np.ndarray] = None


def word_bitmap() -> np.ndarray:
    """0x110000-bit table of CPython's ``\\b`` word class (isalnum() or '_')."""
    global _WORD_BITMAP
    if _WORD_BITMAP is None:
        # re's own word test (_sre: Py_UNICODE_ISALNUM(c) || c == '_', the \b of match_keywords.py:156) run
        # once over every code point in C: the same set as chr(c).isalnum() or c == '_', ~10x faster than a
        # Python loop over 0x110000 characters
        every = np.arange(0x110000, dtype='<u4').tobytes().decode('utf-32-le', 'surrogatepass')
        flags = np.zeros(0x110000, dtype=bool)
        flags[[m.start() for m in re.finditer(r'\w', every)]] = True
        _WORD_BITMAP = np.packbits(flags, bitorder='little').view(np.uint32).copy()
    return _WORD_BITMAP


# --------------------------------------------------------------------- compile
@dataclass
class CompiledKB:
    """Pattern table for kw_compile plus the host-side occurrence index."""

    tickers: List[str]
    names: List[str]                       # pattern id -> name
    classes: List[str]                     # 'U' / 'F'
    pat_bytes: np.ndarray                  # uint8
    pat_off: np.ndarray                    # int64, n+1
    pat_class: np.ndarray                  # uint8
    rx_atoms: np.ndarray                   # int32 [n_atoms, 4]
    rx_off: np.ndarray                     # int64, n+1
    invalid_regex: List[bool]
    # occurrences[pid] = list of (ticker index, traversal rank, start, end)
    occurrences: List[List[Tuple[int, int, object, object]]] = field(default_factory=list)
    n_occurrences: int = 0

    @property
    def n_patterns(self) -> int:
        return len(self.names)

    def occurrences_us(self) -> Optional[List[List[Tuple[int, int, int, int]]]]:
        """``occurrences`` with the periods as integer µs bounds (built once), or ``None`` when a bound has no
        UTC offset and only the datetime comparison can decide."""
        cached = self.__dict__.get('_occ_us', False)
        if cached is False:
            try:
                cached = [[(ti, rank) + period_us(lo, hi) for (ti, rank, lo, hi) in occ] for occ in self.occurrences]
            except TypeError:
                cached = None
            self.__dict__['_occ_us'] = cached
        return cached


PAR_MIN_REGEX = 65536  # regex-bearing names from which compile_kb parses the programs in worker processes
                       # (process start-up costs ~1 s: a 52k-name KB parses faster in one process)


def _atoms_of(names: List[str]):
    """Worker: regex_atoms of each name (UnsupportedPattern propagates to the caller)."""
    return [regex_atoms(n) for n in names]


def regex_programs(names: List[str], fuzzy: List[bool], workers: Optional[int] = None) -> list:
    """regex_atoms of every fuzzy-class name (None for the others), in order.  Only names with a regex
    metacharacter need sre_parse; from PAR_MIN_REGEX of them (a Wikidata-scale KB, config 4) they are
    parsed by ``workers`` spawned processes (default min(16, os.cpu_count())) in contiguous chunks, so
    the first unsupported name in KB order is the one reported, as in the serial loop."""
    progs: list = [None] * len(names)
    todo = [i for i, n in enumerate(names) if fuzzy[i] and (_META & set(n))]
    if workers is None:
        workers = min(16, os.cpu_count() or 1)
    if workers > 1 and len(todo) >= PAR_MIN_REGEX:
        import multiprocessing
        from concurrent.futures import ProcessPoolExecutor
        k = min(workers, max(1, len(todo) // 1024))
        bounds = [len(todo) * j // k for j in range(k + 1)]
        chunks = [todo[bounds[j]:bounds[j + 1]] for j in range(k)]
        with ProcessPoolExecutor(k, mp_context=multiprocessing.get_context('spawn')) as ex:
            futs = [ex.submit(_atoms_of, [names[i] for i in ch]) for ch in chunks]
            for ch, fut in zip(chunks, futs):
                for i, prog in zip(ch, fut.result()):
                    progs[i] = prog
    else:
        for i in todo:
            progs[i] = regex_atoms(names[i])
    return progs


def compile_kb(processed_data: Dict[str, Dict[str, Dict[str, tuple]]], workers: Optional[int] = None) -> CompiledKB:
    """Patterns of the active names in the reference's traversal order.

    The traversal ticker -> attribute -> name (match_keywords.py:159-163)
    assigns every occurrence a rank; a name's dict position inside a ticker's
    ``text_matches``/``title_matches`` is the rank of its first in-period
    occurrence there.  Patterns are ordered for the device: uppercase names
    first, then fuzzy names by decreasing code-point length (stable).  The
    regex programs of a large KB are parsed in parallel (regex_programs).
    """
    tickers = list(processed_data.keys())
    first_seen: Dict[str, int] = {}
    occ_by_name: Dict[str, list] = {}
    cls_of: Dict[str, str] = {}
    rank = 0
    for ti, ticker in enumerate(tickers):
        for _attr, names in processed_data[ticker].items():
            for name, (start, end) in names.items():
                cls = cls_of.get(name)
                if cls is None:
                    cls = cls_of[name] = classify_name(name)
                if cls in (CLASS_UPPER, CLASS_FUZZY):
                    if name not in first_seen:
                        first_seen[name] = len(first_seen)
                        occ_by_name[name] = []
                    occ_by_name[name].append((ti, rank, start, end))
                rank += 1
    uniq = list(first_seen.keys())
    upper = [n for n in uniq if cls_of[n] == CLASS_UPPER]
    fuzzy = [n for n in uniq if cls_of[n] == CLASS_FUZZY]
    fuzzy.sort(key=lambda n: -len(n))
    ordered = upper + fuzzy
    enc = [n.encode('utf-8', 'surrogatepass') for n in ordered]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    pat_off = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=pat_off[1:])
    pat_bytes = np.frombuffer(b''.join(enc), dtype=np.uint8).copy() if enc else np.zeros(0, np.uint8)
    classes = [cls_of[n] for n in ordered]
    pat_class = np.frombuffer(''.join(classes).encode('ascii'), dtype=np.uint8).copy()
    atoms: List[Tuple[int, int, int, int]] = []
    rx_off = np.zeros(len(ordered) + 1, dtype=np.int64)
    invalid = []
    progs = regex_programs(ordered, [c == CLASS_FUZZY for c in classes], workers)
    for i, prog in enumerate(progs):
        rx_off[i] = len(atoms)
        invalid.append(prog == 'invalid')
        if isinstance(prog, list):
            atoms.extend(prog)
    rx_off[len(ordered)] = len(atoms)
    rx = np.asarray(atoms, dtype=np.int32).reshape(-1, 4) if atoms else np.zeros((0, 4), np.int32)
    return CompiledKB(
        tickers=tickers, names=ordered, classes=classes, pat_bytes=pat_bytes, pat_off=pat_off,
        pat_class=pat_class, rx_atoms=rx, rx_off=rx_off, invalid_regex=invalid,
        occurrences=[occ_by_name[n] for n in ordered], n_occurrences=rank)
