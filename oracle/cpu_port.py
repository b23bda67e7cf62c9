"""ORACLE — CPU port timed as bench.py's ``cpu_baseline`` (test infrastructure only).

The reference's own driver shape (match_keywords.py:230-238): the chunk is
split into ``n`` sub-chunks (``np.array_split``) and a process pool runs the
per-article loop on each.  The per-article loop is the oracle's restatement
(oracle/kwmatch_oracle.py: CPython ``re`` for the uppercase branch, the C
restatement of rapidfuzz partial_ratio for the fuzzy branch).  It is kinder
to the CPU than the reference: it decides each distinct name once per field
instead of once per (ticker, attribute) occurrence and it skips the per-hit
pandas CSV appends.
"""
from __future__ import annotations

import multiprocessing as mp
import time
from typing import List, Sequence, Tuple

import numpy as np

_ORACLE = None


def _init(processed):
    global _ORACLE
    from oracle.kwmatch_oracle import Oracle
    _ORACLE = Oracle(processed)


def _run(rows):
    n = 0
    for text, title, date in rows:
        _ORACLE.ticker_matches(text, title, date)
        n += 1
    return n


def time_port(processed, rows: Sequence[Tuple[str, str, object]], procs: int) -> Tuple[float, int]:
    """Wall seconds to match `rows` with `procs` worker processes (pool start-up excluded)."""
    ctx = mp.get_context('spawn')
    with ctx.Pool(procs, initializer=_init, initargs=(processed,)) as pool:
        pool.map(_run, [[] for _ in range(procs)])           # warm the workers (imports, KB)
        parts = [list(p) for p in np.array_split(np.arange(len(rows)), procs)]
        subs = [[rows[i] for i in p] for p in parts]
        t0 = time.perf_counter()
        done = sum(pool.map(_run, subs))
        return time.perf_counter() - t0, done
