"""Run the CPU oracle over many strings in a spawn-based process pool.

Spawn (not fork) so that no worker inherits a HIP context from a test process
that already touched the GPU.  Workers only import oracle/ (no torch).
"""
from __future__ import annotations

import multiprocessing as mp
import os
from typing import Dict, List, Optional, Sequence

_ORACLE = None


def _init(processed):
    global _ORACLE
    from oracle import kwmatch_oracle as orc
    _ORACLE = orc.Oracle(processed)


def _field(s: str):
    return _ORACLE.field_results(s)


def _ticker(args):
    text, title, date = args
    return _ORACLE.ticker_matches(text, title, date)


def workers() -> int:
    return max(1, min(16, (os.cpu_count() or 2)))


def field_results(processed, strings: Sequence[str], procs: Optional[int] = None) -> List[Dict]:
    ctx = mp.get_context('spawn')
    with ctx.Pool(procs or workers(), initializer=_init, initargs=(processed,)) as pool:
        return pool.map(_field, list(strings), chunksize=8)


def ticker_matches(processed, rows, procs: Optional[int] = None) -> List[Dict]:
    ctx = mp.get_context('spawn')
    with ctx.Pool(procs or workers(), initializer=_init, initargs=(processed,)) as pool:
        return pool.map(_ticker, list(rows), chunksize=8)
