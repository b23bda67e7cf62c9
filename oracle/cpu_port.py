"""ORACLE — CPU port timed as bench.py's ``cpu_baseline`` (test infrastructure only).

The reference's matching run the way the reference runs it
(match_keywords.py:148-192 per row, :230-238 for the pool): the rows are split
into ``procs`` sub-chunks (``np.array_split``) and a process pool runs, per
article, the triple loop ticker -> attribute -> name occurrence with
``is_within_period`` on every occurrence, ``re.finditer`` of the ``\\b``
pattern for uppercase names, the two ``partial_ratio(...) > 95`` decisions for
every fuzzy-class occurrence, ``re.finditer(name, s)`` on a fuzzy hit, and one pandas ``DataFrame([row]).to_csv(mode='a')`` append per
matched (article, ticker) into a scratch directory (:128-146).  Pool start-up
is excluded.  rapidfuzz is absent from the image, so its C work is stood in
for by the oracle's C restatement (oracle/partial_ratio.c) run once per field
over the distinct fuzzy names (``pr_decide_many``); the per-occurrence loop
then looks the decision up.  (Calling the restatement once per occurrence, as
the reference calls rapidfuzz, measured ~235 ms per article per core here --
slower than rapidfuzz is believed to be, so it would flatter the GPU.)
"""
from __future__ import annotations

import multiprocessing as mp
import os
import re
import shutil
import tempfile
import time
from typing import Sequence, Tuple

import numpy as np

_STATE = {}


def _init(processed):
    from oracle import kwmatch_oracle as orc
    _STATE['processed'] = processed
    _STATE['orc'] = orc
    _STATE['oracle'] = orc.Oracle(processed)
    _STATE['dir'] = tempfile.mkdtemp(prefix='kw_cpu_port_')


def _append(ticker, matched, row):
    """append_to_csv (match_keywords.py:128-146) into the worker's scratch directory."""
    import json
    import pandas as pd
    from dateutil import parser
    path = os.path.join(_STATE['dir'], f'{ticker}_match.csv')
    text, title, date_s = row
    rec = {'time_unix': int(parser.parse(date_s).timestamp()), 'date_time': date_s,
           'text_matches': json.dumps(matched['text']), 'title_matches': json.dumps(matched['title']),
           'title': title, 'url': '', 'source': '', 'source_url': '', 'article_text': text}
    pd.DataFrame([rec]).to_csv(path, mode='a', header=not os.path.exists(path), index=False)


def _article(text, title, date_s):
    from dateutil import parser
    orc = _STATE['orc']
    article_date = parser.parse(date_s)
    O = _STATE['oracle']
    fz_a = dict(zip(O.fuzzy, O.fset.decide(text)))     # partial_ratio(text, name) > 95, one C pass
    fz_b = dict(zip(O.fuzzy, O.fset.decide(title)))
    ticker_matches = {}
    for ticker, attrs in _STATE['processed'].items():
        tm, ti = {}, {}
        for _attr, names in attrs.items():
            for name, (start, end) in names.items():
                if not orc.in_period(article_date, start, end):
                    continue
                if name.isupper():
                    if len(name) > 1:
                        pat = r'\b' + re.escape(name) + r'\b'
                        a = [x.start() for x in re.finditer(pat, text)]
                        b = [x.start() for x in re.finditer(pat, title)]
                        if a:
                            tm[name] = a
                        if b:
                            ti[name] = b
                elif not (name.islower() and name.replace(' ', '').isalpha()):
                    hit_a = fz_a[name]
                    hit_b = fz_b[name]
                    if hit_a:
                        tm[name] = [x.start() for x in re.finditer(name, text)]
                    if hit_b:
                        ti[name] = [x.start() for x in re.finditer(name, title)]
        if tm or ti:
            ticker_matches[ticker] = {'text': tm, 'title': ti}
    for ticker, matched in ticker_matches.items():
        _append(ticker, matched, (text, title, date_s))
    return len(ticker_matches)


def _run(rows):
    n = 0
    for text, title, date_s in rows:
        _article(text, title, date_s)
        n += 1
    return n


def _cleanup(_):
    shutil.rmtree(_STATE.get('dir', ''), ignore_errors=True)
    return 0


def _reset(_):
    """Empty the worker's scratch directory between timed runs (the next run appends from scratch)."""
    d = _STATE.get('dir', '')
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d, exist_ok=True)
    return 0


def time_port(processed, rows: Sequence[Tuple[str, str, str]], procs: int, runs: int = 1):
    """Wall seconds to match `rows` ((text, title, date string)) with `procs` worker processes: (seconds, rows
    done) for runs = 1, else (the `runs` wall times, rows done) -- every run over the same rows in the same
    warm pool."""
    ctx = mp.get_context('spawn')
    with ctx.Pool(procs, initializer=_init, initargs=(processed,)) as pool:
        pool.map(_run, [[] for _ in range(procs)])           # warm the workers (imports, KB)
        parts = [list(p) for p in np.array_split(np.arange(len(rows)), procs)]
        subs = [[rows[i] for i in p] for p in parts]
        times = []
        for r in range(max(1, runs)):
            if r:
                pool.map(_reset, range(procs))
            t0 = time.perf_counter()
            done = sum(pool.map(_run, subs))
            times.append(time.perf_counter() - t0)
        pool.map(_cleanup, range(procs))
        return (times[0] if runs == 1 else times), done
