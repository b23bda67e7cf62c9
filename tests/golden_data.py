"""Loaders for the committed golden fixtures (tests/golden/, see make_golden.py)."""
from __future__ import annotations

import functools
import gzip
import io
import json
import os
import tarfile
from datetime import datetime
from typing import Dict, List

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _read(name: str) -> bytes:
    with open(os.path.join(HERE, name), 'rb') as fh:
        return fh.read()


@functools.lru_cache(maxsize=None)
def kb_bundle() -> dict:
    return json.loads(gzip.decompress(_read('kb_bundle.json.gz')))


def materialize_kb(dst: str) -> List[str]:
    """Write the KB files to dst; returns the reference's os.listdir order."""
    b = kb_bundle()
    os.makedirs(dst, exist_ok=True)
    for fn, text in b['files'].items():
        with open(os.path.join(dst, fn), 'wb') as fh:
            fh.write(text.encode('utf-8'))
    return list(b['listdir'])


def _dt(s):
    return None if s is None else datetime.fromisoformat(s)


@functools.lru_cache(maxsize=None)
def _kb_processed_raw():
    return json.loads(gzip.decompress(_read('kb_processed.json.gz')))


def processed_from(kb_list) -> Dict:
    """processed_data from its JSON form ([[ticker, [[attr, [[name, start, end], ...]], ...]], ...])."""
    out = {}
    for ticker, attrs in kb_list:
        out[ticker] = {a: {n: (_dt(s), _dt(e)) for n, s, e in names} for a, names in attrs}
    return out


def kb_processed() -> Dict:
    """The reference's processed_data, rebuilt with datetime periods."""
    return processed_from(_kb_processed_raw())


@functools.lru_cache(maxsize=None)
def error_cases() -> dict:
    """tests/golden/error_golden.json.gz (make_error_golden.py): the reference's partial outputs."""
    return json.loads(gzip.decompress(_read('error_golden.json.gz')))


def articles_csv_bytes() -> bytes:
    return gzip.decompress(_read('articles.csv.gz'))


def articles_frame():
    import pandas as pd
    return pd.read_csv(io.BytesIO(articles_csv_bytes()))


@functools.lru_cache(maxsize=None)
def matches() -> List[dict]:
    return [json.loads(l) for l in gzip.decompress(_read('matches.jsonl.gz')).decode().split('\n')]


@functools.lru_cache(maxsize=None)
def outputs() -> Dict[str, bytes]:
    out = {}
    with tarfile.open(fileobj=io.BytesIO(_read('out_c1.tar.gz')), mode='r:gz') as tar:
        for m in tar.getmembers():
            out[m.name] = tar.extractfile(m).read()
    return out


def manifest() -> dict:
    return json.loads(_read('MANIFEST.json'))


def chunksize() -> int:
    return int(manifest()['chunksize'])
