"""Per-document digests of hit records (test infrastructure).

A hit record is kw_scan's ``(doc, pattern, pos, field)`` (uint32 each; ``pos``
= KW_NOPOS for a fuzzy match without a regex position).  ``record_mix`` is the
record hash of bench.hits_digest; a document's digest is the wrapping uint64
sum of its records' mixes, so the sum over all documents is the bench line's
``hits_digest`` and any sharding or record order gives the same numbers.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List

import numpy as np

NOPOS = 0xFFFFFFFF
_K = [np.uint64(0x9E3779B97F4A7C15), np.uint64(0x2545F4914F6CDD1D), np.uint64(0x27D4EB2F165667C5),
      np.uint64(0x165667B19E3779F9)]
_M = np.uint64((-0x40A7B892E31B1A47) & 0xFFFFFFFFFFFFFFFF)


def record_mix(doc, pat, pos, field) -> np.ndarray:
    """uint64 mix of records given as four uint32-valued arrays (bench.hits_digest's formula)."""
    with np.errstate(over='ignore'):
        x = (np.asarray(doc, np.uint64) * _K[0] + np.asarray(pat, np.uint64) * _K[1] +
             np.asarray(pos, np.uint64) * _K[2] + np.asarray(field, np.uint64) * _K[3])
        x ^= x >> np.uint64(31)
        x *= _M
        x ^= x >> np.uint64(29)
    return x


def per_doc(rec: np.ndarray, n_docs: int, doc_base: int = 0):
    """(digest uint64[n_docs], count int64[n_docs]) of structured HIT_DTYPE records whose ``doc`` ids are
    global (``doc_base`` = the first document)."""
    doc = rec['doc'].astype(np.int64) - doc_base
    mix = record_mix(rec['doc'], rec['pattern'], rec['pos'], rec['field'])
    dig = np.zeros(n_docs, np.uint64)
    if len(rec):
        order = np.argsort(doc, kind='stable')
        d, m = doc[order], mix[order]
        starts = np.flatnonzero(np.r_[True, d[1:] != d[:-1]])
        with np.errstate(over='ignore'):
            dig[d[starts]] = np.add.reduceat(m, starts)
    cnt = np.bincount(doc, minlength=n_docs).astype(np.int64)
    return dig, cnt


def total(dig: np.ndarray) -> str:
    with np.errstate(over='ignore'):
        return f'{int(dig.sum(dtype=np.uint64)):016x}'


def oracle_records(doc: int, fields: List[Dict[str, list]], pid: Dict[str, int]) -> List[tuple]:
    """kw_scan-shaped records of one document from the oracle's per-field ``name -> positions``."""
    out = []
    for f, res in enumerate(fields):
        for name, pos in res.items():
            p = pid[name]
            if pos:
                out += [(doc, p, q, f) for q in pos]
            else:
                out.append((doc, p, NOPOS, f))
    return out


def corpus_fingerprint(corpus) -> str:
    """blake2b of the corpus offsets and bytes (the generator must still produce the pinned documents)."""
    h = hashlib.blake2b(digest_size=16)
    h.update(np.ascontiguousarray(corpus.off - corpus.off[0]).tobytes())
    h.update(memoryview(corpus.arena[corpus.off[0]:corpus.off[-1]]))
    return h.hexdigest()
