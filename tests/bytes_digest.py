"""Order-independent digests of a keep-first result over URL rows (test infrastructure, config 5).

Used by tests/golden/make_c5_digest.py (CPU oracle, numpy) and tests/test_gpu_dedup.py (the GPU's kept
rows, torch on the device for the per-byte work, numpy for the final mix), so both sides compute the
same numbers from the same formulas:

* ``row_digest``   = sum over kept rows r of mix64(r + K_ROW)                         (mod 2^64)
* ``bytes_digest`` = sum over kept rows of mix64(bytehash(url) + len(url) * K_LEN)   (mod 2^64)

``bytehash(u)`` = sum_j (u[j] + 1) * W[j] mod 2^64, W[j] = mix64(j + K_POS): a position-weighted byte sum,
so it vectorises as one gather + multiply + segment sum.
"""
from __future__ import annotations

import numpy as np

K_ROW = np.uint64(0x9E3779B97F4A7C15)
K_LEN = np.uint64(0xD6E8FEB86659FD93)
K_POS = np.uint64(0x632BE59BD9B4E019)
MAX_LEN = 1 << 16


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64's finaliser over a uint64 array (wrapping)."""
    x = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over='ignore'):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


_W = None


def weights() -> np.ndarray:
    global _W
    if _W is None:
        with np.errstate(over='ignore'):
            _W = mix64(np.arange(MAX_LEN, dtype=np.uint64) + K_POS)
    return _W


def bytehash_np(arena: np.ndarray, off: np.ndarray) -> np.ndarray:
    """bytehash of rows arena[off[i]:off[i+1]] (uint8 arena, int64 offsets) -> uint64[n]."""
    off = np.asarray(off, dtype=np.int64)
    n = len(off) - 1
    lens = np.diff(off)
    assert n == 0 or lens.max() < MAX_LEN
    total = int(off[-1] - off[0])
    out = np.zeros(n, np.uint64)
    if total == 0:
        return out
    b = arena[off[0]:off[-1]].astype(np.uint64) + np.uint64(1)
    pos = np.arange(total, dtype=np.int64) - np.repeat(off[:-1] - off[0], lens)
    with np.errstate(over='ignore'):
        prod = b * weights()[pos]
        nz = lens > 0
        starts = (off[:-1] - off[0])[nz]
        out[nz] = np.add.reduceat(prod, starts)
    return out


def row_value(bh: np.ndarray, lens: np.ndarray) -> np.ndarray:
    with np.errstate(over='ignore'):
        return mix64(np.asarray(bh, np.uint64) + np.asarray(lens, np.uint64) * K_LEN)


def row_digest(rows: np.ndarray) -> int:
    with np.errstate(over='ignore'):
        return int(mix64(np.asarray(rows, np.uint64) + K_ROW).sum(dtype=np.uint64))


def bytes_digest(bh: np.ndarray, lens: np.ndarray) -> int:
    with np.errstate(over='ignore'):
        return int(row_value(bh, lens).sum(dtype=np.uint64))


def bytehash_torch(dbytes, doff, lo: int, hi: int, w_dev):
    """bytehash of kept rows [lo, hi) of a dense device layout (uint8 bytes, int64 offsets) on the device:
    int64 tensor whose bits equal bytehash_np's uint64 values.  ``w_dev`` = torch.from_numpy(weights()
    .view(np.int64)) on the device."""
    import torch
    o = doff[lo:hi + 1]
    lens = o[1:] - o[:-1]
    b0, b1 = int(o[0]), int(o[-1])
    out = torch.zeros(hi - lo, dtype=torch.int64, device=dbytes.device)
    if b1 == b0:
        return out
    rid = torch.repeat_interleave(torch.arange(hi - lo, device=dbytes.device), lens)
    pos = torch.arange(b1 - b0, device=dbytes.device, dtype=torch.int64) - (o[:-1] - b0)[rid]
    prod = (dbytes[b0:b1].to(torch.int64) + 1) * w_dev[pos]
    out.index_add_(0, rid, prod)
    return out


# ------------------------------------------------------------------ CSV rows (north_star's hit CSV, config 3)
K_TICKER = np.uint64(0xA0761D6478BD642F)
K_DOC = np.uint64(0xE7037ED1A0B428DB)


def line_values(bh: np.ndarray, lens: np.ndarray, ticker: np.ndarray, doc: np.ndarray) -> np.ndarray:
    """Per output row: mix64(bytehash(line) + len * K_LEN + ticker * K_TICKER + doc * K_DOC), where
    ``ticker`` is the row's file's position in the KB's ticker order and ``doc`` the article's global index."""
    with np.errstate(over='ignore'):
        return mix64(np.asarray(bh, np.uint64) + np.asarray(lens, np.uint64) * K_LEN +
                     np.asarray(ticker, np.uint64) * K_TICKER + np.asarray(doc, np.uint64) * K_DOC)


def block_sums(values: np.ndarray, doc: np.ndarray, lo: int, n_blocks: int, per_block: int):
    """(wrapping uint64 sum, count) of ``values`` per ``per_block``-document block, blocks from doc ``lo``."""
    b = (np.asarray(doc, np.int64) - lo) // per_block
    dig = np.zeros(n_blocks, np.uint64)
    with np.errstate(over='ignore'):
        np.add.at(dig, b, np.asarray(values, np.uint64))
    return dig, np.bincount(b, minlength=n_blocks).astype(np.int64)
