"""Device matcher: arena packing, the libkwmatch handle, and result assembly.

Data flow of one batch of articles:

    str fields --pack_fields--> uint8 arena + int64 offsets (host)
               --torch--> HBM (caller-owned tensors)
               --kw_scan--> per-(doc, field, pattern) records in HBM
               --fetch--> numpy records --assemble_ticker_matches--> the
                  reference's ``ticker_matches`` dicts (match_keywords.py:183-187)

PyTorch is only used to own device memory and streams.
"""
from __future__ import annotations

import ctypes
import re
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from .kb import CompiledKB, compile_kb, epoch_us, is_within_period, word_bitmap

ARENA_PAD = 64   # bytes readable past the last field (kw_scan reads 16-B tiles)


# --------------------------------------------------------------------- packing
def field_str(value) -> str:
    """The reference's ``str(v) if v else ""`` (match_keywords.py:150-151)."""
    return str(value) if value else ""


def background_sample(texts: Sequence[str], limit: int = 4 << 20) -> bytes:
    """UTF-8 sample of article text for the anchor statistics (first `limit` bytes)."""
    out, n = [], 0
    for t in texts:
        b = t.encode('utf-8', 'surrogatepass')
        out.append(b)
        n += len(b) + 1
        if n >= limit:
            break
    return b'\n'.join(out)[:limit]


def pack_fields(texts: Sequence[str], titles: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    """Interleave text/title UTF-8 into one arena; offsets have 2n+1 entries."""
    n = len(texts)
    if len(titles) != n:
        raise ValueError("texts and titles differ in length")
    parts: List[bytes] = [b''] * (2 * n)
    for i in range(n):
        parts[2 * i] = texts[i].encode('utf-8', 'surrogatepass')
        parts[2 * i + 1] = titles[i].encode('utf-8', 'surrogatepass')
    lens = np.fromiter((len(p) for p in parts), dtype=np.int64, count=2 * n)
    off = np.zeros(2 * n + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    arena = np.zeros(int(off[-1]) + ARENA_PAD, dtype=np.uint8)
    if off[-1]:
        arena[:off[-1]] = np.frombuffer(b''.join(parts), dtype=np.uint8)
    return arena, off


# --------------------------------------------------------------------- device handle
class GpuMatcher:
    """One compiled knowledge base on one GPU (libkwmatch handle)."""

    def __init__(self, ckb: CompiledKB, device: Optional[int] = None, background: Optional[bytes] = None):
        """``background``: a sample of the article text whose 4-byte statistics
        price the anchor choice (speed only; results never depend on it).

        No torch is needed for the host-buffer methods (:meth:`scan_host`, :meth:`fetch_host`,
        :meth:`match_strings`); the device-tensor methods import it on first use."""
        import sys
        if _native.device_count() == 0:
            raise RuntimeError("GpuMatcher needs a ROCm GPU (no HIP device visible)")
        self.ckb = ckb
        if device is None:
            torch = sys.modules.get('torch')
            device = torch.cuda.current_device() if torch is not None and torch.cuda.is_initialized() else 0
        self.device = int(device)
        L = _native.lib()
        h = ctypes.c_void_p()
        rx = np.ascontiguousarray(ckb.rx_atoms, dtype=np.int32)
        wb = word_bitmap()
        bg = np.frombuffer(background, dtype=np.uint8) if background else np.zeros(0, np.uint8)
        rc = L.kw_compile(_native.ptr(ckb.pat_bytes), _native.ptr(ckb.pat_off), _native.ptr(ckb.pat_class),
                          ckb.n_patterns, _native.ptr(rx) if rx.size else None, _native.ptr(ckb.rx_off),
                          _native.ptr(wb), _native.ptr(bg) if bg.size else None, int(bg.size), self.device,
                          ctypes.byref(h))
        if rc != _native.KW_OK:
            msg = L.kw_last_error(h)
            if h.value:
                L.kw_destroy(h)
            raise _native.KwError(rc, msg.decode() if msg else '')
        self.h = h
        self._keep = None

    @property
    def torch(self):
        import torch
        return torch

    @classmethod
    def from_processed_data(cls, processed_data, device=None, background=None) -> "GpuMatcher":
        return cls(compile_kb(processed_data), device, background)

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            _native.lib().kw_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- device-resident inputs
    def upload(self, arena: np.ndarray, off: np.ndarray):
        t = self.torch
        dev = t.device('cuda', self.device)
        return (t.from_numpy(arena).to(dev, non_blocking=False), t.from_numpy(off).to(dev, non_blocking=False))

    def scan(self, d_arena, d_off, n_docs: int, stream=None) -> None:
        """Launch kw_scan on device tensors (asynchronous)."""
        if stream is None:
            stream = self.torch.cuda.current_stream(self.device)
        sp = ctypes.c_void_p(stream.cuda_stream) if hasattr(stream, 'cuda_stream') else ctypes.c_void_p(stream)
        self._keep = (d_arena, d_off)
        _native.check(_native.lib().kw_scan(self.h, _native.ptr(d_arena), _native.ptr(d_off), int(n_docs), sp), self.h)

    def n_hits(self) -> int:
        n = ctypes.c_int64()
        p = ctypes.c_void_p()
        _native.check(_native.lib().kw_hits(self.h, ctypes.byref(n), ctypes.byref(p)), self.h)
        return int(n.value)

    def hits_device(self):
        """Records of the last scan as a device tensor [n, 4] (uint32 viewed as int32)."""
        t = self.torch
        n = self.n_hits()
        out = t.empty((max(n, 1), 4), dtype=t.int32, device=t.device('cuda', self.device))
        cnt = ctypes.c_int64()
        st = t.cuda.current_stream(self.device)
        _native.check(_native.lib().kw_hits_copy(self.h, _native.ptr(out), n, ctypes.byref(cnt),
                                                 ctypes.c_void_p(st.cuda_stream)), self.h)
        return out[:n]

    def hits_copy_into(self, dst, stream=None) -> int:
        """Copy the last scan's records into the device tensor ``dst`` ([cap, 4] int32) on ``stream``
        (asynchronous); returns the record count."""
        t = self.torch
        st = stream if stream is not None else t.cuda.current_stream(self.device)
        cnt = ctypes.c_int64()
        _native.check(_native.lib().kw_hits_copy(self.h, _native.ptr(dst), int(dst.shape[0]), ctypes.byref(cnt),
                                                 ctypes.c_void_p(st.cuda_stream)), self.h)
        return int(cnt.value)

    def fetch(self) -> np.ndarray:
        """Records of the last scan on the host (structured HIT_DTYPE array)."""
        return records_from_tensor(self.hits_device())

    def doc_routes(self, n_docs: int) -> np.ndarray:
        """Per document of the last scan: which kernel finished it (_native.KW_ROUTE_*)."""
        out = np.zeros(max(n_docs, 1), dtype=np.uint8)
        _native.check(_native.lib().kw_doc_routes(self.h, _native.ptr(out), int(n_docs)), self.h)
        return out[:n_docs]

    STAT_KEYS = ('candidates', 'anchor_hits', 'lcs_windows', 'verifications', 'deferred_docs', 'deferred_items',
                 'deferred_long_nonascii', 'edge_items', 'candidates_stage2', 'resolved_docs', 'regex_searches',
                 'regex_backtracking', 'regex_rounds', 'deferred_long_run', 'deferred_item_caps', 'deferred_flagged',
                 'big_docs', 'rescans', 'transcoded_docs', 'resolve_fallback_docs', 'rescan_causes')

    def stats(self) -> Dict[str, int]:
        v = np.zeros(_native.KW_N_STATS, dtype=np.int64)
        _native.check(_native.lib().kw_stats(self.h, _native.ptr(v), _native.KW_N_STATS), self.h)
        return {k: int(x) for k, x in zip(self.STAT_KEYS, v)}

    def kernel_times(self) -> Dict[str, float]:
        """Per-kernel device times (ms) of the last scan."""
        keys = ('scan', 'resolve', 'generic', 'compact', 'total', 'filter', 'probe', 'epilogue', 'resolve_kernel', 'tasks')
        v = np.zeros(len(keys), dtype=np.float32)
        _native.check(_native.lib().kw_last_kernel_times(self.h, _native.ptr(v), len(keys)), self.h)
        return dict(zip(keys, (float(x) for x in v)))

    def kernel_ms(self) -> Tuple[float, float, float]:
        """(fast kernel, generic kernel, all kernels incl. compaction) in ms for the last scan."""
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        _native.check(_native.lib().kw_last_kernel_ms(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                      self.h)
        return float(a.value), float(b.value), float(c.value)

    def match_strings(self, texts: Sequence[str], titles: Sequence[str]) -> np.ndarray:
        """Convenience: pack, scan through the host-buffer entry points, fetch (no torch)."""
        arena, off = pack_fields(texts, titles)
        self.scan_host(arena, off, len(texts))
        return self.fetch_host()

    # -- host buffers (kw_scan_host / kw_hits_host): the drop-in driver's single-GPU path, no torch
    def scan_host(self, arena: np.ndarray, off: np.ndarray, n_docs: int) -> None:
        """Copy a host arena (its padding included) and its 2n+1 offsets to library-owned device buffers and
        scan them (asynchronous until :meth:`fetch_host`)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(off[:2 * int(n_docs) + 1], dtype=np.int64)
        self._keep = (arena, off)
        _native.check(_native.lib().kw_scan_host(self.h, _native.ptr(arena), int(arena.size), _native.ptr(off),
                                                 int(n_docs)), self.h)

    def fetch_host(self) -> np.ndarray:
        """Records of the last scan on the host (structured HIT_DTYPE array)."""
        n = self.n_hits()
        out = np.empty(max(n, 1), dtype=_native.HIT_DTYPE)
        cnt = ctypes.c_int64()
        _native.check(_native.lib().kw_hits_host(self.h, _native.ptr(out), n, ctypes.byref(cnt)), self.h)
        return out[:cnt.value]

    def match_device(self, texts: Sequence[str], titles: Sequence[str]):
        """Pack, upload and scan; the records as a device tensor [n, 4] (int32 view of kw_hit)."""
        arena, off = pack_fields(texts, titles)
        d_arena, d_off = self.upload(arena, off)
        self.scan(d_arena, d_off, len(texts))
        return self.hits_device()


def records_from_tensor(t) -> np.ndarray:
    """[n, 4] int32 records (device or host tensor) -> structured HIT_DTYPE array on the host."""
    host = t.cpu().numpy() if hasattr(t, 'cpu') else np.asarray(t)
    return np.ascontiguousarray(host).view(np.uint32).reshape(-1, 4).copy().view(_native.HIT_DTYPE).reshape(-1)


# --------------------------------------------------------------------- assembly
def group_hits(hits: np.ndarray) -> Dict[int, Dict[int, Dict[int, List[int]]]]:
    """doc -> field -> pattern -> sorted positions ([] for a position-less match)."""
    out: Dict[int, Dict[int, Dict[int, List[int]]]] = {}
    if len(hits) == 0:
        return out
    order = np.lexsort((hits['pos'], hits['pattern'], hits['field'], hits['doc']))
    h = hits[order]
    docs = h['doc'].tolist()
    fields = h['field'].tolist()
    pats = h['pattern'].tolist()
    poss = h['pos'].tolist()
    nopos = _native.KW_NOPOS
    for d, f, p, q in zip(docs, fields, pats, poss):
        lst = out.setdefault(d, {}).setdefault(f, {}).setdefault(p, [])
        if q != nopos:
            lst.append(q)
    return out


def _rank_order(d):
    """Items of pattern -> (rank, positions) in rank order (dict order when there is at most one)."""
    return sorted(d.items(), key=lambda kv: kv[1][0]) if len(d) > 1 else d.items()


def assemble_ticker_matches(ckb: CompiledKB, doc_fields: Dict[int, Dict[int, List[int]]], article_date):
    """The reference's per-article ``ticker_matches`` (match_keywords.py:153-187).

    ``doc_fields`` holds the device results of one article (field -> pattern
    -> positions).  Each pattern's (ticker, attribute, name) occurrences are
    filtered by ``is_within_period``; inside a ticker a name takes the dict
    position of its first in-period occurrence.
    """
    if article_date is None:
        return {}
    occ_us = ckb.occurrences_us()
    a_us = None
    if occ_us is not None:
        try:
            a_us = epoch_us(article_date)
        except TypeError:
            a_us = None
    per_ticker: Dict[int, Tuple[dict, dict]] = {}
    for field_idx in (0, 1):
        pats = doc_fields.get(field_idx)
        if not pats:
            continue
        for pat, positions in pats.items():
            best: Dict[int, int] = {}
            if a_us is not None:
                # integer form of is_within_period (kb.epoch_us): exact, no per-occurrence tz conversion
                for (ti, rank, lo, hi) in occ_us[pat]:
                    if lo <= a_us <= hi and ti not in best:
                        best[ti] = rank
            else:
                for (ti, rank, start, end) in ckb.occurrences[pat]:
                    if ti in best:
                        continue   # occurrences are in rank order: the first in-period one wins
                    if is_within_period(article_date, start, end):
                        best[ti] = rank
            if best and ckb.invalid_regex[pat]:
                # the reference's re.finditer(name, s) raises re.error here (:178/:180)
                re.compile(ckb.names[pat])
            for ti, rank in best.items():
                slot = per_ticker.setdefault(ti, ({}, {}))
                slot[field_idx][pat] = (rank, positions)
    result = {}
    for ti in sorted(per_ticker):
        text_d, title_d = per_ticker[ti]
        if not text_d and not title_d:
            continue
        text = {ckb.names[p]: list(v[1]) for p, v in _rank_order(text_d)}
        title = {ckb.names[p]: list(v[1]) for p, v in _rank_order(title_d)}
        result[ckb.tickers[ti]] = {'text': text, 'title': title}
    return result
