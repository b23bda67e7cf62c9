"""Seeded synthetic financial-news corpus (bench / test data).

Thin wrapper over ``lib/libsynth.so`` (csrc/synth.c).  Documents are a pure
function of (seed, global index): shards generated on different ranks are
byte-identical to the same documents of the full corpus.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Tuple

import numpy as np

from .kb import CLASS_FUZZY, CLASS_UPPER, CompiledKB
from .matcher import ARENA_PAD

DEFAULT_SEED = 20250905

_VOCAB = """
the of and to in a for on that with as at by from is was are be has have will its it this their
said says reported announced expects expected shares stock stocks market markets investors analysts
quarter quarterly annual revenue revenues earnings profit profits loss losses sales growth guidance
outlook forecast estimate estimates billion million percent higher lower rose fell gained dropped
climbed slipped jumped tumbled rallied surged declined advanced index indexes trading traded session
week month year today yesterday tomorrow company companies firm firms business businesses industry
sector sectors technology energy health care financial financials banking bank banks consumer retail
industrial industrials materials utilities real estate communication services software hardware chips
semiconductor semiconductors cloud data artificial intelligence model models platform platforms device
devices product products launch launched new deal deals merger acquisition acquire acquired bid offer
agreement partnership regulators regulatory approval lawsuit settlement fine investigation board chief
executive officer financial officer president chairman founder management leadership strategy plan
plans cost costs cut cuts jobs workers employees hiring layoffs wage wages inflation rates rate interest
federal reserve central policy economy economic economists recession demand supply chain prices price
oil gas crude gold dollar currency bond bonds yield yields treasury debt credit loan loans deposit
dividend dividends buyback repurchase capital spending investment investments fund funds hedge private
equity venture valuation multiple premium discount target upgrade downgrade rating buy sell hold neutral
overweight underweight consensus beat missed topped fell short results statement filing report call
conference remarks comments noted added told interview according people familiar matter sources
however while although despite because after before during since amid following ahead against over
under about around between through into out up down more most less least much many several some
other another each every all both few first second third last next early late recent strong weak
solid robust modest slight sharp steep record high low peak trough level levels range target margin
margins operating net gross adjusted per share basis points trillion thousand hundreds dozens customers
users subscribers orders backlog shipments production output capacity inventory inventories stores
online digital mobile payments advertising subscription streaming content games gaming travel airline
airlines automaker automakers vehicles electric battery batteries charging insurance insurer pharma drug
drugs trial trials vaccine patients hospital medical devices biotech research development analysts
""".split()

_ACRONYMS = "CEO CFO COO IPO ETF GDP EPS SEC FTC DOJ EU UK US USD EUR NYSE ESG AI EV Q1 Q2 Q3 Q4 YoY M&A".split()

_UNICODE = ["café", "naïve", "Zürich", "São Paulo", "Québec", "Düsseldorf", "résumé", "—", "–", "“quoted”",
            "‘single’", "€12.5", "£3.2", "¥150", "中国", "日本", "한국", "Ελλάδα", "Москва", "ﬁnance", "Ⅷ",
            "２０２４", "ﬀ", "é", "’s", "naïveté", "Øresund", "İstanbul"]


class _Ctx(ctypes.Structure):
    _fields_ = [
        ('vocab', ctypes.c_void_p), ('vocab_off', ctypes.c_void_p), ('n_vocab', ctypes.c_int),
        ('acr', ctypes.c_void_p), ('acr_off', ctypes.c_void_p), ('n_acr', ctypes.c_int),
        ('uni', ctypes.c_void_p), ('uni_off', ctypes.c_void_p), ('n_uni', ctypes.c_int),
        ('names', ctypes.c_void_p), ('name_off', ctypes.c_void_p), ('name_kind', ctypes.c_void_p),
        ('n_names', ctypes.c_int),
        ('u_idx', ctypes.c_void_p), ('n_u', ctypes.c_int),
        ('f_idx', ctypes.c_void_p), ('n_f', ctypes.c_int),
    ]


_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib', 'libsynth.so')
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run python -m advanced_scrapper_amd.build")
        L = ctypes.CDLL(path)
        L.synth_lengths.argtypes = [ctypes.POINTER(_Ctx), ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_void_p]
        L.synth_fill.argtypes = [ctypes.POINTER(_Ctx), ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.synth_ctx_size.restype = ctypes.c_int
        assert L.synth_ctx_size() == ctypes.sizeof(_Ctx), "synth_ctx layout mismatch"
        _LIB = L
    return _LIB


def _blob(strings: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    enc = [s.encode('utf-8', 'surrogatepass') for s in strings]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    data = np.frombuffer(b''.join(enc) + b'\0', dtype=np.uint8).copy()
    return data, off


class Corpus:
    """A generated corpus: arena (uint8, padded), offsets (2n+1), flags (n)."""

    def __init__(self, arena: np.ndarray, off: np.ndarray, flags: np.ndarray, doc_base: int, seed: int):
        self.arena, self.off, self.flags, self.doc_base, self.seed = arena, off, flags, doc_base, seed

    @property
    def n_docs(self) -> int:
        return len(self.flags)

    @property
    def n_bytes(self) -> int:
        return int(self.off[-1] - self.off[0])

    def text(self, i: int) -> str:
        return bytes(self.arena[self.off[2 * i]:self.off[2 * i + 1]]).decode('utf-8', 'surrogatepass')

    def title(self, i: int) -> str:
        return bytes(self.arena[self.off[2 * i + 1]:self.off[2 * i + 2]]).decode('utf-8', 'surrogatepass')

    def texts(self) -> List[str]:
        return [self.text(i) for i in range(self.n_docs)]

    def titles(self) -> List[str]:
        return [self.title(i) for i in range(self.n_docs)]


def injectable_names(ckb: CompiledKB) -> Tuple[List[str], List[int]]:
    """Names the generator injects (the active KB names) and their kinds (0 = U, 1 = F)."""
    names, kinds = [], []
    for name, cls in zip(ckb.names, ckb.classes):
        if not name:
            continue
        names.append(name)
        kinds.append(0 if cls == CLASS_UPPER else 1)
    return names, kinds


def generate(n_docs: int, names: Sequence[str], kinds: Sequence[int], seed: int = DEFAULT_SEED,
             doc_base: int = 0) -> Corpus:
    """Generate documents [doc_base, doc_base + n_docs) of the seeded corpus."""
    L = _lib()
    vocab, vocab_off = _blob(_VOCAB)
    acr, acr_off = _blob(_ACRONYMS)
    uni, uni_off = _blob(_UNICODE)
    nb, noff = _blob(list(names))
    nk = np.asarray(kinds, dtype=np.uint8)
    u_idx = np.flatnonzero(nk == 0).astype(np.int32)
    f_idx = np.flatnonzero(nk == 1).astype(np.int32)
    keep = (vocab, vocab_off, acr, acr_off, uni, uni_off, nb, noff, nk, u_idx, f_idx)
    ctx = _Ctx(vocab.ctypes.data, vocab_off.ctypes.data, len(_VOCAB),
               acr.ctypes.data, acr_off.ctypes.data, len(_ACRONYMS),
               uni.ctypes.data, uni_off.ctypes.data, len(_UNICODE),
               nb.ctypes.data, noff.ctypes.data, nk.ctypes.data, len(names),
               u_idx.ctypes.data if len(u_idx) else None, len(u_idx),
               f_idx.ctypes.data if len(f_idx) else None, len(f_idx))
    lens = np.zeros(2 * n_docs, dtype=np.int64)
    L.synth_lengths(ctypes.byref(ctx), seed, doc_base, n_docs, lens.ctypes.data)
    off = np.zeros(2 * n_docs + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    arena = np.zeros(int(off[-1]) + ARENA_PAD, dtype=np.uint8)
    flags = np.zeros(n_docs, dtype=np.uint8)
    L.synth_fill(ctypes.byref(ctx), seed, doc_base, n_docs, off.ctypes.data, arena.ctypes.data, flags.ctypes.data)
    del keep
    return Corpus(arena, off, flags, doc_base, seed)


def to_dataframe(corpus: Corpus, source: str = 'yahoo', span_docs: int = None, date_perm=None):
    """The article CSV schema the reference reads (match_keywords.py:150-152, :139-143).

    NaN flags become missing values (the CSV round trip turns them into NaN,
    which the reference matches as ``"nan"``).  Dates are unique seconds
    spread over 1980-2025 (naive, ``YYYY-MM-DD HH:MM:SS``); with ``span_docs``
    the spacing is that of a ``span_docs``-document corpus, so the documents of
    every slice of it get the same, increasing dates whatever the slicing.
    ``date_perm = (a, b)`` (with ``span_docs``; gcd(a, span_docs) = 1): document g
    gets the date of slot (a g + b) mod span_docs instead -- the same unique dates,
    in an order that is not the documents' (the output sort then has work to do).
    """
    import pandas as pd
    n = corpus.n_docs
    texts = corpus.texts()
    titles = corpus.titles()
    texts = [None if (corpus.flags[i] & 1) else t for i, t in enumerate(texts)]
    titles = [None if (corpus.flags[i] & 2) else t for i, t in enumerate(titles)]
    start = np.datetime64('1980-01-01T00:00:00')
    span = int((np.datetime64('2025-06-01T00:00:00') - start) / np.timedelta64(1, 's'))
    total = max(n, 1)
    step = max(span // max(span_docs if span_docs else total + corpus.doc_base, 1), 1)
    gidx = np.arange(corpus.doc_base, corpus.doc_base + n, dtype=np.int64)
    didx = gidx
    if date_perm is not None:
        import math
        a, b = date_perm
        assert span_docs and math.gcd(a, span_docs) == 1 and corpus.doc_base + n <= span_docs
        didx = (gidx * a + b) % span_docs
    jitter = (didx * 2654435761) % step
    stamps = start + (didx * step + jitter).astype('timedelta64[s]')
    dates = [str(s).replace('T', ' ') for s in stamps]
    urls = [f"https://finance.yahoo.com/news/synthetic-{corpus.seed}-{g}.html" for g in gidx]
    return pd.DataFrame({
        'article_text': texts, 'title': titles, 'date_time': dates, 'url': urls,
        'source': [source] * n, 'source_url': ['https://finance.yahoo.com'] * n,
    })


# --------------------------------------------------------------------- CDX link rows (config 5)
class UrlRows:
    """Synthetic CDX rows: URL arena (uint8, padded), offsets (n+1), CDX timestamps (int64)."""

    def __init__(self, arena: np.ndarray, off: np.ndarray, ts: np.ndarray, row_base: int, seed: int):
        self.arena, self.off, self.ts, self.row_base, self.seed = arena, off, ts, row_base, seed

    @property
    def n(self) -> int:
        return len(self.ts)

    @property
    def n_bytes(self) -> int:
        return int(self.off[-1] - self.off[0])

    def url(self, i: int) -> str:
        return bytes(self.arena[self.off[i]:self.off[i + 1]]).decode('utf-8', 'surrogatepass')

    def urls(self) -> List[str]:
        return [self.url(i) for i in range(self.n)]

    def cdx_text(self, lo: int = 0, hi: int = None) -> str:
        """The rows as CDX listing lines (urlkey timestamp original mimetype statuscode digest length)."""
        hi = self.n if hi is None else hi
        lines = []
        for i in range(lo, hi):
            u = self.url(i)
            key = 'com,yahoo,finance)/' + u.split('/', 3)[-1].lower()
            lines.append(f"{key} {int(self.ts[i])} {u} text/html 200 SYNTH{(self.row_base + i) % 99991:05d} {len(u) + 900}")
        return '\n'.join(lines) + '\n'


def generate_urls(n_rows: int, seed: int = DEFAULT_SEED, row_base: int = 0, n_articles: int = None) -> UrlRows:
    """Rows [row_base, row_base + n_rows) of the seeded CDX corpus (~30 % repeated articles)."""
    L = _lib()
    if not hasattr(L, '_url_types'):
        L.synth_url_lengths.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
        L.synth_url_fill.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L._url_types = True
    if n_articles is None:
        n_articles = max(1, int(1.31 * (row_base + n_rows)))
    lens = np.zeros(n_rows, dtype=np.int64)
    L.synth_url_lengths(seed, row_base, n_rows, n_articles, lens.ctypes.data)
    off = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    arena = np.zeros(int(off[-1]) + ARENA_PAD, dtype=np.uint8)
    ts = np.zeros(n_rows, dtype=np.int64)
    L.synth_url_fill(seed, row_base, n_rows, n_articles, off.ctypes.data, arena.ctypes.data, ts.ctypes.data)
    return UrlRows(arena, off, ts, row_base, seed)
