"""Drop-in for the CDX link-parts normalise + keep-first dedup of the reference
(yahoo_links_selenium.py:59-82 per part, :160-179 merge), on the GPU.

    process_part(txt_path, csv_path)      :59-82   one yahoo_XY.txt CDX listing -> yahoo_XY.csv
    merge_parts(folder, out='yfin_urls.csv')  :160-179  glob order, concat, keep-first -> yfin_urls.csv
    GpuUrlDedup                           the libkwmatch handle (include/kwdedup.h)

The CDX text is parsed on the host with the reference's own pandas call
(``read_csv(delimiter=' ', header=None, usecols=[1, 2])``); the URL column goes
to HBM as a UTF-8 arena + int64 offsets and the rewrite + keep-first runs in
HIP kernels (csrc/dedup.hip).  CSV writing stays on the host (pandas
``to_csv(index=False)``, as the reference).  There is no CPU fallback: without
a GPU or without libkwmatch.so the entry points raise.

``python -m advanced_scrapper_amd.cdx_dedup [folder]`` runs the reference's
post-scrape pipeline: every ``yahoo_links_1/*.txt`` -> part CSV, then the merge.
"""
from __future__ import annotations

import ctypes
import glob
import io
import os
import sys
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native

ARENA_PAD = 64


def pack_urls(urls: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    """UTF-8 arena (padded: readable 64 B past the end, kw_dedup_run needs 32) + int64 offsets (n + 1)."""
    enc = [u.encode('utf-8', 'surrogatepass') for u in urls]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        np.cumsum(np.fromiter((len(e) for e in enc), dtype=np.int64, count=len(enc)), out=off[1:])
    arena = np.zeros(int(off[-1]) + ARENA_PAD, dtype=np.uint8)
    if off[-1]:
        arena[:off[-1]] = np.frombuffer(b''.join(enc), dtype=np.uint8)
    return arena, off


class GpuUrlDedup:
    """One libkwmatch dedup handle on one GPU."""

    def __init__(self, device: Optional[int] = None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("GpuUrlDedup needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.torch = torch
        self.device = torch.cuda.current_device() if device is None else int(device)
        L = _native.lib()
        h = ctypes.c_void_p()
        rc = L.kw_dedup_create(self.device, ctypes.byref(h))
        if rc != _native.KW_OK:
            raise _native.KwError(rc, L.kw_dedup_last_error(h).decode() if h.value else 'create failed')
        self.h = h

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            _native.lib().kw_dedup_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != _native.KW_OK:
            raise _native.KwError(rc, _native.lib().kw_dedup_last_error(self.h).decode())

    def upload(self, arena: np.ndarray, off: np.ndarray):
        t = self.torch
        dev = t.device('cuda', self.device)
        return t.from_numpy(arena).to(dev), t.from_numpy(off).to(dev)

    def run(self, d_arena, d_off, n: int, normalize: bool = True, stream=None):
        """Codes (uint8 device tensor, KW_URL_*) of n device-resident rows."""
        t = self.torch
        code = t.empty(max(n, 1), dtype=t.uint8, device=t.device('cuda', self.device))
        if stream is None:
            stream = t.cuda.current_stream(self.device)
        self._check(_native.lib().kw_dedup_run(self.h, _native.ptr(d_arena), _native.ptr(d_off), int(n),
                                               _native.KW_DEDUP_NORMALIZE if normalize else 0, _native.ptr(code),
                                               ctypes.c_void_p(stream.cuda_stream)))
        return code[:n]

    def counts(self) -> List[int]:
        c = np.zeros(4, dtype=np.int64)
        self._check(_native.lib().kw_dedup_counts(self.h, _native.ptr(c)))
        return [int(x) for x in c]

    def kept_device(self):
        """(normalised URL bytes, offsets [n_kept + 1], source row indices [n_kept]) of the last run's kept rows,
        dense and in row order, as device tensors."""
        t = self.torch
        nk, nb = ctypes.c_int64(), ctypes.c_int64()
        self._check(_native.lib().kw_dedup_kept_size(self.h, ctypes.byref(nk), ctypes.byref(nb)))
        dev = t.device('cuda', self.device)
        b = t.empty(max(nb.value, 1), dtype=t.uint8, device=dev)
        o = t.empty(nk.value + 1, dtype=t.int64, device=dev)
        r = t.empty(max(nk.value, 1), dtype=t.int64, device=dev)
        st = t.cuda.current_stream(self.device)
        self._check(_native.lib().kw_dedup_kept_copy(self.h, _native.ptr(b), _native.ptr(o), _native.ptr(r),
                                                     ctypes.c_void_p(st.cuda_stream)))
        st.synchronize()
        return b[:nb.value], o, r[:nk.value]

    def kept(self) -> Tuple[np.ndarray, List[str]]:
        """(source row indices, normalised URLs) of the last run's kept rows, on the host."""
        b, o, r = self.kept_device()
        hb, ho, hr = b.cpu().numpy().tobytes(), o.cpu().numpy(), r.cpu().numpy()
        urls = [hb[ho[k]:ho[k + 1]].decode('utf-8', 'surrogatepass') for k in range(len(hr))]
        return hr, urls

    def last_ms(self) -> List[float]:
        """Device times (ms) of the last run: transform + hash + table insert, the byte-serial rows, decide,
        kept compaction, total (include/kwdedup.h kw_dedup_last_ms)."""
        v = np.zeros(5, dtype=np.float32)
        self._check(_native.lib().kw_dedup_last_ms(self.h, _native.ptr(v), 5))
        return [float(x) for x in v]

    def dedup_strings(self, urls: Sequence[str], normalize: bool = True) -> Tuple[np.ndarray, List[str]]:
        """Pack, upload, classify: (kept row indices, their normalised URLs)."""
        arena, off = pack_urls(urls)
        d_arena, d_off = self.upload(arena, off)
        self.run(d_arena, d_off, len(urls), normalize)
        return self.kept()


_DEDUP: Optional[GpuUrlDedup] = None


def _dedup() -> GpuUrlDedup:
    global _DEDUP
    if _DEDUP is None:
        _DEDUP = GpuUrlDedup()
    return _DEDUP


def read_cdx(path_or_text: str, is_text: bool = False):
    """The reference's parse of a CDX listing (yahoo_links_selenium.py:59)."""
    import pandas as pd
    src = io.StringIO(path_or_text) if is_text else path_or_text
    return pd.read_csv(src, delimiter=' ', header=None, usecols=[1, 2], names=['date_time', 'url'])


def dedup_frame(df, normalize: bool = True):
    """Rows of df (columns date_time, url) the reference keeps, with url rewritten (:63-79)."""
    import pandas as pd
    urls = df['url'].tolist()
    if any(not isinstance(u, str) for u in urls):
        # the reference's str.contains yields NaN there and the boolean mask raises (:63)
        raise ValueError("Cannot mask with non-boolean array containing NA / NaN values")
    rows, new = _dedup().dedup_strings(urls, normalize)
    out = df.iloc[rows].copy()
    out['url'] = new
    return out


def process_part(txt_path: str, csv_path: str) -> None:
    """yahoo_links_selenium.py:59-82 for one scraped CDX listing."""
    dedup_frame(read_cdx(txt_path)).to_csv(csv_path, index=False)


def merge_parts(folder: str = 'yahoo_links_1', out: str = 'yfin_urls.csv') -> Optional[int]:
    """yahoo_links_selenium.py:160-179: part CSVs in glob order, concat, keep-first."""
    import pandas as pd
    dfs = []
    for f in glob.glob(os.path.join(folder, '*.csv')):
        try:
            dfs.append(pd.read_csv(f))
        except Exception as e:  # the reference prints and skips unreadable parts (:168-169)
            print(f"Error reading {f}: {e}")
    if not dfs:
        print("No CSV files were processed. Check if the scraping was successful.")
        return None
    merged = pd.concat(dfs, ignore_index=True)
    merged = dedup_frame(merged, normalize=False)
    print(f"Found {len(merged)} unique URLs")
    merged.to_csv(out, index=False)
    print(f"Results saved to {out}")
    return len(merged)


def main(argv=None) -> None:
    folder = (argv or sys.argv[1:] or ['yahoo_links_1'])[0]
    for txt in sorted(glob.glob(os.path.join(folder, 'yahoo_*.txt'))):
        try:
            process_part(txt, txt[:-len('.txt')] + '.csv')
        except Exception as e:   # the reference prints and goes on (:86-88)
            print(f"Error scraping {txt}: {e}")
    merge_parts(folder)


if __name__ == '__main__':
    main()
