"""ctypes binding of libkwmatch.so (include/kwmatch.h).

The library is built in-tree (``advanced_scrapper_amd/lib/``) by
``advanced_scrapper_amd.build`` / ``__graft_entry__.build()``.  There is no
fallback: if the library is missing or fails to load, every GPU entry point
raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib')
DEFAULT_LIB = os.path.join(LIB_DIR, 'libkwmatch.so')
LIB_PATH = DEFAULT_LIB


def _lib_path() -> str:
    """The default in-tree library; ``KW_LIB`` (a tuning variant of build.build_kwmatch_variant) only when
    ``bench.py --lib-variant`` asked for it (``KW_LIB_VARIANT_OK=1``): nothing else may swap the library."""
    alt = os.environ.get('KW_LIB')
    if not alt or os.path.abspath(alt) == DEFAULT_LIB:
        return DEFAULT_LIB
    if os.environ.get('KW_LIB_VARIANT_OK') != '1':
        raise RuntimeError(f"KW_LIB={alt}: only bench.py --lib-variant loads a non-default libkwmatch")
    return os.path.abspath(alt)

KW_OK = 0
KW_EINVAL = -1
KW_EUNSUPPORTED = -2
KW_EHIP = -3
KW_EOVERFLOW = -4
KW_ESTATE = -5
KW_NOPOS = 0xFFFFFFFF

HIT_DTYPE = np.dtype([('doc', '<u4'), ('pattern', '<u4'), ('pos', '<u4'), ('field', '<u4')])

# every symbol include/kwmatch.h and include/kwdedup.h declare
EXPORTS = ('kw_compile', 'kw_scan', 'kw_hits', 'kw_hits_copy', 'kw_stats', 'kw_last_kernel_ms',
           'kw_last_kernel_times', 'kw_doc_routes', 'kw_last_error', 'kw_destroy',
           'kw_scan_host', 'kw_hits_host', 'kw_device_count', 'kw_device_init',
           'kw_comm_unique_id', 'kw_comm_init', 'kw_allgather_counts', 'kw_allgather_hits',
           'kw_allgather_hits_planned', 'kw_exchange_plan', 'kw_exchange_caps_ok', 'kw_comm_last_error',
           'kw_comm_destroy',
           'kw_dedup_create', 'kw_dedup_run', 'kw_dedup_counts', 'kw_dedup_kept_size', 'kw_dedup_kept_copy',
           'kw_dedup_last_ms', 'kw_dedup_last_error', 'kw_dedup_destroy', 'dedup_urls')

# KW_URL_* row codes (include/kwdedup.h)
KW_URL_NO_HTML, KW_URL_KEPT, KW_URL_FILTERED, KW_URL_DUPLICATE = 0, 1, 2, 3
KW_DEDUP_NORMALIZE = 1
KW_N_STATS = 21
# KW_RESCAN_* bits of stats[20] (include/kwmatch.h)
KW_RESCAN_GENERIC_ITEMS, KW_RESCAN_RESULTS, KW_RESCAN_GENERIC_CPS = 1, 2, 4
KW_RESCAN_REGEX_QUEUE, KW_RESCAN_TASK_QUEUES, KW_RESCAN_DECIDED_SET, KW_RESCAN_REGIONS = 16, 32, 64, 128
KW_COMM_ID_BYTES = 128
KW_ROUTE_SCAN, KW_ROUTE_RESOLVE, KW_ROUTE_GENERIC, KW_ROUTE_TRANSCODE = 0, 1, 2, 3
KW_PLAN_SEND, KW_PLAN_RECV = 1, 2


class KwError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libkwmatch error {code}: {msg}")
        self.code = code


_LIB = None


def lib() -> ctypes.CDLL:
    """Load libkwmatch.so (raises if it was not built)."""
    global _LIB, LIB_PATH
    if _LIB is not None:
        return _LIB
    LIB_PATH = _lib_path()
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.kw_dedup_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.kw_dedup_run.argtypes = [vp, vp, vp, i64, i32, vp, vp]
    L.kw_dedup_counts.argtypes = [vp, vp]
    L.kw_dedup_kept_size.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.kw_dedup_kept_copy.argtypes = [vp, vp, vp, vp, vp]
    L.kw_dedup_last_ms.argtypes = [vp, vp, i32]
    L.kw_dedup_last_error.argtypes = [vp]
    L.kw_dedup_last_error.restype = ctypes.c_char_p
    L.kw_dedup_destroy.argtypes = [vp]
    L.dedup_urls.argtypes = [vp, vp, i64, vp, vp]
    for f in ('kw_dedup_create', 'kw_dedup_run', 'kw_dedup_counts', 'kw_dedup_kept_size', 'kw_dedup_kept_copy',
              'kw_dedup_last_ms', 'kw_dedup_destroy', 'dedup_urls'):
        getattr(L, f).restype = ctypes.c_int
    L.kw_compile.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp, i64, i32, ctypes.POINTER(vp)]
    L.kw_compile.restype = ctypes.c_int
    L.kw_scan.argtypes = [vp, vp, vp, i64, vp]
    L.kw_scan.restype = ctypes.c_int
    L.kw_hits.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(vp)]
    L.kw_hits.restype = ctypes.c_int
    L.kw_hits_copy.argtypes = [vp, vp, i64, ctypes.POINTER(i64), vp]
    L.kw_hits_copy.restype = ctypes.c_int
    L.kw_stats.argtypes = [vp, vp, i32]
    L.kw_stats.restype = ctypes.c_int
    L.kw_last_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                    ctypes.POINTER(ctypes.c_float)]
    L.kw_last_kernel_ms.restype = ctypes.c_int
    L.kw_last_kernel_times.argtypes = [vp, vp, i32]
    L.kw_last_kernel_times.restype = ctypes.c_int
    L.kw_doc_routes.argtypes = [vp, vp, i64]
    L.kw_doc_routes.restype = ctypes.c_int
    L.kw_scan_host.argtypes = [vp, vp, i64, vp, i64]
    L.kw_scan_host.restype = ctypes.c_int
    L.kw_hits_host.argtypes = [vp, vp, i64, ctypes.POINTER(i64)]
    L.kw_hits_host.restype = ctypes.c_int
    L.kw_device_count.argtypes = [ctypes.POINTER(i32)]
    L.kw_device_count.restype = ctypes.c_int
    L.kw_device_init.argtypes = [i32]
    L.kw_device_init.restype = ctypes.c_int
    L.kw_comm_unique_id.argtypes = [vp]
    L.kw_comm_init.argtypes = [i32, i32, vp, i32, ctypes.POINTER(vp)]
    L.kw_allgather_counts.argtypes = [vp, i64, vp, vp]
    L.kw_allgather_hits.argtypes = [vp, vp, i64, i64, i32, vp, i64, ctypes.POINTER(i64), vp, vp]
    L.kw_allgather_hits_planned.argtypes = [vp, vp, i64, i64, i32, vp, vp, i64, ctypes.POINTER(i64), vp]
    L.kw_exchange_caps_ok.argtypes = [i32, i32, vp, vp, ctypes.POINTER(i32)]
    L.kw_exchange_caps_ok.restype = ctypes.c_int
    L.kw_comm_destroy.argtypes = [vp]
    L.kw_exchange_plan.argtypes = [i32, i32, i32, vp, vp, vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.kw_exchange_plan.restype = ctypes.c_int
    for f in ('kw_comm_unique_id', 'kw_comm_init', 'kw_allgather_counts', 'kw_allgather_hits',
              'kw_allgather_hits_planned', 'kw_comm_destroy'):
        getattr(L, f).restype = ctypes.c_int
    L.kw_comm_last_error.argtypes = [vp]
    L.kw_comm_last_error.restype = ctypes.c_char_p
    L.kw_last_error.argtypes = [vp]
    L.kw_last_error.restype = ctypes.c_char_p
    L.kw_destroy.argtypes = [vp]
    L.kw_destroy.restype = ctypes.c_int
    _LIB = L
    return L


def lib_identity() -> dict:
    """Which libkwmatch this process loaded: path (relative to the package), sha256, default or variant."""
    import hashlib
    lib()
    with open(LIB_PATH, 'rb') as fh:
        digest = hashlib.sha256(fh.read()).hexdigest()
    return {'path': os.path.relpath(LIB_PATH, os.path.dirname(LIB_DIR)), 'sha256': digest,
            'default': LIB_PATH == DEFAULT_LIB,
            'env': {k: v for k, v in sorted(os.environ.items()) if k.startswith('KW_')}}


def device_count() -> int:
    """HIP devices visible to this process (libkwmatch's hipGetDeviceCount; no torch)."""
    n = ctypes.c_int32()
    lib().kw_device_count(ctypes.byref(n))
    return int(n.value)


def exchange_plan(nranks: int, rank: int, root: int, counts):
    """kw_exchange_plan (pure host): (recv_off[nranks + 1], ops[nranks], n_total, n_recv) of `rank`."""
    cnt = np.ascontiguousarray(counts, dtype=np.int64)
    off = np.zeros(nranks + 1, dtype=np.int64)
    ops = np.zeros(nranks, dtype=np.int32)
    tot, nrecv = ctypes.c_int64(), ctypes.c_int64()
    rc = lib().kw_exchange_plan(nranks, rank, root, ptr(cnt), ptr(off), ptr(ops), ctypes.byref(tot), ctypes.byref(nrecv))
    if rc != KW_OK:
        raise KwError(rc, 'kw_exchange_plan: bad arguments')
    return off, ops, int(tot.value), int(nrecv.value)


def exchange_caps_ok(nranks: int, root: int, counts, caps):
    """kw_exchange_caps_ok (pure host): (ok, first short receiver or -1)."""
    cnt = np.ascontiguousarray(counts, dtype=np.int64)
    cap = np.ascontiguousarray(caps, dtype=np.int64)
    bad = ctypes.c_int32(-1)
    rc = lib().kw_exchange_caps_ok(nranks, root, ptr(cnt), ptr(cap), ctypes.byref(bad))
    if rc not in (KW_OK, KW_EOVERFLOW):
        raise KwError(rc, 'kw_exchange_caps_ok: bad arguments')
    return rc == KW_OK, int(bad.value)


def check(rc: int, handle=None) -> None:
    if rc != KW_OK:
        msg = lib().kw_last_error(handle)
        raise KwError(rc, msg.decode('utf-8', 'replace') if msg else '')


def check_comm(rc: int, comm=None) -> None:
    if rc != KW_OK:
        msg = lib().kw_comm_last_error(comm)
        raise KwError(rc, msg.decode('utf-8', 'replace') if msg else '')


def ptr(a) -> ctypes.c_void_p:
    """Raw pointer of a numpy array or torch tensor."""
    if a is None:
        return ctypes.c_void_p(0)
    if isinstance(a, np.ndarray):
        return ctypes.c_void_p(a.ctypes.data)
    return ctypes.c_void_p(a.data_ptr())
