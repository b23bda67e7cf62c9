"""A stand-in for GpuMatcher below kw_scan, for CPU tests of the host path (tests only).

It returns the records kw_scan returns ([n, 4] int32 = kw_hit: doc, pattern,
code-point position or KW_NOPOS, field) computed by the CPU oracle, so the
drop-in's assembly, row building, error handling, sharding and CSV egress run
unchanged on a machine without a GPU.
"""
import numpy as np
import torch


class OracleMatcher:
    def __init__(self, processed):
        from advanced_scrapper_amd.kb import compile_kb
        from oracle import kwmatch_oracle as orc
        self.ckb = compile_kb(processed)
        self.oracle = orc.Oracle(processed)
        self.pid = {n: i for i, n in enumerate(self.ckb.names)}
        self.uploads = []        # (documents, arena bytes) of every upload: what this process scanned

    def _field(self, s):
        """name -> positions as kw_scan reports them (a name whose regex does not compile keeps its
        decision with no position: the host assembly raises the reference's re.error for it)."""
        import re
        from oracle import kwmatch_oracle as orc
        out = {}
        for n in self.oracle.upper:
            pos = orc.upper_positions(n, s)
            if pos:
                out[n] = pos
        for n, hit in zip(self.oracle.fuzzy, self.oracle.fset.decide(s)):
            if hit:
                try:
                    out[n] = orc.regex_positions(n, s)
                except re.error:
                    out[n] = []
        return out

    def match_device(self, texts, titles):
        rows = []
        for d, pair in enumerate(zip(texts, titles)):
            for f, s in enumerate(pair):
                for name, pos in self._field(s).items():
                    p = self.pid[name]
                    rows += [(d, p, q, f) for q in pos] if pos else [(d, p, 0xFFFFFFFF, f)]
        a = np.asarray(rows, dtype=np.uint32).reshape(-1, 4)
        return torch.from_numpy(a.view(np.int32).copy())

    # the kw_scan-shaped calls of the native ingest path: an arena + offsets "upload", a scan of n documents
    # starting at an offsets slice, the records of the last scan
    def upload(self, arena, off):
        self.uploads.append(((len(off) - 1) // 2, int(off[-1] - off[0])))
        return arena, off

    def scan(self, d_arena, d_off, n_docs, stream=None):
        b = bytes(d_arena)
        texts = [b[d_off[2 * i]:d_off[2 * i + 1]].decode('utf-8', 'surrogatepass') for i in range(n_docs)]
        titles = [b[d_off[2 * i + 1]:d_off[2 * i + 2]].decode('utf-8', 'surrogatepass') for i in range(n_docs)]
        self._last = self.match_device(texts, titles)

    def scan_host(self, arena, off, n_docs):
        self.upload(arena, off[:2 * n_docs + 1])
        self.scan(arena, off, n_docs)

    def fetch_host(self):
        return self.fetch()

    def hits_device(self):
        return self._last

    def fetch(self):
        from advanced_scrapper_amd.matcher import records_from_tensor
        return records_from_tensor(self._last)

    def match_strings(self, texts, titles):
        from advanced_scrapper_amd.matcher import records_from_tensor
        return records_from_tensor(self.match_device(texts, titles))
