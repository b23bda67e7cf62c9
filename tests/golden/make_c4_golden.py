"""Generate the config-4 golden fixture: the ~50k-pattern synthetic KB vs seeded articles.

Inputs are a pure function of seeds (advanced_scrapper_amd/synth_kb.py for the
KB, csrc/synth.c for the articles), so the fixture stores only digests of them
and the expected per-field results, computed by the CPU oracle
(oracle/kwmatch_oracle.py: CPython ``re`` for ``\\b`` literals and regex
positions, oracle/partial_ratio.c for rapidfuzz ``partial_ratio > 95``; the
oracle itself is pinned against the reference's own outputs on config 1 by
tests/golden/make_golden.py).

    python tests/golden/make_c4_golden.py      # ~2 min on 8 cores

Output: tests/golden/c4_golden.json.gz
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

KB_SEED = 20250905
N_TICKERS = 2300
DOC_SEED = 41
N_DOCS = 200


def inputs():
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.synth_kb import synthetic_kb
    kb = synthetic_kb(N_TICKERS, KB_SEED)
    ckb = compile_kb(kb)
    names, kinds = synth.injectable_names(ckb)
    corpus = synth.generate(N_DOCS, names, kinds, seed=DOC_SEED)
    return kb, ckb, corpus


def digests(ckb, corpus):
    return {'kb_names_sha256': hashlib.sha256('\n'.join(ckb.names).encode('utf-8', 'surrogatepass')).hexdigest(),
            'arena_sha256': hashlib.sha256(corpus.arena[:corpus.n_bytes].tobytes()).hexdigest()}


def main():
    from tests import oracle_pool
    kb, ckb, corpus = inputs()
    t0 = time.time()
    texts, titles = corpus.texts(), corpus.titles()
    want_t = oracle_pool.field_results(kb, texts, procs=os.cpu_count())
    want_i = oracle_pool.field_results(kb, titles, procs=os.cpu_count())
    docs = [[sorted(want_t[d].items()), sorted(want_i[d].items())] for d in range(N_DOCS)]
    out = {'kb_seed': KB_SEED, 'n_tickers': N_TICKERS, 'doc_seed': DOC_SEED, 'n_docs': N_DOCS,
           'n_patterns': ckb.n_patterns, **digests(ckb, corpus), 'oracle_seconds': round(time.time() - t0, 1),
           'docs': docs}
    with gzip.open(os.path.join(HERE, 'c4_golden.json.gz'), 'wt', encoding='utf-8') as fh:
        json.dump(out, fh, ensure_ascii=True)
    n = sum(len(a) + len(b) for a, b in docs)
    print(f"{N_DOCS} docs, {ckb.n_patterns} patterns, {n} field results, {out['oracle_seconds']} s")


if __name__ == '__main__':
    main()
