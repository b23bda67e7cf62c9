"""The drop-in's CSV bytes on a 20k-row slice of the config-2 corpus, produced by the REFERENCE itself.

Input: documents 0..19 999 of bench.py's corpus (csrc/synth.c, seed 20250905)
as the reference's article CSV (synth.to_dataframe: the dataset schema, unique
naive dates, NaN text/title where the generator flags them), one chunk of
20 000 rows (the reference's chunksize, match_keywords.py:227).  The reference
match_keywords.py is imported in this container with rapidfuzz stubbed by the
oracle's restatement (as make_golden.py does) and its own ``process_chunk``
(:148-192) runs over the rows, then ``sort_matched_csv`` (:195-217) over every
output file.  To finish in minutes, contiguous row ranges run in separate
processes, each appending into its own directory; a range's per-ticker file is
then the rows that range appended, so concatenating the ranges in order (one
header) is byte for byte the file one sequential process_chunk writes (every
row is its own ``to_csv(mode='a')``, :145-146).

Only digests are committed (tests/golden/c2_slice.json): the CSV's sha256 and
every output file's sha256 and size.  tests/test_gpu_scale.py rebuilds the
CSV on the GPU box, runs the drop-in's main path over it and compares.

    python tests/golden/make_c2_slice.py [--procs 7]
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import io
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)

SEED = 20250905
N_ROWS = 20000
OUT_DIR = 'yahoo_ticker_matched_articles'


def slice_csv_bytes(n_rows: int = N_ROWS) -> bytes:
    """The article CSV of documents [0, n_rows) of the config-2 corpus (also used by the GPU test)."""
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb
    from tests import golden_data
    ckb = compile_kb(golden_data.kb_processed())
    names, kinds = synth.injectable_names(ckb)
    corpus = synth.generate(n_rows, names, kinds, seed=SEED, doc_base=0)
    return synth.to_dataframe(corpus).to_csv(index=False).encode('utf-8')


def _worker(args):
    csv_path, lo, hi, work = args
    os.environ['TZ'] = 'UTC'
    time.tzset()
    from tests.golden.make_golden import _stub_rapidfuzz
    _stub_rapidfuzz()
    sys.path.insert(0, REF)
    import pandas as pd
    import match_keywords as ref      # the reference, imported (not copied)
    with contextlib.redirect_stdout(io.StringIO()):
        processed = ref.read_and_process_json_files(os.path.join(REF, 'info', 'ticker'))
    from tests import golden_data
    want = golden_data.kb_processed()
    assert list(processed) == list(want) and all(list(processed[t]) == list(want[t]) for t in want), 'KB order'
    df = pd.read_csv(csv_path)        # one 20k-row chunk, dtypes inferred over it as the reference's reader does
    os.makedirs(os.path.join(work, OUT_DIR), exist_ok=True)
    os.chdir(work)
    with contextlib.redirect_stderr(io.StringIO()):
        ref.process_chunk('yahoo', df.iloc[lo:hi], processed)
    return lo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=7)
    ap.add_argument('--rows', type=int, default=N_ROWS)
    ap.add_argument('--out', default=os.path.join(HERE, 'c2_slice.json'))
    args = ap.parse_args()
    n_rows = args.rows
    os.environ['TZ'] = 'UTC'
    time.tzset()
    from tests import golden_data
    csv_bytes = slice_csv_bytes(n_rows)
    t0 = time.time()
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, 'articles.csv')
        with open(src, 'wb') as fh:
            fh.write(csv_bytes)
        cuts = [n_rows * k // (4 * args.procs) for k in range(4 * args.procs + 1)]
        jobs = [(src, cuts[k], cuts[k + 1], os.path.join(tmp, f'part{k:03d}')) for k in range(len(cuts) - 1)]
        with mp.get_context('spawn').Pool(args.procs) as pool:
            pool.map(_worker, jobs, chunksize=1)
        merged = os.path.join(tmp, 'merged', OUT_DIR)
        os.makedirs(merged)
        files = {}
        for _s, _lo, _hi, work in jobs:                       # ranges in document order
            d = os.path.join(work, OUT_DIR)
            for fn in os.listdir(d):
                data = open(os.path.join(d, fn), 'rb').read()
                if fn in files:
                    data = data[data.index(b'\n') + 1:]       # the header is the first line
                files.setdefault(fn, []).append(data)
        for fn, parts in files.items():
            with open(os.path.join(merged, fn), 'wb') as fh:
                fh.write(b''.join(parts))
        # the reference's final pass over the directory (:243-244)
        from tests.golden.make_golden import _stub_rapidfuzz
        _stub_rapidfuzz()
        sys.path.insert(0, REF)
        import match_keywords as ref
        cwd = os.getcwd()
        os.chdir(os.path.dirname(merged))
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                for fn in os.listdir(OUT_DIR):
                    ref.sort_matched_csv(f'{OUT_DIR}/{fn}')
        finally:
            os.chdir(cwd)
        out = {}
        for fn in sorted(os.listdir(merged)):
            data = open(os.path.join(merged, fn), 'rb').read()
            out[fn] = {'sha256': hashlib.sha256(data).hexdigest(), 'bytes': len(data)}
    meta = {'generator': 'tests/golden/make_c2_slice.py (the reference match_keywords.py imported, rapidfuzz '
                         'stubbed by oracle/partial_ratio.c)',
            'seed': SEED, 'rows': n_rows, 'chunksize': N_ROWS,
            'kb_manifest_sha256': golden_data.manifest()['files']['kb_bundle.json.gz']['sha256'],
            'csv_sha256': hashlib.sha256(csv_bytes).hexdigest(), 'csv_bytes': len(csv_bytes),
            'reference_seconds': round(time.time() - t0, 1), 'procs': args.procs, 'files': out}
    with open(args.out, 'w') as fh:
        json.dump(meta, fh, indent=1)
    print(len(out), 'files', meta['reference_seconds'], 's')


if __name__ == '__main__':
    main()
