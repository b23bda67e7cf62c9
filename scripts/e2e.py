"""End-to-end drop-in timing: ``match_keywords.main`` itself over N synthetic articles, then a per-phase split.

Generates N articles of the config-2 corpus (csrc/synth.c, bench seed), writes them as the reference's article
CSV and the reference's KB JSON files (tests/golden/kb_bundle.json.gz, the reference's info/ticker) into a
scratch directory, and times ``python -m advanced_scrapper_amd.match_keywords --info-dir ... --articles ...``'s
``main()`` in-process from its first line to its return: KB load (read_and_process_json_files, prints
included), KB compile + kw_compile, native CSV ingest, GPU matching, JSON cells, row rendering, the appends
and the final sort (match_keywords.py:220-246).  A second pass over the same CSV runs main's per-chunk phases
one by one (read, dates, arena, GPU, render, write, sort) for the split; both passes must write the same
bytes.  One JSON line: end-to-end articles/s of main(), the split, the host threads.

    python scripts/e2e.py [--docs 200000] [--chunksize 20000]
"""
import argparse
import contextlib
import hashlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _digest(out_dir):
    h = hashlib.sha256()
    for fn in sorted(os.listdir(out_dir)):
        h.update(fn.encode())
        with open(os.path.join(out_dir, fn), 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()


def phases(args, csv_path, processed):
    """main()'s per-chunk steps timed one by one (the split; same writes as main)."""
    from advanced_scrapper_amd import egress, ingest, match_keywords as mk
    t = dict(read=0.0, dates=0.0, arena=0.0, gpu_match=0.0, render=0.0, write=0.0, sort=0.0)
    os.makedirs('yahoo_ticker_matched_articles')
    mk._RUN = egress.RunFiles('yahoo_ticker_matched_articles')
    matcher = None
    c0 = time.perf_counter()
    for chunk in ingest.read_chunks(csv_path, args.chunksize):
        c1 = time.perf_counter(); t['read'] += c1 - c0
        if not isinstance(chunk, ingest.NativeChunk):
            matcher = mk._write_chunk('yahoo', chunk, processed, matcher)
            c0 = time.perf_counter(); t['write'] += c0 - c1
            continue
        dates, error = chunk.dates()
        c2 = time.perf_counter(); t['dates'] += c2 - c1
        if matcher is None:
            matcher = mk.get_matcher(processed, 0, mk._native_sample(chunk))
        c2 = time.perf_counter()
        arena, off = chunk.arena()
        off = off[:2 * len(dates) + 1]
        c3 = time.perf_counter(); t['arena'] += c3 - c2
        matcher.scan_host(arena, off, len(dates))
        hits = matcher.fetch_host()
        c4 = time.perf_counter(); t['gpu_match'] += c4 - c3
        rendered, exc, _row = mk._native_rows(chunk, matcher, hits, dates, error)
        c5 = time.perf_counter(); t['render'] += c5 - c4
        egress.append_rendered('yahoo_ticker_matched_articles', rendered, mk._RUN)
        c0 = time.perf_counter(); t['write'] += c0 - c5
    c7 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        for name in os.listdir('yahoo_ticker_matched_articles'):
            if not mk._RUN.finish(name):
                mk.sort_matched_csv(f'yahoo_ticker_matched_articles/{name}')
    t['sort'] = time.perf_counter() - c7
    mk._RUN = None
    return {k: round(v, 3) for k, v in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--docs', type=int, default=200000)
    ap.add_argument('--chunksize', type=int, default=20000)
    ap.add_argument('--profile', action='store_true', help='cProfile main() (top functions by cumulative time)')
    args = ap.parse_args()
    os.environ.setdefault('TZ', 'UTC')
    time.tzset()
    import bench
    from advanced_scrapper_amd import ingest, match_keywords as mk, synth
    from advanced_scrapper_amd.kb import compile_kb
    work = tempfile.mkdtemp(prefix='e2e_')
    processed = bench.load_kb(os.path.join(work, 'ticker'))      # the reference's KB files, materialised
    names, kinds = synth.injectable_names(compile_kb(processed))
    corpus = synth.generate(args.docs, names, kinds, seed=20250905, doc_base=0)
    csv_path = os.path.join(work, 'articles.csv')
    synth.to_dataframe(corpus).to_csv(csv_path, index=False)
    csv_bytes = os.path.getsize(csv_path)
    del corpus
    os.chdir(work)
    # 1) the product's driver, end to end
    sink = io.StringIO()
    prof = None
    if args.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(sink):
        rc = mk.main(['--info-dir', os.path.join(work, 'ticker'), '--articles', csv_path,
                      '--chunksize', str(args.chunksize), '--device', '0'])
    total = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats('cumtime').print_stats(40)
    assert rc == 0
    d_main = _digest('yahoo_ticker_matched_articles')
    n_files = len(os.listdir('yahoo_ticker_matched_articles'))
    shutil.rmtree('yahoo_ticker_matched_articles')
    # 2) the split (the KB compile happens before the first chunk's phases and is not in them)
    split = phases(args, csv_path, processed)
    d_split = _digest('yahoo_ticker_matched_articles')
    out = {'docs': args.docs, 'chunksize': args.chunksize, 'csv_bytes': csv_bytes, 'files': n_files,
           'main_s': round(total, 3), 'articles_per_s': round(args.docs / total, 1),
           'phases_s': split, 'same_bytes': d_main == d_split, 'host_threads': ingest.host_threads(),
           'what': 'match_keywords.main() wall time: KB load from the reference JSON files + compile + ingest + '
                   'GPU match + render + append + final sort'}
    print(json.dumps(out), flush=True)
    os.chdir(REPO)
    shutil.rmtree(work, ignore_errors=True)


if __name__ == '__main__':
    main()
