"""End-to-end drop-in timing: match_keywords.main's per-chunk phases around the GPU scan, then the sort.

Generates N synthetic articles (config-2 corpus), writes them as the reference's article CSV, then runs the
drop-in main loop's phases on chunks of 20 000 rows -- native CSV ingest (libkwcsv), date parse, arena +
GPU match, JSON cells (libkwrows) + rows rendered in C (kwcsv_emit), the per-ticker appends -- and the final
sort of every per-ticker file (match_keywords.py:243-244: from the run's write index, the re-read path for
the files it cannot decide), and prints one JSON line with seconds per phase and the end-to-end articles/s
(the reference's CPU path on the same rows is bench.py's cpu_baseline).

    python scripts/e2e.py [--docs 200000] [--chunksize 20000]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--docs', type=int, default=200000)
    ap.add_argument('--chunksize', type=int, default=20000)
    args = ap.parse_args()
    os.environ.setdefault('TZ', 'UTC')
    time.tzset()
    from advanced_scrapper_amd import ingest, match_keywords as mk, synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.rows import assemble_json_rows
    from tests import golden_data
    processed = golden_data.kb_processed()
    ckb = compile_kb(processed)
    names, kinds = synth.injectable_names(ckb)
    corpus = synth.generate(args.docs, names, kinds, seed=20250905, doc_base=0)
    work = tempfile.mkdtemp(prefix='e2e_')
    csv_path = os.path.join(work, 'articles.csv')
    synth.to_dataframe(corpus).to_csv(csv_path, index=False)
    os.chdir(work)
    os.makedirs('yahoo_ticker_matched_articles')
    t = dict(read=0.0, dates=0.0, arena=0.0, gpu_match=0.0, render=0.0, write=0.0, sort=0.0)
    matcher = None
    n_rows = n_native = n_chunks = 0
    from advanced_scrapper_amd import egress
    mk._RUN = egress.RunFiles('yahoo_ticker_matched_articles')
    t_all = time.perf_counter()
    c0 = time.perf_counter()
    for chunk in ingest.read_chunks(csv_path, args.chunksize):
        c1 = time.perf_counter(); t['read'] += c1 - c0
        n_chunks += 1
        if not isinstance(chunk, ingest.NativeChunk):
            matcher = mk._write_chunk('yahoo', chunk, processed, matcher)
            c0 = time.perf_counter(); t['write'] += c0 - c1
            continue
        n_native += 1
        dates, error = mk._dates(chunk.column_list('date_time'))
        c2 = time.perf_counter(); t['dates'] += c2 - c1
        if matcher is None:
            matcher = mk.get_matcher(processed, 0, mk._native_sample(chunk))
        c2 = time.perf_counter()
        arena, off = chunk.arena()
        off = off[:2 * len(dates) + 1]
        c3 = time.perf_counter(); t['arena'] += c3 - c2
        d_arena, d_off = matcher.upload(arena, off)
        matcher.scan(d_arena, d_off, len(dates))
        hits = matcher.fetch()
        c4 = time.perf_counter(); t['gpu_match'] += c4 - c3
        rendered, exc, _row = mk._native_rows(chunk, matcher, hits, dates, error)
        c5 = time.perf_counter(); t['render'] += c5 - c4
        egress.append_rendered('yahoo_ticker_matched_articles', rendered, mk._RUN)
        n_rows += sum(len(r[2]) for r in rendered)
        c0 = time.perf_counter(); t['write'] += c0 - c5
    c7 = time.perf_counter()
    import contextlib
    import io
    n_reread = 0
    with contextlib.redirect_stdout(io.StringIO()):
        for name in os.listdir('yahoo_ticker_matched_articles'):
            if not mk._RUN.finish(name):
                n_reread += 1
                mk.sort_matched_csv(f'yahoo_ticker_matched_articles/{name}')
    t['sort'] = time.perf_counter() - c7
    mk._RUN = None
    total = time.perf_counter() - t_all
    out = {'docs': args.docs, 'chunksize': args.chunksize, 'chunks': n_chunks, 'native_chunks': n_native,
           'rows': n_rows, 'files_reread_for_sort': n_reread, 'total_s': round(total, 3), 'articles_per_s': round(args.docs / total, 1),
           'phases_s': {k: round(v, 3) for k, v in t.items()}}
    print(json.dumps(out), flush=True)
    os.chdir(REPO)
    shutil.rmtree(work, ignore_errors=True)


if __name__ == '__main__':
    main()
