"""End-to-end drop-in timing: match_keywords' per-chunk host phases around the GPU scan.

Generates N synthetic articles (config-2 corpus), writes them as the reference's article CSV, then runs the
drop-in main loop's phases on chunks of 20 000 rows and prints one JSON line with seconds per phase and the
end-to-end articles/s (the reference's CPU path on the same rows is bench.py's cpu_baseline).

    python scripts/e2e.py [--docs 100000] [--chunksize 20000]
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
    ap.add_argument('--docs', type=int, default=100000)
    ap.add_argument('--chunksize', type=int, default=20000)
    args = ap.parse_args()
    import pandas as pd
    from advanced_scrapper_amd import match_keywords as mk, synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import field_str
    from advanced_scrapper_amd.rows import assemble_json_rows
    from advanced_scrapper_amd.dates import parse_date
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
    t = dict(read=0.0, prep=0.0, dates=0.0, gpu_match=0.0, assemble=0.0, rows=0.0, write=0.0)
    matcher = None
    n_rows = 0
    t_all = time.perf_counter()
    c0 = time.perf_counter()
    for chunk in pd.read_csv(csv_path, chunksize=args.chunksize):
        c1 = time.perf_counter(); t['read'] += c1 - c0
        texts = [field_str(v) for v in chunk['article_text'].tolist()]
        titles = [field_str(v) for v in chunk['title'].tolist()]
        c2 = time.perf_counter(); t['prep'] += c2 - c1
        dates = [parse_date(str(v)) if pd.notna(v) else None for v in chunk['date_time'].tolist()]
        c3 = time.perf_counter(); t['dates'] += c3 - c2
        if matcher is None:
            matcher = mk.get_matcher(processed, 0, texts)
        c3 = time.perf_counter()
        hits = matcher.match_strings(texts, titles)
        c4 = time.perf_counter(); t['gpu_match'] += c4 - c3
        cells = assemble_json_rows(matcher.ckb, hits, dates)
        c5 = time.perf_counter(); t['assemble'] += c5 - c4
        by, _err = mk._cell_rows(chunk, cells, dates)
        c6 = time.perf_counter(); t['rows'] += c6 - c5
        for ticker, rows in by.items():
            mk._append_rows('yahoo', ticker, rows)
            n_rows += len(rows)
        c0 = time.perf_counter(); t['write'] += c0 - c6
    total = time.perf_counter() - t_all
    out = {'docs': args.docs, 'chunksize': args.chunksize, 'rows': n_rows, 'total_s': round(total, 3),
           'articles_per_s': round(args.docs / total, 1), 'phases_s': {k: round(v, 3) for k, v in t.items()}}
    print(json.dumps(out), flush=True)
    os.chdir(REPO)
    shutil.rmtree(work, ignore_errors=True)


if __name__ == '__main__':
    main()
