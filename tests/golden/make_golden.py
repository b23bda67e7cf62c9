"""Generate the golden fixtures by running the REFERENCE match_keywords.py.

Runs only in the build container, where /root/reference exists (it does not
exist on the GPU box; the committed fixtures travel instead).  Nothing of the
reference's source is copied: the script imports it, runs it, and stores
inputs and outputs as data.

rapidfuzz (requirements.txt:5, unpinned) is not installed anywhere in the
image, so ``rapidfuzz.fuzz.partial_ratio`` is injected as a stub returning
100.0 / 0.0 from the oracle's restatement (oracle/partial_ratio.c,
``pr_decide``).  The reference only consumes ``partial_ratio(...) > 95``
(match_keywords.py:175-176), so the stub is exact for it.  Everything else —
KB parsing and ordering, the period filter, ``\\b`` and regex positions via
CPython ``re``, dict/JSON ordering, CSV bytes and the final sort — is the
reference's own code.

Pinning protocol: single process, process_chunk called chunk
by chunk in file order (no Pool races), fresh output directory, TZ=UTC,
unique article timestamps, os.listdir order of the KB recorded.

Outputs (tests/golden/):
  kb_bundle.json.gz      raw text of every info/ticker/*.json + listdir order
  kb_processed.json.gz   the reference's processed_data (periods as ISO strings)
  articles.csv.gz        the article CSV the reference read
  matches.jsonl.gz       per article row: the ticker_matches the reference built
  out_c1.tar.gz          the per-ticker CSVs after sort_matched_csv
  MANIFEST.json          sizes, counts, sha256
"""
from __future__ import annotations

import contextlib
import gzip
import hashlib
import io
import json
import os
import sqlite3
import sys
import tarfile
import tempfile
import time
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)

CHUNKSIZE = 400
N_SYNTH = 600
SEED = 20250905


def _stub_rapidfuzz():
    from oracle import kwmatch_oracle as orc

    def partial_ratio(s1, s2, *a, **k):
        return 100.0 if orc.partial_ratio_gt95(s1, s2) else 0.0
    mod = types.ModuleType('rapidfuzz')
    mod.fuzz = types.SimpleNamespace(partial_ratio=partial_ratio)
    sys.modules['rapidfuzz'] = mod


def _adversarial():
    """Hand-made rows that hit the edge cases of SURVEY.md §8(a)."""
    A = []

    def add(text, title, date=''):
        if date == '':   # unique default timestamps (the final sort is unstable)
            date = f'2015-06-01 12:{len(A):02d}:00'
        A.append((text, title, date))
    add("ESPN+X streams. ESPN+ app. The ESPN+ bundle, ESPN+1 and ESPN+_ too.", "ESPN+ deal")
    add("xAAPL AAPL_ AAPL's (AAPL) éAAPL AAPLé 中AAPL中 ÉAAPL AAPL. AAPL", "AAPL beats")
    add("ADOBE INC.X and ADOBE INC. later; ADOBE INC.", "ADOBE INC.")
    add("Apple Computer Inc, said. Apple Computer Inc. said. Apple Computer Inc\nsaid.", "Apple Computer In")
    add("Disney+ Hotstar and Disneyyy Hotstar and Disney Hotstar launched.", "Disney+ Hotstar")
    add("Adobe Systems Software(Beijing)Co.,Ltd. reported; Adobe Systems SoftwareBeijingCo.,Ltd! too.",
        "Adobe Systems SoftwareBeijingCo,Ltd")
    add("pple Computer Inc. opened the session higher", "Walt Disney Music Compan")
    add("the session closed lower for Apple Computer In", "Andrés R. Gluski")
    add("Andres R. Gluski and Andrés R. Gluski spoke; Moisés Naím too", "Thomas F. O’Toole")
    add("Walt Disney Parks and Resort U.S. and Walt Disney Parks and Resorts U.S. expanded",
        "Walt Disney Parks and Resorts U.S.")
    add("Walt Disney Parks and Resortz US expanded; Walt Disnep Parks and Resorts U.S expanded", "nan")
    add("nan", "nan")
    add("Caesars Entertainment, Inc. and Caesars Entertainment Inc and Caesars Entertainmen, Inc.", "Eldorado Resorts, Inc.")
    add("Steve Jobs returned to Apple; Tim Cook commented.", "Steve Jobs", date='1999-01-01 00:00:00')
    add("Steve Jobs returned to Apple; Tim Cook commented.", "Steve Jobs", date='2020-01-01 00:00:00')
    add("Steve Jobs returned to Apple; Tim Cook commented.", "Steve Jobs", date='1975-01-01 00:00:00')
    add("no date here Apple Inc. AAPL", "no date", date=None)
    add("thewaltdisneycompany.com and thewaltdisneycompanyXcom and babble.com babbleXcom", "spoonful.com")
    add("Euro Disney S.C.A. and Euro Disney SxCxAx and Euro Disney S C A", "Roy O. Disney")
    add("AT&T and T-Mobile; AT&Tx; xAT&T", "IBM, GE, HP and 3M")
    add("Coca-Cola İçecek sales; Coca-Cola Icecek; Estée Lauder Companies; Estee Lauder Companies", "Ørsted")
    add("Accenture Central Europe B.V., organizační složka and Accenture Central Europe B.V., organizacni slozka",
        "Chevron México")
    add("“Apple Inc.” said — ‘Microsoft’ — and AMAZON.COM too", "Amazon.com, Inc.")
    add("Walt Disney Company", "The Walt Disney Company")
    add("The Walt Disney Compan", "he Walt Disney Company")
    return A


def _real_articles():
    path = os.path.join(REF, 'experiental', 'crypto_news.db')
    con = sqlite3.connect(f'file:{path}?mode=ro', uri=True)
    rows = con.execute('select title, content, datetime_utc, url from articles order by url').fetchall()
    con.close()
    return [(c, t, str(d)[:19] if d else None, u) for (t, c, d, u) in rows]


def main():
    os.environ['TZ'] = 'UTC'
    time.tzset()
    _stub_rapidfuzz()
    sys.path.insert(0, REF)
    import match_keywords as ref      # the reference, imported (not copied)
    import pandas as pd
    from advanced_scrapper_amd import synth
    from advanced_scrapper_amd.kb import compile_kb

    kb_dir = os.path.join(REF, 'info', 'ticker')
    listdir = os.listdir(kb_dir)
    files = {}
    for fn in listdir:
        with open(os.path.join(kb_dir, fn), 'rb') as fh:
            files[fn] = fh.read().decode('utf-8')
    with contextlib.redirect_stdout(io.StringIO()):
        processed = ref.read_and_process_json_files(kb_dir)

    def iso(d):
        return None if d is None else d.isoformat()
    kb_proc = [[t, [[a, [[n, iso(s), iso(e)] for n, (s, e) in names.items()]] for a, names in attrs.items()]]
               for t, attrs in processed.items()]

    # ---- corpus: synthetic + adversarial + real
    ckb = compile_kb(processed)
    names, kinds = synth.injectable_names(ckb)
    corpus = synth.generate(N_SYNTH, names, kinds, seed=SEED)
    df = synth.to_dataframe(corpus)
    extra = []
    for i, (text, title, date) in enumerate(_adversarial()):
        extra.append({'article_text': text, 'title': title, 'date_time': date,
                      'url': f'https://example.invalid/adv/{i}.html', 'source': 'yahoo',
                      'source_url': 'https://finance.yahoo.com'})
    for i, (text, title, date, url) in enumerate(_real_articles()):
        extra.append({'article_text': text, 'title': title, 'date_time': date, 'url': url, 'source': 'yahoo',
                      'source_url': 'https://finance.yahoo.com'})
    df = pd.concat([df, pd.DataFrame(extra)], ignore_index=True)
    # unique timestamps for the unstable sort (keep adversarial dates that test periods)
    csv_bytes = df.to_csv(index=False).encode('utf-8')

    captured = {}
    orig_append = ref.append_to_csv

    def recording_append(source_name, ticker, matched_names, article):
        captured.setdefault(int(article.name), {})[ticker] = json.loads(json.dumps(matched_names))
        return orig_append(source_name, ticker, matched_names, article)
    ref.append_to_csv = recording_append

    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, 'articles.csv')
        with open(src, 'wb') as fh:
            fh.write(csv_bytes)
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            os.makedirs('yahoo_ticker_matched_articles', exist_ok=True)
            t0 = time.time()
            with contextlib.redirect_stderr(io.StringIO()), contextlib.redirect_stdout(io.StringIO()):
                for chunk in pd.read_csv('articles.csv', chunksize=CHUNKSIZE):
                    ref.process_chunk('yahoo', chunk, processed)
                out_listdir = os.listdir('yahoo_ticker_matched_articles')
                for fn in out_listdir:
                    ref.sort_matched_csv(f'yahoo_ticker_matched_articles/{fn}')
            elapsed = time.time() - t0
            tar_buf = io.BytesIO()
            with tarfile.open(fileobj=tar_buf, mode='w:gz') as tar:
                for fn in sorted(out_listdir):
                    tar.add(os.path.join('yahoo_ticker_matched_articles', fn), arcname=fn)
        finally:
            os.chdir(cwd)

    n_rows = len(df)
    outs = {
        'kb_bundle.json.gz': gzip.compress(json.dumps({'listdir': listdir, 'files': files}).encode(), mtime=0),
        'kb_processed.json.gz': gzip.compress(json.dumps(kb_proc).encode(), mtime=0),
        'articles.csv.gz': gzip.compress(csv_bytes, mtime=0),
        'matches.jsonl.gz': gzip.compress('\n'.join(json.dumps(captured.get(i, {})) for i in range(n_rows)).encode(),
                                          mtime=0),
        'out_c1.tar.gz': tar_buf.getvalue(),
    }
    manifest = {'reference': 'lwowlwowl/advanced_scrapper match_keywords.py (imported, rapidfuzz stubbed by oracle)',
                'rows': n_rows, 'synthetic_rows': N_SYNTH, 'seed': SEED, 'chunksize': CHUNKSIZE,
                'rows_with_matches': len(captured), 'tickers_written': len(out_listdir),
                'reference_seconds': round(elapsed, 1), 'files': {}}
    for name, data in outs.items():
        with open(os.path.join(HERE, name), 'wb') as fh:
            fh.write(data)
        manifest['files'][name] = {'bytes': len(data), 'sha256': hashlib.sha256(data).hexdigest()}
    with open(os.path.join(HERE, 'MANIFEST.json'), 'w') as fh:
        json.dump(manifest, fh, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == '__main__':
    main()
