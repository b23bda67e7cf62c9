"""Generate tests/golden/error_golden.json.gz: the reference's partial output when process_chunk raises.

Runs only in the build container, where /root/reference exists.  It imports
the reference's match_keywords.py (rapidfuzz stubbed by the oracle's
restatement, as make_golden.py does), runs ``process_chunk`` on small chunks
that raise mid-way, and stores the inputs, the per-ticker CSV bytes the
reference wrote before raising (no sort: the run aborts first) and the
exception class.  Nothing of the reference's source is copied.

Cases (match_keywords.py line numbers):
  invalid_regex  an in-period fuzzy name whose regex does not compile
                 ('Notepad++', ``multiple repeat`` in CPython 3.10) matches
                 article 2: re.finditer raises re.error at :178 while article
                 2's ticker_matches is built; articles 0-1 were appended.
  bad_date       article 3's date_time does not parse: dateutil raises at :152;
                 articles 0-2 were appended.
  int_dates      the chunk's date_time column is int64 (yyyymmdd): :152 parses
                 str(v), but :131 parser.parse(int) raises TypeError in the first
                 append_to_csv: nothing is written.
"""
from __future__ import annotations

import contextlib
import gzip
import io
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)


def _companies():
    return [
        {'id_label': 'Acme Corp', 'ticker': 'ACM', 'country': ['United States'], 'industry': [],
         'aliases': ['ACME', 'Acme Widgets Group'], 'products': ['Notepad++', 'Acme Rocket Skates'],
         'subsidiaries': [], 'owned_entities': [], 'ceos': ['Wile E. Coyote (Start: 1990-01-01T00:00:00Z)'],
         'board_members': []},
        {'id_label': 'Roadrunner Inc', 'ticker': 'RRN', 'country': ['United States'], 'industry': [],
         'aliases': ['RRN', 'Roadrunner Holdings'], 'products': ['Birdseed Deluxe'], 'subsidiaries': [],
         'owned_entities': [], 'ceos': [], 'board_members': []},
    ]


def _articles(case):
    texts = [
        'ACME shares rose as Acme Widgets Group unveiled Acme Rocket Skates.',
        'Roadrunner Holdings (RRN) sold Birdseed Deluxe; ACME fell.',
        'The Notepad++ editor shipped; ACME and RRN were unmoved.',
        'Wile E. Coyote ordered more Acme Rocket Skates from ACME.',
        'RRN guided higher; Roadrunner Holdings beat estimates.',
        'Nothing relevant here at all.',
    ]
    dates = [f'2021-03-0{i + 1} 10:00:00' for i in range(len(texts))]
    if case == 'invalid_regex':
        pass
    elif case == 'bad_date':
        texts[2] = 'The editor shipped; ACME and RRN were unmoved.'
        dates[3] = 'not a date at all'
    elif case == 'int_dates':
        texts[2] = 'The editor shipped; ACME and RRN were unmoved.'
        dates = [20210301 + i for i in range(len(texts))]
    rows = []
    for i, (t, d) in enumerate(zip(texts, dates)):
        rows.append({'article_text': t, 'title': f'Headline {i}', 'date_time': d,
                     'url': f'https://example.invalid/e/{i}.html', 'source': 'yahoo',
                     'source_url': 'https://finance.yahoo.com'})
    return rows


def main():
    os.environ['TZ'] = 'UTC'
    time.tzset()
    from make_golden import _stub_rapidfuzz
    _stub_rapidfuzz()
    sys.path.insert(0, REF)
    import match_keywords as ref      # the reference, imported (not copied)
    import pandas as pd
    with contextlib.redirect_stdout(io.StringIO()):
        processed = ref.process_json_data(_companies())

    def iso(d):
        return None if d is None else d.isoformat()
    kb = [[t, [[a, [[n, iso(s), iso(e)] for n, (s, e) in names.items()]] for a, names in attrs.items()]]
          for t, attrs in processed.items()]
    cases = {}
    for case in ('invalid_regex', 'bad_date', 'int_dates'):
        csv_bytes = pd.DataFrame(_articles(case)).to_csv(index=False).encode('utf-8')
        with tempfile.TemporaryDirectory() as tmp:
            cwd = os.getcwd()
            os.chdir(tmp)
            try:
                with open('articles.csv', 'wb') as fh:
                    fh.write(csv_bytes)
                os.makedirs('yahoo_ticker_matched_articles')
                exc_name = None
                try:
                    with contextlib.redirect_stdout(io.StringIO()):
                        for chunk in pd.read_csv('articles.csv', chunksize=100):
                            ref.process_chunk('yahoo', chunk, processed)
                except Exception as exc:   # noqa: BLE001 - recorded as the expected outcome
                    exc_name = type(exc).__name__
                files = {}
                for fn in sorted(os.listdir('yahoo_ticker_matched_articles')):
                    with open(os.path.join('yahoo_ticker_matched_articles', fn), 'rb') as fh:
                        files[fn] = fh.read().decode('utf-8')
            finally:
                os.chdir(cwd)
        cases[case] = {'articles_csv': csv_bytes.decode('utf-8'), 'files': files, 'exception': exc_name}
        print(case, exc_name, {k: v.count('\n') - 1 for k, v in files.items()})
    out = {'reference': 'lwowlwowl/advanced_scrapper match_keywords.py process_chunk (imported, rapidfuzz '
                        'stubbed by the oracle)', 'kb_processed': kb, 'chunksize': 100, 'cases': cases}
    with open(os.path.join(HERE, 'error_golden.json.gz'), 'wb') as fh:
        fh.write(gzip.compress(json.dumps(out, sort_keys=True).encode(), mtime=0))


if __name__ == '__main__':
    main()
