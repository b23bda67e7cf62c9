"""The CDX-dedup oracle (oracle/dedup_oracle.py) against the reference's own outputs.

tests/golden/dedup_golden.json.gz was produced by running yahoo_links_selenium.py
itself (tests/golden/make_dedup_golden.py): per-part CSVs (:59-82) and the
merged yfin_urls.csv (:160-179).
"""
import gzip
import io
import json
import os

import pandas as pd
import pytest

from oracle import dedup_oracle as dd

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'dedup_golden.json.gz')


@pytest.fixture(scope='module')
def gold():
    with gzip.open(GOLD, 'rt', encoding='utf-8') as f:
        return json.load(f)


def test_part_csvs_match_reference(gold):
    for p in gold['parts']:
        assert dd.part_csv_bytes(dd.cdx_part(gold['cdx'][p])).decode() == gold['part_csv'][p], p


def test_merge_matches_reference(gold):
    order = [n[len('yahoo_'):-len('.csv')] for n in gold['glob_order']]
    merged = dd.merge_parts(gold['part_csv'][p].encode() for p in order)
    assert merged.to_csv(index=False) == gold['merged_csv']


def test_rowwise_restatement_matches_reference(gold):
    """url_transform + keep_first over the rows in glob order == the reference's merged rows."""
    order = [n[len('yahoo_'):-len('.csv')] for n in gold['glob_order']]
    ts, urls = [], []
    for p in order:
        t, u = dd.parse_cdx(gold['cdx'][p])
        ts += t
        urls += u
    kept, keys = dd.dedup_rows(urls)
    want = pd.read_csv(io.StringIO(gold['merged_csv']))
    assert keys == want['url'].tolist()
    assert [ts[i] for i in kept] == want['date_time'].tolist()


@pytest.mark.parametrize('url,want', [
    ('https://finance.yahoo.com/news/a-1.html', 'https://finance.yahoo.com/news/a-1.html'),
    ('http://finance.yahoo.com:80/news/a-1.html?x=1', 'https://finance.yahoo.com/news/a-1.html'),
    ('https://finance.yahoo.com/news/a-1xhtml', 'https://finance.yahoo.com/news/a-1.html'),   # '.' = any char
    ('https://finance.yahoo.com/news/a-1éhtml', 'https://finance.yahoo.com/news/a-1.html'),   # one code point
    ('https://finance.yahoo.com/news/a-1.htm', None),
    ('https://finance.yahoo.com/news/%20a.html', None),
    ("https://finance.yahoo.com/news/'a.html", None),
    ('https://finance.yahoo.com/news/:80%a.html', None),             # ':80' removal creates 'news/%'
    ('htt:80p://x.com/a.html', 'https://x.com/a.html'),                # removal creates 'http:'
    ('html.html', 'html.html'),                                        # first match needs a code point before
    ('\nhtml', None),                                                  # '.' does not match '\n'
    ('a\nhtmlbhtml', 'a\nhtml.html'),                                # the first 'html' has '\n' before it
    (':8:800.html', ':80.html'),                                       # one left-to-right pass
    ('x:80:80.html', 'x.html'),
    ('http:http:a.html', 'https:https:a.html'),
])
def test_url_transform_rules(url, want):
    assert dd.url_transform(url) == want
    # the pandas calls of the reference agree
    s = pd.Series([url])
    s = s[s.str.contains('.html')]
    s = s.str.split('.html').str[0] + '.html'
    s = s.str.replace(':80', '', regex=False).str.replace('http:', 'https:', regex=False)
    s = s[~s.str.contains('news/%')]
    s = s[~s.str.contains("news/'")]
    assert (s.tolist() or [None])[0] == want
