"""Generate the CDX-dedup golden fixture by running the REFERENCE yahoo_links_selenium.py.

Runs only in the build container, where /root/reference exists (the GPU box
gets the committed fixture instead).  Nothing of the reference's source is
copied: the script imports and runs it, and stores inputs and outputs as data.

selenium and bs4 are not installed in the image and sit outside the dedup
path, so they are injected as stubs: the fake driver "loads" a synthetic CDX
listing and the BeautifulSoup stub returns it as text (the listing holds no
markup; ``get_text(separator='\\n', strip=True)`` of a tag-free page is the
stripped text).  Everything on the path is the reference's own code:

* ``scrape_article_content`` (yahoo_links_selenium.py:38-88) writes
  ``yahoo_links_1/yahoo_XY.txt``, reads it with pandas, filters / rewrites /
  dedups (:59-79) and writes ``yahoo_XY.csv`` (:82);
* the ``__main__`` block (:129-182) with every CDX prefix already scraped
  (so no driver starts) merges the part CSVs in glob order and keeps the first
  of every URL (:160-179), writing ``yfin_urls.csv``.

Output: tests/golden/dedup_golden.json.gz with the CDX listings, the part CSVs,
the glob order and the merged CSV (as text).
"""
from __future__ import annotations

import glob
import gzip
import importlib.util
import json
import os
import runpy
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference/yahoo_links_selenium.py'
sys.path.insert(0, REPO)

SEED = 20250905
PARTS = ('ab', 'q7', '-_')          # three CDX prefixes (their listings overlap in articles)
ROWS_PER_PART = 2500


def _stubs():
    class Options:
        def set_preference(self, *a, **k):
            pass

        def add_argument(self, *a, **k):
            pass

    class Service:
        def __init__(self, *a, **k):
            pass

    class WebDriverWait:
        def __init__(self, driver, timeout):
            self.driver = driver

        def until(self, cond):
            return cond(self.driver)

    class BeautifulSoup:
        def __init__(self, page, parser=None):
            self.page = page

        def get_text(self, separator='', strip=False):
            return self.page.strip() if strip else self.page

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mod('selenium')
    mod('selenium.webdriver', Firefox=None)
    mod('selenium.webdriver.firefox')
    mod('selenium.webdriver.firefox.service', Service=Service)
    mod('selenium.webdriver.firefox.options', Options=Options)
    mod('selenium.webdriver.support')
    mod('selenium.webdriver.support.ui', WebDriverWait=WebDriverWait)
    mod('selenium.webdriver.support.expected_conditions')
    sys.modules['selenium'].webdriver = sys.modules['selenium.webdriver']
    mod('bs4', BeautifulSoup=BeautifulSoup)


class FakeDriver:
    def __init__(self, page):
        self.page_source = page

    def get(self, url):
        pass

    def execute_script(self, script):
        return 'complete'


def main():
    from advanced_scrapper_amd import synth
    _stubs()
    rows = synth.generate_urls(ROWS_PER_PART * len(PARTS), seed=SEED)
    cdx = {p: rows.cdx_text(k * ROWS_PER_PART, (k + 1) * ROWS_PER_PART) for k, p in enumerate(PARTS)}
    chars = [c for c in 'abcdefghijklmnopqrstuvwxyz1234567890-_$']
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            os.makedirs('yahoo_links_1')
            # every prefix counts as scraped, so the reference's __main__ starts no driver
            for a in chars:
                for b in chars:
                    open(f'yahoo_links_1/yahoo_{a}{b}.txt', 'w').close()
            spec = importlib.util.spec_from_file_location('yahoo_links_selenium_ref', REF)
            ref = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(ref)
            for p in PARTS:
                url = f'http://web.archive.org/cdx/search/?url=https://www.finance.yahoo.com/news/{p}*'
                ref.scrape_article_content(url, FakeDriver(cdx[p]))
                assert os.path.exists(f'yahoo_links_1/yahoo_{p}.csv'), p
            part_csv = {p: open(f'yahoo_links_1/yahoo_{p}.csv', encoding='utf-8').read() for p in PARTS}
            glob_order = [os.path.basename(f) for f in glob.glob(os.path.join('yahoo_links_1', '*.csv'))]
            runpy.run_path(REF, run_name='__main__')
            merged = open('yfin_urls.csv', encoding='utf-8').read()
        finally:
            os.chdir(cwd)
    out = {'seed': SEED, 'parts': list(PARTS), 'rows_per_part': ROWS_PER_PART, 'cdx': cdx, 'part_csv': part_csv,
           'glob_order': glob_order, 'merged_csv': merged,
           'generator': 'advanced_scrapper_amd.synth.generate_urls(n, seed) rows split into equal parts'}
    path = os.path.join(HERE, 'dedup_golden.json.gz')
    with gzip.open(path, 'wt', encoding='utf-8') as f:
        json.dump(out, f)
    print(path, {p: len(v.splitlines()) - 1 for p, v in part_csv.items()}, 'merged', len(merged.splitlines()) - 1,
          'glob', glob_order)


if __name__ == '__main__':
    main()
