"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline).

The product (advanced_scrapper_amd/) never imports this module.

CPU restatement of the CDX link-parts normalise + keep-first dedup of the
reference (lwowlwowl/advanced_scrapper yahoo_links_selenium.py):

* ``cdx_part``        <- :59-79   one ``yahoo_XY.txt`` CDX listing -> the rows of ``yahoo_XY.csv``
* ``merge_parts``     <- :160-174 concat of the part CSVs in glob order, keep-first again
* ``url_transform``   <- :63-68   per-URL rule, restated without pandas (used to check the GPU
                                  transform row by row and to time the CPU baseline)
* ``keep_first``      <- :79/:174 ``drop_duplicates(subset=['url'])`` (keep='first')

``cdx_part`` / ``merge_parts`` run pandas exactly the way the reference does
(same calls, same order, same defaults); ``url_transform`` restates the rules
those pandas calls implement:

  contains('.html')   regex: some "html" preceded by one code point that is not '\\n'
  split('.html').str[0] + '.html'
                      pandas 2.x treats a pattern longer than one character as a
                      regex, so the URL is cut at the start of the code point
                      before the first such "html"
  replace(':80', '')  literal, every non-overlapping occurrence, left to right
  replace('http:', 'https:')  literal, on the result of the previous replace
  ~contains('news/%') / ~contains("news/'")  literal substrings (no metacharacters)

Parity status: pinned by tests/golden/dedup_golden.json.gz, produced by running
the reference's own ``scrape_article_content`` and ``__main__`` merge block in
the build container (tests/golden/make_dedup_golden.py).
"""
from __future__ import annotations

import io
import re
from typing import Iterable, List, Optional, Sequence, Tuple

_HTML = re.compile('.html')


def url_transform(url: str) -> Optional[str]:
    """The normalised URL of one CDX row, or None when the row is dropped
    (no '.html' match, or a 'news/%' / "news/'" URL after the rewrite)."""
    m = _HTML.search(url)
    if m is None:
        return None
    s = url[:m.start()] + '.html'
    s = s.replace(':80', '')
    s = s.replace('http:', 'https:')
    if 'news/%' in s or "news/'" in s:
        return None
    return s


def url_transform_bytes(url: bytes) -> Optional[bytes]:
    """Byte-level form of url_transform for UTF-8 input (what the GPU kernel computes)."""
    r = url_transform(url.decode('utf-8', 'surrogatepass'))
    return None if r is None else r.encode('utf-8', 'surrogatepass')


def keep_first(keys: Sequence[Optional[str]]) -> List[int]:
    """Indices kept by drop_duplicates(keep='first') over the non-None keys, in order."""
    seen = set()
    out = []
    for i, k in enumerate(keys):
        if k is None or k in seen:
            continue
        seen.add(k)
        out.append(i)
    return out


def dedup_rows(urls: Sequence[str]) -> Tuple[List[int], List[str]]:
    """Global keep-first over the transformed URLs of rows in order: (kept row
    indices, their normalised URLs).  Equal to cdx_part on every part followed by
    merge_parts, because the first occurrence of a URL in the concatenation is
    also the first in its own part."""
    keys = [url_transform(u) for u in urls]
    kept = keep_first(keys)
    return kept, [keys[i] for i in kept]


# ------------------------------------------------------------------ pandas forms (the reference's calls)
def cdx_part(cdx_text: str):
    """yahoo_links_selenium.py:59-79 on the text of one CDX listing -> DataFrame(date_time, url)."""
    import pandas as pd
    df = pd.read_csv(io.StringIO(cdx_text), delimiter=' ', header=None, usecols=[1, 2], names=['date_time', 'url'])
    df = df[df['url'].str.contains('.html')]
    df['url'] = df['url'].str.split('.html').str[0] + '.html'
    df['url'] = df['url'].str.replace(':80', '', regex=False)
    df['url'] = df['url'].str.replace('http:', 'https:', regex=False)
    df = df[~df['url'].str.contains('news/%')]
    df = df[~df['url'].str.contains("news/'")]
    df.drop_duplicates(subset=['url'], inplace=True)
    return df


def part_csv_bytes(df) -> bytes:
    """:82 ``df.to_csv(output_filename, index=False)``."""
    return df.to_csv(index=False).encode('utf-8')


def merge_parts(part_csvs: Iterable[bytes]):
    """:164-174: read every part CSV (glob order given by the caller), concat, keep-first."""
    import pandas as pd
    dfs = [pd.read_csv(io.BytesIO(b)) for b in part_csvs]
    merged = pd.concat(dfs, ignore_index=True)
    merged.drop_duplicates(subset=['url'], inplace=True)
    return merged


def parse_cdx(cdx_text: str) -> Tuple[List[int], List[str]]:
    """The two columns the reference reads (:59), via the same pandas call."""
    import pandas as pd
    df = pd.read_csv(io.StringIO(cdx_text), delimiter=' ', header=None, usecols=[1, 2], names=['date_time', 'url'])
    return df['date_time'].tolist(), df['url'].tolist()
