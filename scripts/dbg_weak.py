"""Debug aid: the weak-hash dedup path vs the oracle, row by row (prints the differing rows)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ['KW_TEST_HOOKS'] = '1'
os.environ['KW_TEST_DEDUP_WEAK_HASH'] = '1'
import numpy as np
from advanced_scrapper_amd import synth
from advanced_scrapper_amd.cdx_dedup import GpuUrlDedup, pack_urls
from oracle import dedup_oracle as dd
g = GpuUrlDedup()
urls = synth.generate_urls(3000, seed=4).urls()
arena, off = pack_urls(urls)
da, do = g.upload(arena, off)
code = g.run(da, do, len(urls)).cpu().numpy()
keys = [dd.url_transform(u) for u in urls]
kept = set(dd.keep_first(keys))
first = {}
for i, k in enumerate(keys):
    if k is not None:
        first.setdefault(k, i)
want = np.array([1 if i in kept else (0 if keys[i] is None and dd._HTML.search(urls[i]) is None
                                      else (2 if keys[i] is None else 3)) for i in range(len(urls))], np.uint8)
bad = np.flatnonzero(code != want)
print('counts', g.counts(), 'bad', len(bad))
for i in bad[:10]:
    k = keys[i]
    print(i, 'gpu', code[i], 'want', want[i], 'first', first.get(k), repr(urls[i])[:120], repr(k)[:100])
    f = first.get(k)
    if f is not None and f != i:
        print('   first row', f, 'gpu', code[f], repr(urls[f])[:120])
