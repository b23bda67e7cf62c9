"""The output sort at scale: ``match_keywords.main`` end to end on articles whose dates are NOT in article order.

tests/test_gpu_c3_csv.py pins every row at 10M articles, but its dates increase with the article, so the
reference's ``sort_matched_csv`` (match_keywords.py:195-217) leaves every file as appended and the product's
sort (egress.RunFiles: the time index of the rows it wrote, np.argsort quicksort = pandas' nargsort) is never
asked to move a row there.  Here the same generator's first documents get a seeded permutation of the same
unique dates (make_n1_digests.py --perm, synth.to_dataframe ``date_perm``), written as ONE article CSV of
the reference's schema; the drop-in's ``main()`` reads it in 20 000-row chunks (:227), matches on the GPU,
appends, and sorts the files it created.  Every final per-ticker file must equal, byte for byte (sha256 and
size), the file the reference's own ``sort_matched_csv`` produced from the oracle's appended rows in the build
container (tests/golden/c3_csv_perm.json).
"""
import contextlib
import hashlib
import io
import json
import os
import time

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(__file__), 'golden')
FIX = os.path.join(HERE, 'c3_csv_perm.json')


@pytest.mark.skipif(not os.path.exists(FIX), reason='tests/golden/c3_csv_perm.json not made')
def test_sort_out_of_order_dates_vs_reference_sort(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    import bench
    from advanced_scrapper_amd import match_keywords as mk
    from tests.golden.make_n1_digests import CHUNK, chunk_csv_bytes, _names_kinds
    meta = json.load(open(FIX))
    assert meta['date_perm'] and meta['chunk_rows'] == CHUNK
    files = meta['files']
    # the fixture is a real test of the sort: most files are reordered by the reference's sort
    assert meta['files_sorted_unchanged'] < meta['n_files'] // 2, meta['files_sorted_unchanged']
    n_docs = meta['n_docs']
    t0 = time.time()
    nk = _names_kinds()
    csv_path = tmp_path / 'articles.csv'
    chain = hashlib.sha256()
    with open(csv_path, 'wb') as fh:
        for lo in range(0, n_docs, CHUNK):
            data = chunk_csv_bytes(lo, CHUNK, nk, perm=True)
            chain.update(hashlib.sha256(data).digest())
            fh.write(data if lo == 0 else data[data.index(b'\n') + 1:])   # one CSV: the header once
    assert chain.hexdigest() == meta['csv_chain_sha256'], 'the article CSVs differ from the ones the oracle read'
    t1 = time.time()
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        bench.load_kb(str(tmp_path / 'ticker'))           # the reference's KB files, materialised
        with contextlib.redirect_stdout(io.StringIO()):
            rc = mk.main(['--info-dir', str(tmp_path / 'ticker'), '--articles', str(csv_path), '--device', '0'])
        assert rc in (0, None)
        out = tmp_path / 'yahoo_ticker_matched_articles'
        got = sorted(os.listdir(out))
        assert got == sorted(files), (set(got) ^ set(files))
        bad = []
        for name in got:
            data = (out / name).read_bytes()
            if (hashlib.sha256(data).hexdigest(), len(data)) != (files[name]['sorted_sha256'],
                                                                 files[name]['sorted_bytes']):
                bad.append(name)
        assert not bad, f'{len(bad)} of {len(got)} sorted files differ from the reference sort: {bad[:10]}'
    finally:
        os.chdir(cwd)
    print(f'{n_docs} articles, {len(files)} files ({meta["n_files"] - meta["files_sorted_unchanged"]} reordered by '
          f'the sort) equal the reference sort; CSV {t1 - t0:.0f} s, main {time.time() - t1:.0f} s')
