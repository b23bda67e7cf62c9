"""Multi-process (world_size 2, gloo on CPU) coverage of the sharded path.

The GPU run uses the same functions over RCCL (backend "nccl"); here the
collectives run over gloo so the N > 1 logic is exercised without a GPU:
contiguous byte-balanced shards, the hit-count all-gather and the padded
all-gather of packed hit records, whose rank-order concatenation must equal
the single-process result in document order.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _fake_hits(lo: int, hi: int) -> np.ndarray:
    """Deterministic [n, 4] int32 records for documents [lo, hi) (doc ids local to the shard)."""
    rows = []
    for d in range(lo, hi):
        for k in range(d % 3):                 # 0, 1 or 2 hits per document: ragged ranks
            rows.append((d - lo, 7 * d + k, k, d & 1))
    return np.asarray(rows, dtype=np.int32).reshape(-1, 4)


def _worker(rank, world, port, off, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from advanced_scrapper_amd import dist
    r, w, _ = dist.init('gloo')
    assert (r, w) == (rank, world)
    lo, hi = dist.byte_balanced_ranges(off, world)[rank]
    local = torch.from_numpy(_fake_hits(lo, hi))
    counts = dist.allgather_counts(local.shape[0], torch.device('cpu'))
    allh = dist.gather_hits(local, lo, torch.device('cpu'))
    q.put((rank, counts, allh.numpy().tolist()))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def _run(world, off):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, off, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_gloo_sharded_gather_equals_single_process():
    from advanced_scrapper_amd import dist
    world = 2
    rng = np.random.default_rng(3)
    n_docs = 97
    lens = rng.integers(0, 5000, size=2 * n_docs)
    off = np.zeros(2 * n_docs + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    ranges = dist.byte_balanced_ranges(off, world)
    res = _run(world, off)
    want_counts = [len(_fake_hits(lo, hi)) for lo, hi in ranges]
    exp = []
    for lo, hi in ranges:
        h = _fake_hits(lo, hi)
        h[:, 0] += lo
        exp.append(h)
    exp = np.concatenate(exp)
    single = _fake_hits(0, n_docs)          # one process over every document (global doc ids)
    assert np.array_equal(exp, single)
    for rank, counts, allh in res:
        assert counts == want_counts, rank
        got = np.asarray(allh, dtype=np.int32).reshape(-1, 4)
        assert np.array_equal(got, single), rank


def _main_worker(rank, world, port, work, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TZ='UTC')
    import time
    time.tzset()
    from advanced_scrapper_amd import dist
    from advanced_scrapper_amd import match_keywords as mk
    from tests import golden_data
    dist.init('gloo')
    os.chdir(work)
    processed = golden_data.kb_processed()
    mk.read_and_process_json_files = lambda _d: processed      # the golden KB (fixed ticker order)
    args = mk._parse(['--info-dir', 'unused', '--articles', os.path.join(work, 'articles.csv'),
                      '--chunksize', str(golden_data.chunksize()), '--gpus', str(world)])
    from tests.oracle_matcher import OracleMatcher
    m = OracleMatcher(processed)
    rereads = []
    real_sort = mk.sort_matched_csv
    mk.sort_matched_csv = lambda path: (rereads.append(path), real_sort(path))
    rc = mk.run(args, rank, world, None, 'gloo', matcher=m)
    q.put((rank, rc, (m.uploads, rereads)))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_gloo_main_sharded_equals_reference_outputs(tmp_path):
    """match_keywords.main's multi-rank loop (byte-balanced row shards of every chunk, the records moved to
    rank 0, rank 0 writes and sorts) over 2 gloo ranks, with only the scan stubbed by the oracle, writes the
    reference's own per-ticker files byte for byte (tests/golden/out_c1)."""
    from tests import golden_data
    (tmp_path / 'articles.csv').write_bytes(golden_data.articles_csv_bytes())
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_main_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r, rc) for r, rc, _u in res] == [(0, 0), (1, 0)]
    # every output file was sorted from the ranks' merged write index (egress.RunFiles), none re-read
    assert [u[1] for _r, _rc, u in res] == [[], []]
    # each rank packed and scanned only its own byte-balanced share of every chunk
    n_rows = len(golden_data.articles_frame())
    chunk = golden_data.chunksize()
    ups = [u[0] for _r, _rc, u in res]
    assert all(len(u) == -(-n_rows // chunk) for u in ups)
    for c, size in enumerate([min(chunk, n_rows - k) for k in range(0, n_rows, chunk)]):
        shares = [u[c][0] for u in ups]
        assert sum(shares) == size, (c, shares)
        assert all(0 < s < size for s in shares), (c, shares)
        nbytes = [u[c][1] for u in ups]
        assert max(nbytes) < 0.75 * sum(nbytes), (c, nbytes)
    out = tmp_path / 'yahoo_ticker_matched_articles'
    want = golden_data.outputs()
    assert sorted(os.listdir(out)) == sorted(want)
    for fn in want:
        assert (out / fn).read_bytes() == want[fn], fn


def test_shard_rows_balance_bytes():
    from advanced_scrapper_amd.match_keywords import shard_rows
    texts = ['a' * (i % 7) + 'é' * (i % 3) for i in range(50)]
    titles = ['t' * (i % 5) for i in range(50)]
    for world in (1, 2, 3, 8):
        rr = [shard_rows(texts, titles, 40, r, world) for r in range(world)]
        assert rr[0][0] == 0 and rr[-1][1] == 40
        assert all(rr[i][1] == rr[i + 1][0] for i in range(world - 1))


def test_byte_balanced_ranges_cover_and_balance():
    from advanced_scrapper_amd import dist
    rng = np.random.default_rng(5)
    for world in (1, 2, 4, 8):
        n = 1000
        lens = rng.lognormal(7.6, 0.6, size=2 * n).astype(np.int64)
        off = np.zeros(2 * n + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        rr = dist.byte_balanced_ranges(off, world)
        assert rr[0][0] == 0 and rr[-1][1] == n
        assert all(rr[i][1] == rr[i + 1][0] for i in range(world - 1))
        sizes = [off[2 * hi] - off[2 * lo] for lo, hi in rr]
        assert max(sizes) - min(sizes) <= 2 * lens.reshape(-1, 2).sum(1).max()


def test_shard_range_partitions():
    from advanced_scrapper_amd import dist
    for n in (0, 1, 7, 1000):
        for world in (1, 2, 3, 8):
            rr = [dist.shard_range(n, r, world) for r in range(world)]
            assert rr[0][0] == 0 and rr[-1][1] == n
            assert all(rr[i][1] == rr[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in rr) - min(h - l for l, h in rr) <= 1


def test_main_single_rank_equals_reference_outputs(tmp_path, monkeypatch):
    """match_keywords.main's single-GPU loop -- native CSV ingest (libkwcsv), matching, libkwrows cells, CSV
    egress, the final sort -- with only the scan stubbed by the oracle, writes the reference's own per-ticker
    files byte for byte (tests/golden/out_c1)."""
    import time
    from advanced_scrapper_amd import ingest
    from advanced_scrapper_amd import match_keywords as mk
    from tests import golden_data
    from tests.oracle_matcher import OracleMatcher
    monkeypatch.setenv('TZ', 'UTC')
    time.tzset()
    (tmp_path / 'articles.csv').write_bytes(golden_data.articles_csv_bytes())
    kinds = [type(c).__name__ for c in ingest.read_chunks(str(tmp_path / 'articles.csv'), golden_data.chunksize())]
    assert 'NativeChunk' in kinds
    monkeypatch.chdir(tmp_path)
    processed = golden_data.kb_processed()
    monkeypatch.setattr(mk, 'read_and_process_json_files', lambda _d: processed)
    args = mk._parse(['--info-dir', 'unused', '--articles', str(tmp_path / 'articles.csv'),
                      '--chunksize', str(golden_data.chunksize())])
    assert mk.run(args, 0, 1, None, None, matcher=OracleMatcher(processed)) == 0
    out = tmp_path / 'yahoo_ticker_matched_articles'
    want = golden_data.outputs()
    assert sorted(os.listdir(out)) == sorted(want)
    for fn in want:
        assert (out / fn).read_bytes() == want[fn], fn


def _plan_worker(rank, world, port, q):
    """Execute libkwmatch's exchange plan (kw_exchange_plan, the send/recv pairs kw_allgather_hits issues
    over RCCL) with gloo point-to-point calls, for every root, and report what each rank received."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from advanced_scrapper_amd import _native
    dist.init_process_group('gloo', rank=rank, world_size=world)
    out = {}
    for trial in range(3):
        counts = [((r * 7 + trial * 3) % 5) * (r + 1) for r in range(world)]     # ragged, some ranks empty
        mine = torch.tensor([[trial, r, k, world] for r in [rank] for k in range(counts[rank])],
                            dtype=torch.int32).reshape(-1, 4)
        for root in (-1, 0, world - 1, world // 2):
            off, ops, total, nrecv = _native.exchange_plan(world, rank, root, counts)
            recv = torch.full((nrecv, 4), -1, dtype=torch.int32)
            if nrecv:
                recv[off[rank]:off[rank + 1]] = mine
            reqs = []
            for p in range(world):
                if ops[p] & _native.KW_PLAN_SEND:
                    reqs.append(dist.isend(mine.contiguous(), p, tag=trial * 100 + root + 10))
                if ops[p] & _native.KW_PLAN_RECV:
                    buf = torch.empty((counts[p], 4), dtype=torch.int32)
                    reqs.append((dist.irecv(buf, p, tag=trial * 100 + root + 10), buf, p))
            for r in reqs:
                if isinstance(r, tuple):
                    r[0].wait()
                    recv[off[r[2]]:off[r[2] + 1]] = r[1]
                else:
                    r.wait()
            out[(trial, root)] = (total, recv.numpy().tolist())
            dist.barrier()
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_exchange_plan_gloo_matches_concatenation():
    """kw_exchange_plan, run with gloo send/recv for world sizes 2-8 and roots -1 (all), 0, the last and a
    middle rank: every receiver ends with every rank's records in rank order, non-receivers with nothing,
    and no send lacks its receive (a mismatch would hang and fail the timeout)."""
    for world in (2, 3, 5, 8):
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_plan_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for trial in range(3):
            counts = [((r * 7 + trial * 3) % 5) * (r + 1) for r in range(world)]
            want = [[trial, r, k, world] for r in range(world) for k in range(counts[r])]
            for root in (-1, 0, world - 1, world // 2):
                for rank in range(world):
                    total, got = res[rank][(trial, root)]
                    assert total == len(want)
                    if root < 0 or root == rank:
                        assert got == want, (world, trial, root, rank)
                    else:
                        assert got == [], (world, trial, root, rank)


def test_exchange_plan_rejects_bad_arguments():
    import pytest
    from advanced_scrapper_amd import _native
    for args in ((0, 0, -1, [1]), (2, 2, -1, [1, 1]), (2, 0, 2, [1, 1]), (2, 0, -1, [1, -1])):
        with pytest.raises(_native.KwError):
            _native.exchange_plan(*args)


def _error_worker(rank, world, port, work, case, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TZ='UTC')
    import io
    import time
    import pandas as pd
    time.tzset()
    from advanced_scrapper_amd import dist
    from advanced_scrapper_amd import match_keywords as mk
    from tests import golden_data
    from tests.oracle_matcher import OracleMatcher
    dist.init('gloo')
    os.chdir(work)
    g = golden_data.error_cases()
    c = g['cases'][case]
    processed = golden_data.processed_from(g['kb_processed'])
    os.makedirs('yahoo_ticker_matched_articles', exist_ok=True)
    ex = dist.Exchange(rank, world, None, 'gloo')
    m = OracleMatcher(processed)
    raised = None
    try:
        for chunk in pd.read_csv(io.StringIO(c['articles_csv']), chunksize=g['chunksize']):
            mk._write_chunk_sharded('yahoo', chunk, processed, m, ex)
            ex.barrier()
    except Exception as exc:   # noqa: BLE001
        raised = type(exc).__name__
    q.put((rank, raised))
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


def test_gloo_pandas_chunk_errors_release_every_rank(tmp_path):
    """A pandas-path chunk (parsed whole by every rank, written by rank 0) whose rows raise -- an in-period
    invalid-regex name (re.error at :178), a bad date (:152), integer dates (:131) -- ends on EVERY rank
    (no rank left waiting in a collective): rank 0 raises the reference's exception after writing exactly
    the reference's partial files, the other rank raises the same date error or ShardError."""
    from tests import golden_data
    g = golden_data.error_cases()
    for case in ('invalid_regex', 'bad_date', 'int_dates'):
        c = g['cases'][case]
        work = tmp_path / case
        work.mkdir()
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_error_worker, args=(r, 2, port, str(work), case, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(2))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert res[0] == c['exception'], (case, res)
        assert res[1] in (c['exception'], 'ShardError'), (case, res)
        out = work / 'yahoo_ticker_matched_articles'
        got = {fn: (out / fn).read_text(encoding='utf-8') for fn in os.listdir(out)}
        assert got == c['files'], case


def test_native_chunk_year_one_date_writes_rows_before_it(tmp_path, monkeypatch):
    """An article dated '0001-01-01 00:00:00' (parsed by dateutil: year < 1000) that matches a name without a
    start date: the reference's append_to_csv raises at its ``timestamp()`` (:131-132, 'year 0 is out of
    range' in a UTC process) after the earlier articles' rows were written.  The native chunk path must write
    exactly those rows and raise the same error (Dates.utc_stamps stops at that row)."""
    import time
    from advanced_scrapper_amd import egress
    from advanced_scrapper_amd import match_keywords as mk
    from tests import golden_data
    from tests.oracle_matcher import OracleMatcher
    monkeypatch.setenv('TZ', 'UTC')
    time.tzset()
    processed = golden_data.kb_processed()
    frame = golden_data.articles_frame().iloc[:60].copy()
    bad = 37
    frame.iloc[bad, frame.columns.get_loc('date_time')] = '0001-01-01 00:00:00'
    frame.iloc[bad, frame.columns.get_loc('article_text')] = 'Caesars Entertainment and CZR today.'
    monkeypatch.setattr(mk, 'read_and_process_json_files', lambda _d: processed)
    outs = {}
    for tag, rows in (('error', frame), ('before', frame.iloc[:bad])):
        d = tmp_path / tag
        d.mkdir()
        rows.to_csv(d / 'articles.csv', index=False)
        monkeypatch.chdir(d)
        args = mk._parse(['--info-dir', 'unused', '--articles', str(d / 'articles.csv'), '--chunksize', '1000'])
        if tag == 'error':
            from advanced_scrapper_amd import ingest
            assert isinstance(next(iter(ingest.read_chunks(str(d / 'articles.csv'), 1000))), ingest.NativeChunk)
            with pytest.raises(ValueError, match='year 0 is out of range'):
                mk.run(args, 0, 1, None, None, matcher=OracleMatcher(processed))
        else:   # the reference stops before its final sort: compare the appended rows
            monkeypatch.setattr(egress.RunFiles, 'finish', lambda self, name: True)
            mk.run(args, 0, 1, None, None, matcher=OracleMatcher(processed))
            monkeypatch.undo()
            monkeypatch.setenv('TZ', 'UTC')
            monkeypatch.setattr(mk, 'read_and_process_json_files', lambda _d: processed)
        out = d / 'yahoo_ticker_matched_articles'
        outs[tag] = {f: (out / f).read_bytes() for f in os.listdir(out)}
    assert outs['error'] == outs['before']
    assert len(outs['before']) > 0


def _caps_worker(rank, world, port, q):
    """Each rank all-gathers its (count, receiver capacity) pair with gloo -- the one exchange kw_allgather_hits
    makes over RCCL -- and applies libkwmatch's kw_exchange_caps_ok to the gathered pairs."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from advanced_scrapper_amd import _native
    dist.init_process_group('gloo', rank=rank, world_size=world)
    out = {}
    for trial in range(4):
        counts = [(r * 5 + trial * 7) % 11 for r in range(world)]
        total = sum(counts)
        for root in (-1, 0, world - 1):
            receives = root < 0 or root == rank
            short = trial == 1 and rank == world - 1 or trial == 3 and rank == 0
            cap = (total - 1 if short else total + trial) if receives else np.iinfo(np.int64).max
            mine = torch.tensor([counts[rank], cap], dtype=torch.int64)
            got = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(got, mine)
            c = [int(g[0]) for g in got]
            k = [int(g[1]) for g in got]
            out[(trial, root)] = _native.exchange_caps_ok(world, root, c, k)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_exchange_capacity_verdict_agreed_on_every_rank():
    """A receiver whose destination cannot hold the exchange fails the exchange on EVERY rank (the verdict comes
    from the gathered (count, capacity) pairs, before any record moves), so no peer is left waiting in a send;
    world sizes 2 and 3, roots -1 / 0 / last, short receivers at either end."""
    for world in (2, 3):
        ctx = mp.get_context('spawn')
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_caps_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=300) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        for key, v in res[0].items():
            assert all(res[r][key] == v for r in range(world)), (world, key, [res[r][key] for r in range(world)])
            trial, root = key
            short = {1: world - 1, 3: 0}.get(trial)
            receivers = range(world) if root < 0 else [root]
            want_bad = min((r for r in receivers if r == short), default=-1)
            assert v == (want_bad < 0, want_bad), (world, key, v)
