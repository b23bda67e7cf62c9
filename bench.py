"""Benchmark: article GB/s keyword-matched (S&P500 KB) on MI355X — BASELINE.json's metric.

One step = one kw_scan pass (scan + resolve + result compaction) over the
rank's whole shard of synthetic articles, already resident in HBM, followed
by the exchange of the per-rank hits (N > 1).  Workloads (BASELINE.json):
N = 1 scans config 2's 1M documents; N > 1 scans config 3's 10M documents
(documents 0..9 999 999 of the seeded generator) as N contiguous shards of
10M / N (strong scaling).  ``--total-docs T`` fixes another total,
``--docs-per-gpu D`` gives every rank D documents (weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Rank 0 prints one JSON line.  ``roofline`` prices the scan kernel against
HBM (8.0 TB/s) with the algorithmic bytes = sum of UTF-8 bytes of every
article's text and title; the kernel time is the HIP-event
time of the scan kernel on the stream it runs on.  ``cpu_baseline`` times the
oracle's CPU port (oracle/cpu_port.py) on a bounded sample of the same
corpus, rank 0 at N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0
METRIC = "article GB/s keyword-matched (S&P500 set) at 1 & 8 GPUs; % of HBM peak"


def _parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--docs-per-gpu', type=int, default=None,
                    help='documents per rank (weak scaling); default: the --total-docs split over the ranks')
    ap.add_argument('--total-docs', type=int, default=None,
                    help='documents of the whole job, split in contiguous shards (default: 1M = config 2 at N = 1, '
                         '10M = config 3 at N > 1)')
    ap.add_argument('--seed', type=int, default=20250905)
    ap.add_argument('--cpu-sample', type=int, default=10000,
                    help='docs of the same corpus timed on the CPU port of the reference loop (0 = skip)')
    ap.add_argument('--cpu-procs', type=int, default=0,
                    help='CPU port processes (0 = the CPUs this process may use: affinity, capped by the cgroup '
                         'CPU quota; the reference uses Pool(cpu_count()))')
    ap.add_argument('--lib-variant', default=None,
                    help='time lib/libkwmatch_<TAG>.so (a tuning build, advanced_scrapper_amd/build.py) instead of '
                         'the default library; the line names the library and its sha256 either way')
    ap.add_argument('--hits', choices=('root', 'all', 'none'), default='root',
                    help='N > 1: hit records exchanged every step over libkwmatch\'s RCCL communicator '
                         '(root = to rank 0, the writer; all = all-gather; none = counts only)')
    ap.add_argument('--traffic-json', default=None,
                    help='per-launch HBM bytes from the rocprofv3 PMC passes (profiles/pmc_traffic.py)')
    ap.add_argument('--workload', choices=('match', 'kb50k', 'dedup'), default='match',
                    help='match = BASELINE.json metric (config 2/3); kb50k = ~50k-pattern synthetic KB '
                         '(config 4); dedup = CDX URL dedup (config 5)')
    ap.add_argument('--rows-per-gpu', type=int, default=500_000_000, help='dedup: CDX rows per GPU (config 5)')
    ap.add_argument('--inflight', type=int, choices=(1, 2), default=1,
                    help='scans in flight per GPU: 2 = two libkwmatch handles on two streams, step i + 1 is '
                         'launched before step i\'s hits are read (its filter overlaps step i\'s latency-bound '
                         'epilogue and task kernels); 1 = one scan at a time')
    return ap.parse_args()


def _launch_ranks(args) -> int:
    """``--gpus N`` without torchrun's environment: start N rank processes (torch.distributed.run) before
    this process touches the GPU, and return their exit code.  With torchrun's environment, WORLD_SIZE must
    equal --gpus."""
    world = os.environ.get('WORLD_SIZE')
    if world is not None:
        if int(world) != args.gpus:
            raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
        return -1
    if args.gpus <= 1:
        return -1
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', f'--master-port={port}', os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


CONFIG2_DOCS = 1_000_000
CONFIG3_DOCS = 10_000_000


def shard_plan(args, rank: int, world: int):
    """(first document, documents of this rank, documents of the job, scaling) of the bench's workload."""
    if args.docs_per_gpu is not None:
        n = args.docs_per_gpu
        return rank * n, n, n * world, 'weak'
    total = args.total_docs if args.total_docs is not None else (CONFIG2_DOCS if world == 1 else CONFIG3_DOCS)
    per = -(-total // world)
    lo = min(rank * per, total)
    return lo, min(per, total - lo), total, 'strong'


def workload_label(total_docs: int, world: int) -> str:
    if total_docs == CONFIG3_DOCS:
        return 'config 3'
    if total_docs == CONFIG2_DOCS and world == 1:
        return 'config 2'
    return f'{total_docs} documents'


def load_kb(kb_dir: str):
    """The reference KB (info/ticker, 216 tickers after its filter) through the product's own loader: the KB
    JSON files (tests/golden/kb_bundle.json.gz, written by make_golden.py from the reference's info/ticker)
    are materialised in kb_dir and read by kb.read_and_process_json_files in the reference's listdir order."""
    import gzip
    import io
    from contextlib import redirect_stdout
    from advanced_scrapper_amd.kb import read_and_process_json_files
    b = json.loads(gzip.decompress(open(os.path.join(REPO, 'tests', 'golden', 'kb_bundle.json.gz'), 'rb').read()))
    os.makedirs(kb_dir, exist_ok=True)
    for fn, text in b['files'].items():
        with open(os.path.join(kb_dir, fn), 'wb') as fh:
            fh.write(text.encode('utf-8'))
    order = list(b['listdir'])
    with redirect_stdout(io.StringIO()):          # the reference prints every ticker and the whole dict
        return read_and_process_json_files(kb_dir, _listdir=lambda _d: order)


def hits_digest(hits) -> str:
    """Order-independent 64-bit digest of [n, 4] int32 records (doc, pattern, pos, field) with global doc
    ids: the wrapping sum of a mixed hash of every record, so shardings and record orders agree."""
    import torch
    if hits.numel() == 0:
        return '0' * 16
    h = hits.to(torch.int64) & 0xFFFFFFFF
    x = (h[:, 0] * 0x9E3779B97F4A7C15 + h[:, 1] * 0x2545F4914F6CDD1D + h[:, 2] * 0x27D4EB2F165667C5 +
         h[:, 3] * 0x165667B19E3779F9)
    x = x ^ ((x >> 31) & 0x1FFFFFFFF)
    x = x * -0x40A7B892E31B1A47
    x = x ^ ((x >> 29) & 0x7FFFFFFFF)
    return f'{int(x.sum().item()) & 0xFFFFFFFFFFFFFFFF:016x}'


def host_cpus() -> dict:
    """CPUs this process may use: os.cpu_count(), the affinity mask, the cgroup v2 CPU quota (cpu.max) and
    the usable count = min(affinity, quota)."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return {'os_cpu_count': os.cpu_count(), 'affinity': n_aff, 'cgroup_quota': quota,
            'usable': min(n_aff, quota) if quota else n_aff}


def main():
    args = _parse()
    if args.lib_variant:
        os.environ['KW_LIB'] = os.path.join(REPO, 'advanced_scrapper_amd', 'lib', f'libkwmatch_{args.lib_variant}.so')
        os.environ['KW_LIB_VARIANT_OK'] = '1'
    rc = _launch_ranks(args)
    if rc >= 0:
        sys.exit(rc)
    if args.workload == 'dedup':
        return bench_dedup(args)

    import torch
    from advanced_scrapper_amd import _native, dist, synth
    from advanced_scrapper_amd.kb import compile_kb
    from advanced_scrapper_amd.matcher import GpuMatcher, background_sample

    rank, world, local = dist.init('nccl')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)

    t_kb = time.perf_counter()
    if args.workload == 'kb50k':                     # config 4: synthetic Wikidata-style KB, ~52k names
        from advanced_scrapper_amd.synth_kb import synthetic_kb
        processed = synthetic_kb(2300, args.seed)
    else:
        import tempfile
        with tempfile.TemporaryDirectory() as tmp:  # info/ticker KB (S&P500 subset), 216 tickers
            processed = load_kb(os.path.join(tmp, 'ticker'))
    ckb = compile_kb(processed)
    t_kb = time.perf_counter() - t_kb
    names, kinds = synth.injectable_names(ckb)
    doc_base, n_local, total_docs, scaling = shard_plan(args, rank, world)
    t_gen = time.perf_counter()
    corpus = synth.generate(n_local, names, kinds, seed=args.seed, doc_base=doc_base)
    t_gen = time.perf_counter() - t_gen
    # anchor statistics from an independent sample (different seed, not the timed documents)
    bg_corpus = synth.generate(2000, names, kinds, seed=args.seed + 7777, doc_base=0)
    bgs = background_sample(bg_corpus.texts() + bg_corpus.titles())
    m = GpuMatcher(ckb, local, bgs)
    # --inflight 2: a second handle (its own scratch and streams) so two complete scans overlap
    ms = [m] + [GpuMatcher(ckb, local, bgs) for _ in range(args.inflight - 1)]
    t_up = time.perf_counter()
    d_arena, d_off = m.upload(corpus.arena, corpus.off)
    torch.cuda.synchronize()
    t_up = time.perf_counter() - t_up
    local_bytes = corpus.n_bytes

    # N > 1: the hit records of step i move over libkwmatch's RCCL communicator on a stream of their own
    # while step i + 1 scans (double-buffered staging copies; the counts exchange is the step's rendezvous)
    comm = dist.KwComm(rank, world, local) if world > 1 else None
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(args.inflight - 1)]
    comm_stream = torch.cuda.Stream(dev) if comm is not None else None
    stage = [None, None]
    copied = [torch.cuda.Event(), torch.cuda.Event()]
    sent = [None, None]
    last = {'gathered': None, 'counts': None}

    def launch(i):
        k = i % len(ms)
        ms[k].scan(d_arena, d_off, n_local, streams[k])

    def collect(i):
        k = i % len(ms)
        mk, compute = ms[k], streams[k]
        n = mk.n_hits()                                  # waits for that scan, reads the count
        if comm is None:
            return [n]
        b = i & 1
        if sent[b] is not None:
            compute.wait_event(sent[b])                  # the exchange that read this staging buffer is done
        if stage[b] is None or stage[b].shape[0] < max(n, 1):
            stage[b] = torch.empty((max(n + n // 4, 1), 4), dtype=torch.int32, device=dev)
        mk.hits_copy_into(stage[b], compute)
        copied[b].record(compute)
        if args.hits == 'none':
            return comm.allgather_counts(n, comm_stream)
        comm_stream.wait_event(copied[b])
        g, counts = comm.gather_hits(stage[b][:n], doc_base, root=0 if args.hits == 'root' else -1,
                                     stream=comm_stream)
        ev = torch.cuda.Event()
        ev.record(comm_stream)
        sent[b] = ev
        last['gathered'], last['counts'] = g, counts
        return counts

    def sync_all():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    def run(n_steps, times=None):
        # step i + 1 is launched before step i's hits are read: with two handles their kernels overlap
        out = None
        if len(ms) == 1:
            for i in range(n_steps):
                launch(i)
                out = collect(i)
                if times is not None:
                    times.append(m.kernel_times())
            return out
        for i in range(n_steps):
            launch(i)
            if i >= 1:
                out = collect(i - 1)
                if times is not None:
                    times.append(ms[(i - 1) % len(ms)].kernel_times())
        if n_steps:
            out = collect(n_steps - 1)
            if times is not None:
                times.append(ms[(n_steps - 1) % len(ms)].kernel_times())
        return out

    run(args.warmup)
    sync_all()
    ktimes = []
    t0 = time.perf_counter()
    counts = run(args.steps, ktimes)
    sync_all()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    nb = torch.tensor([float(local_bytes)], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(nb, op=torch.distributed.ReduceOp.SUM)
    elapsed = float(el.item())
    total_bytes = float(nb.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = total_bytes / (elapsed / args.steps) / 1e9

    # the digest of every hit record of the whole job (global document ids), on rank 0
    if comm is None:
        digest = hits_digest(m.hits_device())
    elif args.hits in ('root', 'all'):
        digest = hits_digest(last['gathered']) if rank == 0 else None
    else:
        digest = None
    st = m.stats()
    if comm is not None:
        comm.close()
    if rank != 0:
        return
    kavg = {k: float(np.mean([t[k] for t in ktimes])) for k in ktimes[0]}
    lib_id = _native.lib_identity()
    lib_sha = lib_id['sha256']
    scan_avg = kavg['filter']         # the kernel that streams every article byte (HIP events on its stream)
    achieved = local_bytes / (scan_avg * 1e-3) / 1e9
    cpu = None
    if world == 1 and args.cpu_sample > 0:
        # the port walks every name occurrence per field: config 4's 52k names take ~1 s per article
        n_cpu = args.cpu_sample if args.workload == 'match' else min(args.cpu_sample, 64)
        cpu = cpu_baseline(processed, corpus, n_cpu, args.cpu_procs)
    if args.workload == 'kb50k':
        n_act = ckb.n_patterns
        workload = (f'config 4: synthetic Wikidata-style KB ({len(processed)} tickers, {n_act} active names, '
                    f'all <= 64 code points) vs synthetic ~2 KB articles, {n_local} docs per GPU')
        metric = 'article GB/s keyword-matched (~50k-pattern synthetic KB, config 4); % of HBM peak'
        data = 'synthetic (seeded generators: csrc/synth.c articles, synth_kb.py KB)'
    else:
        cfg = workload_label(total_docs, world)
        workload = (f'{cfg}: S&P500 KB (216 tickers, 2462 active names) vs synthetic ~2 KB articles, '
                    f'{total_docs} docs in {world} contiguous shard(s), {n_local} on rank 0')
        metric = METRIC
        data = ('synthetic (seeded generator, csrc/synth.c, documents 0..total_docs-1; KB = the reference\'s '
                'info/ticker JSON files read by the product\'s read_and_process_json_files)')
    exch = {'root': 'RCCL send/recv of every hit record to rank 0',
            'all': 'RCCL all-gather of every hit record', 'none': 'RCCL all-gather of counts'}[args.hits]
    out = {
        'metric': metric,
        'value': round(value, 2),
        'unit': 'GB/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_per_step, 4),
        'higher_is_better': True,
        'scaling': scaling,
        'vs_baseline': None,
        'dtype': 'u8',
        'data': data,
        'config': {
            'workload': workload,
            'docs_per_gpu': n_local, 'total_docs': total_docs, 'bytes_per_gpu': local_bytes,
            'total_bytes': int(total_bytes), 'hits_total': int(sum(counts)) if counts else None,
            'hits_digest': digest,
            'parallelism': (f'dp{world} (contiguous document shards; per step: {exch}, overlapped with the '
                            f'next scan)' if world > 1 else 'dp1'),
            'scans_in_flight': args.inflight,
        },
        'roofline': {
            'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBS, 4),
            'traffic': (pmc_traffic(args.traffic_json or TRAFFIC_KW, 'kw_filter_kernel', docs_per_gpu=n_local,
                                    seed=args.seed, library_sha256=lib_sha)
                        if args.workload == 'match' else
                        pmc_traffic(args.traffic_json or TRAFFIC_C4, 'kw_filter_kernel', docs_per_gpu=n_local,
                                    seed=args.seed, workload='kb50k', library_sha256=lib_sha)),
            'step_traffic': pmc_step_traffic(args.traffic_json or (TRAFFIC_KW if args.workload == 'match'
                                                                    else TRAFFIC_C4),
                                             docs_per_gpu=n_local, seed=args.seed, library_sha256=lib_sha,
                                             **({} if args.workload == 'match' else {'workload': 'kb50k'})),
            # the metric's own "% of HBM peak": the whole step's article bytes per second (value) over 8 TB/s;
            # frac above prices the filter kernel alone
            'step_frac': round(value / HBM_PEAK_GBS, 4),
            'algorithmic_bytes_per_launch': local_bytes,
            'kernel': 'kw::kw_filter_kernel', 'kernel_ms_avg': round(scan_avg, 4),
            'kernels_ms_avg': {k: round(v, 4) for k, v in kavg.items()},
            'all_kernels_GBps': round(local_bytes / (kavg['total'] * 1e-3) / 1e9, 2),
        },
        'cpu_baseline': cpu,
        'scan_stats': st,
        'library': lib_id,
        'host': {'kb_load_compile_s': round(t_kb, 3), 'generate_s': round(t_gen, 2), 'h2d_s': round(t_up, 3),
                 'h2d_GBps_pcie_inclusive': round(local_bytes / t_up / 1e9, 2) if t_up > 0 else None,
                 **host_cpus()},
    }
    print(json.dumps(out), flush=True)


def bench_dedup(args):
    """Config 5: CDX link-row normalise + keep-first dedup (yahoo_links_selenium.py:59-82,160-179).

    One step = one kw_dedup_run over the rank's rows (resident in HBM): rewrite +
    hash + table insert, rep compare, dense kept rows.  value = (URL bytes + 8 B
    per offset) of all ranks / step time."""
    import torch
    from advanced_scrapper_amd import _native, dist, synth
    from advanced_scrapper_amd.cdx_dedup import GpuUrlDedup
    rank, world, local = dist.init('nccl')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    n = args.rows_per_gpu
    t_gen = time.perf_counter()
    rows = synth.generate_urls(n, seed=args.seed, row_base=rank * n, n_articles=int(1.31 * n * world))
    t_gen = time.perf_counter() - t_gen
    g = GpuUrlDedup(local)
    d_a, d_o = g.upload(rows.arena, rows.off)
    torch.cuda.synchronize()
    local_bytes = rows.n_bytes + 8 * rows.n
    for _ in range(args.warmup):
        g.run(d_a, d_o, rows.n)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    kt = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.run(d_a, d_o, rows.n)
        kt.append(g.last_ms())
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    nb = torch.tensor([float(local_bytes)], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(nb, op=torch.distributed.ReduceOp.SUM)
    elapsed = float(el.item())
    counts = g.counts()
    if rank != 0:
        return
    k = np.mean(np.asarray(kt), axis=0)
    names = ('transform_insert', 'slow_rows', 'decide', 'compact', 'total')
    kms = {a: round(float(b), 4) for a, b in zip(names, k)}
    transform_gbs = rows.n_bytes / (kms['transform_insert'] * 1e-3) / 1e9
    lib_id = _native.lib_identity()
    cpu = None
    if world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline_dedup(rows, min(n, 2_000_000))
    out = {
        'metric': 'CDX URL dedup GB/s (URL bytes + 8 B offsets), bit-exact vs pandas drop_duplicates keep-first',
        'value': round(float(nb.item()) / (elapsed / args.steps) / 1e9, 2), 'unit': 'GB/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8',
        'data': 'synthetic CDX rows (csrc/synth.c generate_urls, ~30 % repeated articles)',
        'config': {'workload': f'config 5: CDX link-row normalise + keep-first dedup, {n} rows per GPU',
                   'rows_per_gpu': n, 'bytes_per_gpu': local_bytes, 'kept': counts[1],
                   'dropped_no_html': counts[0], 'dropped_filter': counts[2], 'duplicates': counts[3],
                   'parallelism': 'replicas only (one independent keep-first per GPU)' if world > 1 else 'single GPU'},
        'roofline': {'bound': 'hbm', 'achieved': round(transform_gbs, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': round(transform_gbs / HBM_PEAK_GBS, 4),
                     'traffic': pmc_traffic(args.traffic_json or TRAFFIC_DEDUP, 'dd_transform_kernel', rows_per_gpu=n,
                                            seed=args.seed, library_sha256=lib_id['sha256']),
                     'step_traffic': pmc_step_traffic(args.traffic_json or TRAFFIC_DEDUP, rows_per_gpu=n,
                                                      seed=args.seed, library_sha256=lib_id['sha256'],
                                                      prefix='dd_'),
                     'step_frac': round(float(nb.item()) / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                     'algorithmic_bytes_per_launch': rows.n_bytes, 'kernel': 'dd::dd_transform_kernel',
                     'kernel_ms_avg': kms['transform_insert'], 'kernels_ms_avg': kms},
        'cpu_baseline': cpu,
        'library': lib_id,
        'host': {'generate_s': round(t_gen, 2)},
    }
    print(json.dumps(out), flush=True)


def cpu_baseline_dedup(rows, n_sample: int):
    """The reference's pandas steps (:63-79 + the :174 keep-first) on the first n_sample rows, one process."""
    import pandas as pd
    urls = [rows.url(i) for i in range(n_sample)]
    nbytes = int(rows.off[n_sample] - rows.off[0]) + 8 * n_sample
    df = pd.DataFrame({'date_time': rows.ts[:n_sample], 'url': urls})
    t = time.perf_counter()
    df = df[df['url'].str.contains('.html')]
    df['url'] = df['url'].str.split('.html').str[0] + '.html'
    df['url'] = df['url'].str.replace(':80', '', regex=False)
    df['url'] = df['url'].str.replace('http:', 'https:', regex=False)
    df = df[~df['url'].str.contains('news/%')]
    df = df[~df['url'].str.contains("news/'")]
    df = df.drop_duplicates(subset=['url'])
    secs = time.perf_counter() - t
    return {'value': round(nbytes / secs / 1e9, 6), 'unit': 'GB/s', 'cores': 1, 'kind': 'port',
            'sample': f'first {n_sample} rows ({nbytes} bytes incl. offsets), the reference\'s pandas calls '
                      f'(yahoo_links_selenium.py:63-79), one process, {secs:.2f} s', 'kept': int(len(df))}


# this round's PMC passes (scripts/gpu_profile.sh); each file's workload key carries the sha256 of the library it
# profiled, so a file left from an older build prices nothing (traffic = None) instead of an old kernel's bytes
TRAFFIC_KW = os.path.join(REPO, 'profiles', 'traffic_r06.json')
TRAFFIC_DEDUP = os.path.join(REPO, 'profiles', 'traffic_dedup_r06.json')
TRAFFIC_C4 = os.path.join(REPO, 'profiles', 'traffic_c4_r06.json')


def _traffic_file(path: str, workload: dict):
    """The PMC traffic JSON at `path` if it was measured on this workload with this library (every given key
    equal, the library's sha256 included), else None."""
    if not path or path == 'none':
        return None
    try:
        j = json.load(open(path))
    except (OSError, ValueError):
        return None
    w = j.get('workload', {})
    if any(str(w.get(k)) != str(v) for k, v in workload.items()):
        return None
    return j


def pmc_traffic(path: str, kernel: str, **workload):
    """HBM bytes per launch of `kernel` measured by the PMC passes of the same
    workload and library (FETCH_SIZE x2 + WRITE_SIZE, see profiles/pmc_traffic.py), or None."""
    j = _traffic_file(path, workload)
    if j is None:
        return None
    for k, v in j.get('kernels', {}).items():
        if kernel in k:
            return int(v['hbm_bytes_per_launch'])
    return None


def pmc_step_traffic(path: str, prefix: str = 'kw', **workload):
    """HBM bytes per step of the library's own kernels (names starting with `prefix`; the runtime's copy / fill
    kernels and torch's digest kernels outside the timed region are left out), or None."""
    j = _traffic_file(path, workload)
    if j is None:
        return None
    tot = 0.0
    for k, v in j.get('kernels', {}).items():
        name = k.split('(')[0]
        if name.startswith('void '):   # (a template instance's demangled name carries its return type)
            name = name[5:]
        if name.startswith(prefix) or name.startswith(prefix.rstrip('_') + '::'):
            # a kernel launched twice a step (the regex tasks' two phases) counts twice
            tot += v['hbm_bytes_per_launch'] * v.get('launches_per_step', 1)
    return int(tot)


def cpu_baseline(processed, corpus, n_sample: int, procs: int):
    """Time the CPU port of the reference loop (oracle/cpu_port.py) on the first n_sample documents of the
    same corpus, in the reference's pool shape; procs = the host share (min(16, os.cpu_count()))."""
    from oracle import cpu_port
    hc = host_cpus()
    procs = procs or hc['usable']
    n = min(n_sample, corpus.n_docs)
    rows = []
    nbytes = 0
    base = np.datetime64('1980-01-01T00:00:00')
    for i in range(n):
        t, ti = corpus.text(i), corpus.title(i)
        nbytes += len(t.encode('utf-8', 'surrogatepass')) + len(ti.encode('utf-8', 'surrogatepass'))
        rows.append((t, ti, str(base + np.timedelta64(1420 * (corpus.doc_base + i), 's')).replace('T', ' ')))
    # three timed runs over the same sample in the same warm pool: the line states their median (value) and
    # spread; the host's other tenants moved single runs by 2x in round 5
    times, done = cpu_port.time_port(processed, rows, procs, runs=3)
    secs = float(np.median(times))
    # one core: the same sample's first 1/procs share in one process (the per-core rate without pool effects)
    n1 = max(1, n // procs)
    t1, done1 = cpu_port.time_port(processed, rows[:n1], 1)
    return {'value': round(nbytes / secs / 1e9, 6), 'unit': 'GB/s', 'cores': procs, 'kind': 'port',
            'runs': len(times), 'median': round(nbytes / secs / 1e9, 6),
            'min': round(nbytes / max(times) / 1e9, 6), 'max': round(nbytes / min(times) / 1e9, 6),
            'wall_s': [round(t, 3) for t in times],
            'sample': f'first {done} docs of the same corpus ({nbytes} bytes): the reference loop '
                      f'(match_keywords.py:148-192: per name occurrence period check, re, partial_ratio '
                      f'decisions by the oracle C restatement, per-hit pandas appends) in its pool shape '
                      f'(:230-238), {procs} processes = the CPUs this process may use (affinity '
                      f'{hc["affinity"]}, cgroup quota {hc["cgroup_quota"]}; os.cpu_count() = {hc["os_cpu_count"]}), '
                      f'median of {len(times)} runs {secs:.2f} s wall (min {min(times):.2f}, max {max(times):.2f})',
            'docs_per_s': round(done / secs, 2), 'docs_per_s_per_core': round(done / secs / procs, 3),
            'single_core': {'docs': done1, 'wall_s': round(t1, 3), 'docs_per_s': round(done1 / t1, 2)},
            'host_cpus': hc}


if __name__ == '__main__':
    main()
