"""One rank of tests/test_gpu_multi.py (started by torch.distributed.run, one process per GPU, RCCL).

1. libkwmatch's RCCL exchange (KwComm.gather_hits) with root 0 and root -1: every receiver ends with
   every rank's records, doc ids rebased, in rank order.
2. The drop-in's --gpus N main path (sharded ingest, RCCL where the writer needs records, ordered writes,
   split sort) over the golden article CSV: rank 0 checks the per-ticker files against the reference's
   own outputs (tests/golden/out_c1) byte for byte.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    work = sys.argv[1]
    os.environ['TZ'] = 'UTC'
    time.tzset()
    import torch
    from advanced_scrapper_amd import dist
    rank, world, local = dist.init('nccl')
    dev = torch.device('cuda', local)
    comm = dist.KwComm(rank, world, local)
    n = 5 + 3 * rank
    mine = torch.tensor([[k, 100 + rank, k * 7, rank & 1] for k in range(n)], dtype=torch.int32, device=dev)
    bases = [sum(10 * (r + 1) for r in range(q)) for q in range(world)]
    want = []
    for r in range(world):
        want += [[bases[r] + k, 100 + r, k * 7, r & 1] for k in range(5 + 3 * r)]
    for root in (0, -1):
        got, counts = comm.gather_hits(mine, bases[rank], root=root)
        torch.cuda.synchronize()
        assert counts == [5 + 3 * r for r in range(world)], counts
        if root < 0 or rank == root:
            assert got.cpu().tolist() == want, (rank, root)
        else:
            assert got is None
    comm.close()

    from advanced_scrapper_amd import match_keywords as mk
    from tests import golden_data
    os.chdir(work)
    processed = golden_data.kb_processed()
    mk.read_and_process_json_files = lambda _d: processed
    args = mk._parse(['--info-dir', 'unused', '--articles', os.path.join(work, 'articles.csv'),
                      '--chunksize', str(golden_data.chunksize()), '--gpus', str(world)])
    assert mk.run(args, rank, world, local, 'nccl') == 0
    if rank == 0:
        out = os.path.join(work, 'yahoo_ticker_matched_articles')
        want_files = golden_data.outputs()
        assert sorted(os.listdir(out)) == sorted(want_files)
        for fn, data in want_files.items():
            with open(os.path.join(out, fn), 'rb') as fh:
                assert fh.read() == data, fn
        print('multi-GPU ok', world, flush=True)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
