"""libkwmatch's RCCL exchange (csrc/kwcomm.hip) on one GPU: a one-rank communicator.

The driver's scaling runs put one rank on each GPU of a node (bench.py --gpus N, match_keywords.py:231-238's
shards); a one-GPU box cannot start two ranks on one device under RCCL, so test_gpu_multi.py skips here.  One
rank still runs every call of the exchange on the hardware: librccl resolved at run time, the communicator,
the counts all-gather, the planned record exchange (Send / Recv to itself inside a group) for every root, the
shard's doc-id offset, an empty shard, and the receiver-capacity verdict (dist.KwComm.gather_hits)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def comm():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from advanced_scrapper_amd.dist import KwComm
    c = KwComm(0, 1, torch.cuda.current_device())
    yield c
    c.close()


def test_one_rank_exchange_all_roots(comm):
    import torch
    rng = np.random.default_rng(3)
    for n in (0, 1, 37, 5000):
        h = rng.integers(0, 1 << 20, size=(n, 4)).astype(np.int32)
        h[:, 0] = np.sort(rng.integers(0, 1000, size=n)).astype(np.int32)
        d = torch.from_numpy(h).cuda()
        for root in (-1, 0):
            out, counts = comm.gather_hits(d, doc_base=123, root=root)
            torch.cuda.synchronize()
            assert counts == [n]
            got = out.cpu().numpy()
            want = h.copy()
            want[:, 0] += 123
            assert got.shape == (n, 4) and np.array_equal(got, want), (n, root)


def test_one_rank_counts(comm):
    assert comm.allgather_counts(42) == [42]
    assert comm.allgather_counts(0) == [0]
