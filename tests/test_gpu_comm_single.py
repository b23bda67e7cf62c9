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


def test_one_rank_short_destination_and_errors(comm):
    """the receiver-capacity verdict of both exchange calls on the hardware (KW_EOVERFLOW), the
    planned call's local argument errors (KW_EINVAL after posting its matching half), the negative-count error
    flag -- and the communicator still works for a following good exchange."""
    import ctypes
    import torch
    from advanced_scrapper_amd import _native
    L, h = _native.lib(), comm.h
    n = 100
    src = torch.arange(n * 4, dtype=torch.int32, device='cuda').reshape(n, 4)
    short = torch.zeros((n - 1, 4), dtype=torch.int32, device='cuda')
    nt = ctypes.c_int64()
    cnt = np.zeros(1, dtype=np.int64)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.kw_allgather_hits(h, _native.ptr(src), n, 0, 0, _native.ptr(short), n - 1, ctypes.byref(nt),
                             _native.ptr(cnt), sp)
    assert rc == _native.KW_EOVERFLOW and b'destination holds' in L.kw_comm_last_error(h)
    counts = np.array([n], dtype=np.int64)
    rc = L.kw_allgather_hits_planned(h, _native.ptr(src), n, 0, -1, _native.ptr(counts), _native.ptr(short), n - 1,
                                     ctypes.byref(nt), sp)
    assert rc == _native.KW_EOVERFLOW and b'too small' in L.kw_comm_last_error(h)
    # ids past 2^32: the self-contained call agrees on the error before any record moves
    rc = L.kw_allgather_hits(h, _native.ptr(src), n, 0xFFFFFFFF - 10, 0, _native.ptr(src), n, ctypes.byref(nt),
                             _native.ptr(cnt), sp)
    assert rc == _native.KW_EINVAL and b'beyond 2^32' in L.kw_comm_last_error(h)
    # the planned call: counts that disagree with n, and the negative-count flag
    wrong = np.array([n + 5], dtype=np.int64)
    big = torch.zeros((n + 5, 4), dtype=torch.int32, device='cuda')
    rc = L.kw_allgather_hits_planned(h, _native.ptr(src), n, 0, -1, _native.ptr(wrong), _native.ptr(big), n + 5,
                                     ctypes.byref(nt), sp)
    assert rc == _native.KW_EINVAL and b'counts[rank]' in L.kw_comm_last_error(h)
    neg = np.array([-1], dtype=np.int64)
    rc = L.kw_allgather_hits_planned(h, _native.ptr(src), n, 0, -1, _native.ptr(neg), _native.ptr(big), n + 5,
                                     ctypes.byref(nt), sp)
    assert rc == _native.KW_EINVAL and b'negative count' in L.kw_comm_last_error(h)
    with pytest.raises(Exception):
        comm.gather_hits(src, doc_base=0xFFFFFFFF - 10, root=0)
    torch.cuda.synchronize()
    # a good exchange after all of them
    out, counts = comm.gather_hits(src, doc_base=7, root=0)
    torch.cuda.synchronize()
    want = src.cpu().numpy().copy()
    want[:, 0] += 7
    assert counts == [n] and np.array_equal(out.cpu().numpy(), want)
