"""Multi-GPU sharding of the article stream (one process per GPU, RCCL over xGMI).

Matching shards with no data-path exchange: every article is independent
(SURVEY.md §8(e)).  Each rank owns a contiguous, byte-balanced range of
documents and a full copy of the compiled KB.  The only collectives are

* ``allgather_counts``  — per-rank hit counts (8 B x world), and
* ``gather_hits``       — the packed 16-B hit records, padded to the largest
                          rank, all-gathered so any rank can write the output.

On the GPU the exchange is libkwmatch's own RCCL communicator
(:class:`KwComm`, ``kw_comm_*`` in include/kwmatch.h: counts all-gather, then
point-to-point send/recv of the exact records over the xGMI mesh);
torch.distributed only carries the communicator id and the barriers.  The
torch-collective forms below (``allgather_counts`` / ``gather_hits``) are the
same exchange over any backend, used by the ``gloo`` CPU tests.
"""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from torchrun's environment (defaults 0, 1, 0)."""
    return (int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)),
            int(os.environ.get('LOCAL_RANK', 0)))


def init(backend: str = 'nccl'):
    import torch
    import torch.distributed as dist
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29512')
        if backend == 'nccl':
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', rank=rank, world_size=world,
                                    device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


class KwComm:
    """libkwmatch's RCCL communicator (kw_comm_init / kw_allgather_counts / kw_allgather_hits).

    The id is made by rank 0 (ncclGetUniqueId) and broadcast over the
    torch.distributed process group; every rank then joins on its device.
    """

    def __init__(self, rank: int, world: int, device: int):
        import ctypes
        import torch.distributed as td
        from . import _native
        self._n = _native
        self.rank, self.world, self.device = rank, world, device
        L = _native.lib()
        idb = np.zeros(_native.KW_COMM_ID_BYTES, dtype=np.uint8)
        if rank == 0:
            _native.check_comm(L.kw_comm_unique_id(_native.ptr(idb)))
        if world > 1:
            obj = [idb.tobytes()]
            td.broadcast_object_list(obj, src=0)
            idb = np.frombuffer(obj[0], dtype=np.uint8).copy()
        h = ctypes.c_void_p()
        rc = L.kw_comm_init(world, rank, _native.ptr(idb), device, ctypes.byref(h))
        if rc != _native.KW_OK:
            msg = L.kw_comm_last_error(h if h.value else None)
            if h.value:
                L.kw_comm_destroy(h)
            raise _native.KwError(rc, msg.decode() if msg else '')
        self.h = h
        self._out = None

    def close(self):
        if getattr(self, 'h', None) is not None and self.h.value:
            self._n.lib().kw_comm_destroy(self.h)
            self.h = None

    @staticmethod
    def _sp(stream):
        import ctypes
        return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, 'cuda_stream') else (stream or 0))

    def allgather_counts(self, count: int, stream=None) -> List[int]:
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(self.device)
        out = np.zeros(self.world, dtype=np.int64)
        self._n.check_comm(self._n.lib().kw_allgather_counts(self.h, int(count), self._n.ptr(out), self._sp(stream)),
                           self.h)
        return [int(x) for x in out]

    def gather_hits(self, hits, doc_base: int, root: int = -1, stream=None):
        """Exchange [n, 4] int32 device records (doc ids local to the rank's shard).  Returns
        (records of every rank in document order with global doc ids -- on receiving ranks, else
        None -- and the per-rank counts).  Asynchronous on ``stream`` after the counts exchange; the
        default is torch's current stream of the device, the stream the records were produced on."""
        import ctypes
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        n = int(hits.shape[0])
        # a shard whose global document ids overflow the records' 32 bits sends the error flag (a negative count)
        # in the counts exchange: every rank's planned exchange then fails before anything is posted
        counts = self.allgather_counts(-1 if int(doc_base) + n > 0xFFFFFFFF else n, stream)
        total = sum(c for c in counts if c > 0)
        receive = root < 0 or root == self.rank
        if receive and (self._out is None or self._out.shape[0] < max(total, 1)):
            self._out = torch.empty((max(total + total // 4, 1), 4), dtype=torch.int32,
                                    device=torch.device('cuda', self.device))
        out = self._out if receive else None
        nt = ctypes.c_int64()
        cnt = np.asarray(counts, dtype=np.int64)
        # the counts above are this step's one exchange: the records move without a second one
        self._n.check_comm(self._n.lib().kw_allgather_hits_planned(
            self.h, self._n.ptr(hits) if n else None, n, int(doc_base), int(root), self._n.ptr(cnt),
            self._n.ptr(out) if out is not None else None, int(out.shape[0]) if out is not None else 0,
            ctypes.byref(nt), self._sp(stream)), self.h)
        return (out[:total] if receive else None), counts


class Exchange:
    """Moves a rank's hit records ([n, 4] int32, doc ids local to its shard) to rank 0, the writer.

    backend "nccl": libkwmatch's RCCL communicator (:class:`KwComm`, device tensors);
    any other backend (the gloo CPU tests): the torch-collective :func:`gather_hits`."""

    def __init__(self, rank: int, world: int, device, backend: str):
        self.rank, self.world, self.backend = rank, world, backend
        self.device = device
        self.comm = KwComm(rank, world, device) if backend == 'nccl' and world > 1 else None

    def _dev(self):
        import torch
        return torch.device('cuda', self.device if self.device is not None else torch.cuda.current_device()) \
            if self.backend == 'nccl' else torch.device('cpu')

    def allreduce_min(self, values) -> np.ndarray:
        """Element-wise MIN of a small int64 vector over the ranks (the sharded reader's chunk decisions,
        the first failing row of a chunk)."""
        import torch
        import torch.distributed as td
        v = np.ascontiguousarray(values, dtype=np.int64)
        if self.world == 1:
            return v.copy()
        t = torch.from_numpy(v.copy()).to(self._dev())
        td.all_reduce(t, op=td.ReduceOp.MIN)
        return t.cpu().numpy()

    def exchange_objects(self, send: list) -> list:
        """``send[r]`` (a picklable object) goes to rank r; returns what every rank sent to this one, in rank
        order (one gather per destination rank; host-side bookkeeping, e.g. the output files' write index)."""
        if self.world == 1:
            return [send[0]]
        import torch.distributed as td
        recv = None
        for dst in range(self.world):
            lst = [None] * self.world if dst == self.rank else None
            td.gather_object(send[dst], lst, dst=dst)
            if dst == self.rank:
                recv = lst
        return recv

    def barrier(self):
        if self.world > 1:
            import torch.distributed as td
            td.barrier()

    def gather(self, hits, doc_base: int):
        """Records of every rank with batch-global doc ids, in document order, on rank 0 (None elsewhere)."""
        if self.world == 1:
            out = hits.clone()
            if out.numel():
                out[:, 0] += doc_base
            return out
        if self.comm is not None:
            out, _ = self.comm.gather_hits(hits, doc_base, root=0)
            return out
        allh = gather_hits(hits, doc_base, hits.device)
        return allh if self.rank == 0 else None

    def close(self):
        if self.comm is not None:
            self.comm.close()


def shard_range(n_docs: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous document range of a rank (equal counts; the corpus generator's
    documents have identically distributed lengths, so counts balance bytes)."""
    per = n_docs // world
    extra = n_docs % world
    lo = rank * per + min(rank, extra)
    hi = lo + per + (1 if rank < extra else 0)
    return lo, hi


def byte_balanced_ranges(off: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Split documents (offsets of 2n+1 fields) into `world` contiguous ranges of ~equal bytes."""
    n = (len(off) - 1) // 2
    doc_end = off[2::2]
    total = off[-1] - off[0]
    cuts = [0]
    for r in range(1, world):
        target = off[0] + total * r / world
        cuts.append(int(np.searchsorted(doc_end, target, side='left')) + 1)
    cuts.append(n)
    cuts = [min(max(c, 0), n) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


def allgather_counts(count: int, device) -> List[int]:
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [int(count)]
    t = torch.tensor([int(count)], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(x.item()) for x in out]


def gather_hits(hits, doc_base: int, device):
    """All-gather [n, 4] int32 hit records (doc ids made global) from every rank.

    Returns the concatenation in rank order; since ranks own contiguous document
    ranges, rank order is document order.
    """
    import torch
    import torch.distributed as dist
    hits = hits.clone()
    if hits.numel():
        hits[:, 0] += doc_base
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return hits
    counts = allgather_counts(hits.shape[0], device)
    mx = max(counts)
    pad = torch.zeros((mx, 4), dtype=hits.dtype, device=device)
    pad[:hits.shape[0]] = hits
    out = [torch.empty_like(pad) for _ in counts]
    dist.all_gather(out, pad)
    return torch.cat([o[:c] for o, c in zip(out, counts)], dim=0)
