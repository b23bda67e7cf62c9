"""Multi-GPU sharding of the article stream (one process per GPU, RCCL over xGMI).

Matching shards with no data-path exchange: every article is independent
(SURVEY.md §8(e)).  Each rank owns a contiguous, byte-balanced range of
documents and a full copy of the compiled KB.  The only collectives are

* ``allgather_counts``  — per-rank hit counts (8 B x world), and
* ``gather_hits``       — the packed 16-B hit records, padded to the largest
                          rank, all-gathered so any rank can write the output.

With backend "nccl" torch.distributed is RCCL on ROCm; "gloo" is used for the
CPU tests.
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
