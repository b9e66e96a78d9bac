"""Data-parallel sharding of the Monte-Carlo loop.

Realisations are independent and the Philox streams are keyed by the global
realisation index, so every rank runs a contiguous slice of [0, R) and the
only exchange is one all-reduce (sum) of the int64 error counters at the end
(RCCL over xGMI with backend 'nccl', gloo on CPU).  Results are bit-identical
for any world size.
"""
from __future__ import annotations

import numpy as np


def shard_range(first_rep, n_rep, world, rank, align=64):
    """Contiguous slice of [first_rep, first_rep + n_rep) for `rank`; slice
    lengths are multiples of `align` (one wavefront of realisations) except
    possibly the last."""
    if n_rep % align:
        raise ValueError("n_rep must be a multiple of %d" % align)
    blocks = n_rep // align
    lo = (blocks * rank) // world
    hi = (blocks * (rank + 1)) // world
    return first_rep + lo * align, (hi - lo) * align


def allreduce_counts(counts, device=None):
    """Sum an int64 counter array over all ranks of the default process group."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(counts))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t)
    return t.cpu().numpy()
