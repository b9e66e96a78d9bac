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
    """Contiguous slice of [first_rep, first_rep + n_rep) for `rank`.  Slice
    boundaries sit on multiples of `align` (one wavefront of realisations) so
    every rank but the one holding the end of the range runs whole waves; any
    n_rep is allowed (dsce_run pads a partial tail wave and counts only its
    real realisations, so the slices still add up to the one-rank counts)."""
    if n_rep < 0 or align < 1:
        raise ValueError("n_rep must be >= 0 and align >= 1")
    blocks = (n_rep + align - 1) // align
    lo = min((blocks * rank) // world * align, n_rep)
    hi = min((blocks * (rank + 1)) // world * align, n_rep)
    return first_rep + lo, hi - lo


def allreduce_counts(counts, device=None, info=None):
    """Sum a counter array (int64 counts, fp64 MSE sums) over all ranks of the
    default process group.  ``device``: where the reduction runs ('cuda' with
    the nccl backend: RCCL over xGMI reads device tensors).  ``info`` (a dict)
    receives the backend, the tensor's device and the world size of the call."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(counts))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t)
    if info is not None:
        info.update(backend=dist.get_backend(), device=str(t.device), world=dist.get_world_size())
    return t.cpu().numpy()
