"""CPU, world_size 2 (gloo): the N>1 path of bench.py — contiguous realisation
shards per rank and ONE all-reduce of the int64 error counters — gives the
same counts as a single process over the whole range.  The per-rank compute
is the CPU oracle here (no GPU in this container)."""
import os
import socket

import numpy as np
import pytest

import harness

torch = pytest.importorskip("torch")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    import harness as h  # noqa: F401
    from dsce.parallel import allreduce_counts, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    S = h.setup("default", schemes=("ofdm",), snr_db=[20.0, 35.0])
    first, n = shard_range(0, 128, world, rank, align=64)
    res = h.simulate(S, 11, first, n // 32, ["ofdm"])
    tot = allreduce_counts(res["err"])
    q.put((rank, first, n, tot))
    dist.destroy_process_group()


def test_two_rank_counter_allreduce():
    import torch.multiprocessing as mp
    from dsce.parallel import shard_range
    assert shard_range(0, 128, 2, 0) == (0, 64) and shard_range(0, 128, 2, 1) == (64, 64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(60)
    out.sort()
    assert np.array_equal(out[0][3], out[1][3])
    # single-process reference over the same realisations (2 per rank)
    S = harness.setup("default", schemes=("ofdm",), snr_db=[20.0, 35.0])
    ref = np.zeros_like(out[0][3])
    for _, first, n, _ in out:
        ref += harness.simulate(S, 11, first, n // 32, ["ofdm"])["err"]
    assert np.array_equal(out[0][3], ref)
