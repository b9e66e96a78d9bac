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
    from dsce.configs import build_setup
    from dsce.parallel import allreduce_counts, shard_range
    from oracle import refsim
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    S = build_setup("default", schemes=("ofdm",), snr_db=[20.0, 35.0])
    sc = S.schemes["ofdm"]
    mm = h.oracle_mmse(S, sc)
    first, n = shard_range(0, 128, world, rank, align=64)
    res = refsim.simulate(11, first, n // 32, h.oracle_chan(S), [h.oracle_scheme(sc)], S.pn_time, S.n_iter, [mm])
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
    from dsce.configs import build_setup
    from oracle import refsim
    S = build_setup("default", schemes=("ofdm",), snr_db=[20.0, 35.0])
    sc = S.schemes["ofdm"]
    mm = harness.oracle_mmse(S, sc)
    ref = np.zeros_like(out[0][3])
    for _, first, n, _ in out:
        ref += refsim.simulate(11, first, n // 32, harness.oracle_chan(S), [harness.oracle_scheme(sc)], S.pn_time,
                               S.n_iter, [mm])["err"]
    assert np.array_equal(out[0][3], ref)
