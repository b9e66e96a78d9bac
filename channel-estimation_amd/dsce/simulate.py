"""Command-line Monte-Carlo run: the reference script's loop and plots
(DoublySelectiveChannelEstimation.m:350-631) on one MI355X, or sharded over the
GPUs of a node (one process per GPU, one all-reduce of the counters and MSE
sums — SURVEY §8e; bit-identical counts for any number of ranks).  Two shard
axes: realisations (contiguous slices, the default) or SNR points (--shard snr:
each rank builds the estimator for its own SNR points only, so the setup is
split too; the noise keeps the sweep's SNR index through the engine's snr_base
option):

    python -m dsce.simulate --config default --reps 4096 --out run.json --figures figs/
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m dsce.simulate --config c5 --reps 10048 --out c5.json     # BASELINE config 5
    python -m dsce.simulate --config c5 --devices 0,1,2,3,4,5,6,7   # one process, one multi-device
                                                                    # context (dsce_create_multi: the
                                                                    # in-library RCCL all-reduce)
    python -m dsce.simulate --config paper --checkpoint ck.json --stop-after 4096   # time-boxed slot
    python -m dsce.simulate --config paper --checkpoint ck.json --resume --out paper.json

Checkpoint / resume (the reference has none): --checkpoint
writes the int64 counters, the MSE sums and the next realisation after every
batch (atomically, one file per rank).  The streams are keyed by the global
realisation index, so a resumed run's counts equal an uninterrupted run's bit
for bit.

Progress lines mirror the script's `disp` (script:567); results go through
dsce.results (JSON [+ NPZ], Figures 2-5)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--config", default="default", help="default (C2-C4) | c5 | paper | doubly_flat (config 1)")
    ap.add_argument("--schemes", default="fbmc_aux,fbmc_cod,ofdm")
    ap.add_argument("--reps", type=int, default=None, help="realisations (any count; default: the config's NrRepetitions)")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--seed", type=int, default=0x5EED0000)
    ap.add_argument("--out", default=None, help="result JSON")
    ap.add_argument("--npz", action="store_true")
    ap.add_argument("--figures", default=None, help="directory for Figure2-5.png")
    ap.add_argument("--mse", action="store_true", help="also accumulate the channel-estimation NMSE per stage")
    ap.add_argument("--interpolation", default="linear",
                    choices=("linear", "nearest", "natural", "FullAverage"),
                    help="doubly_flat: PSACE interpolation method (the script uses 'linear')")
    ap.add_argument("--shard", choices=("reps", "snr"), default="reps",
                    help="multi-rank split: realisation slices (default) or SNR points")
    ap.add_argument("--devices", default=None,
                    help="comma-separated HIP devices of ONE multi-device context (dsce_create_multi, ABI 7): "
                         "the engine shards the realisations and all-reduces the counters itself (RCCL)")
    ap.add_argument("--checkpoint", default=None,
                    help="JSON checkpoint written after every batch (counters, MSE sums, next realisation); "
                         "one file per rank under a launcher (.rankR suffix)")
    ap.add_argument("--resume", action="store_true", help="continue from --checkpoint if it exists")
    ap.add_argument("--stop-after", type=int, default=None,
                    help="process at most this many realisations (per rank) in this invocation, then leave "
                         "the checkpoint for --resume (needs --checkpoint)")
    a = ap.parse_args(argv)
    if (a.resume or a.stop_after is not None) and not a.checkpoint:
        raise SystemExit("--resume / --stop-after need --checkpoint")

    from dsce import results
    from dsce.configs import build_setup
    from dsce.engine import build_engine

    if a.config == "doubly_flat":
        return _doubly_flat(a)

    from dsce.parallel import allreduce_counts, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    device = 0
    # under a launcher (torch.distributed.run sets WORLD_SIZE) the process group
    # and the all-reduce run at every world size, 1 included: the RCCL path of
    # the counters is the same code with one rank or eight
    distributed = "WORLD_SIZE" in os.environ
    devices = [int(d) for d in a.devices.split(",")] if a.devices else None
    if devices and distributed:
        raise SystemExit("--devices is the single-process multi-device path; do not combine it with a launcher")
    if distributed:
        import torch
        import torch.distributed as dist
        # DSCE_DIST_BACKEND=gloo rehearses on a one-GPU box (ranks share the device)
        device = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        dist.init_process_group(os.environ.get("DSCE_DIST_BACKEND", "nccl"))
    names = tuple(a.schemes.split(","))
    from dsce.engine import gpu_tx
    S = build_setup(a.config, schemes=names, tx=gpu_tx(devices[0] if devices else device))   # G / Q on the GPU (row f1)
    reps = a.reps if a.reps is not None else S.n_repetitions    # script:19 / :44, exactly (no rounding)
    if reps < 1:
        raise SystemExit("--reps must be >= 1")
    nsnr = len(S.snr_db)
    if a.shard == "snr":
        # SNR points [s0, s0 + ns) on this rank, every realisation
        s0, ns = shard_range(0, nsnr, world, rank, align=1)
        first, mine = 0, (reps if ns else 0)
        Sr = _snr_subset(S, s0, ns) if ns else None
        options = {"snr_base": s0}
    else:
        s0, ns = 0, nsnr
        first, mine = shard_range(0, reps, world, rank)
        Sr, options = S, {}
    nst = S.n_iter + 1
    counts = np.zeros((len(names), 2, 2, nsnr, nst), dtype=np.int64)
    err = np.zeros((len(names), nsnr, nst))
    pw = np.zeros((len(names), nsnr))
    bits = None
    setup_s, t0 = 0.0, time.perf_counter()
    ck_path = None
    if a.checkpoint:
        ck_path = a.checkpoint + (".rank%d" % rank if world > 1 else "")
    ck_key = {"config": a.config, "schemes": list(names), "seed": int(a.seed), "reps": int(reps),
              "shard": a.shard, "world": world, "rank": rank, "first": int(first), "mine": int(mine),
              "mse": bool(a.mse), "snr": [int(s0), int(ns)]}
    done, prior_s = 0, 0.0
    if mine:                                         # a rank with an empty shard contributes zeros
        eng = build_engine(Sr, device=devices or device, batch=max(64, min(a.batch, mine)), options=options)
        setup_s = time.perf_counter() - t0
        sub = np.zeros(eng.counter_shape(), dtype=np.int64)
        e0 = np.zeros((len(names), ns, nst))
        p0 = np.zeros((len(names), ns))
        if a.resume and os.path.exists(ck_path):
            ck = load_checkpoint(ck_path, ck_key)
            done, prior_s = ck["done"], ck["seconds"]
            sub[...] = np.asarray(ck["counts"], dtype=np.int64).reshape(sub.shape)
            if a.mse:
                e0[...] = np.asarray(ck["mse_err"]).reshape(e0.shape)
                p0[...] = np.asarray(ck["mse_pow"]).reshape(p0.shape)
            if rank == 0:
                print("resumed from %s at realisation %d of %d" % (ck_path, first + done, first + mine), flush=True)
        if a.mse:
            eng.enable_mse()
        t0 = time.perf_counter()
        step = min(a.batch * (len(devices) if devices else 1), mine)
        stop = mine if a.stop_after is None else min(mine, done + max(0, a.stop_after))
        start = done
        while done < stop:
            n = min(step, stop - done)
            eng.run(a.seed, first + done, n, sub)
            done += n
            el = time.perf_counter() - t0
            if ck_path:
                e_, p_ = eng.mse() if a.mse else (None, None)
                save_checkpoint(ck_path, ck_key, done, sub, prior_s + el,
                                (e0 + e_, p0 + p_) if a.mse else None)
            if rank == 0:
                print("%d%% Completed! Time Left: %.1f s"
                      % (100 * done // mine, el / (done - start) * (mine - done)), flush=True)
        counts[:, :, :, s0:s0 + ns, :] = sub
        bits = np.array([eng.bits_per_rep(i) for i in range(len(names))])
        if a.mse:
            e_, p_ = eng.mse()
            err[:, s0:s0 + ns, :] = e0 + e_
            pw[:, s0:s0 + ns] = p0 + p_
        eng.close()
    complete = done >= mine
    if distributed:
        # every rank must take the same branch before the collectives below
        import torch
        import torch.distributed as dist
        f = torch.tensor([0 if complete else 1], dtype=torch.int64)
        if os.environ.get("DSCE_DIST_BACKEND", "nccl") == "nccl":
            f = f.to("cuda")
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        if int(f.item()):
            complete = False
    if not complete:
        if rank == 0:
            print("stopped at realisation %d of %d; resume with --checkpoint %s --resume"
                  % (first + done, first + mine, a.checkpoint), flush=True)
        if distributed:
            dist.destroy_process_group()
        return 0
    extra = {"setup_s": setup_s, "seconds": prior_s + time.perf_counter() - t0, "ranks": world, "shard": a.shard}
    if ck_path and a.resume:
        extra["resumed"] = True
    if devices:
        extra["devices"] = devices
    if distributed:
        dev = "cuda" if os.environ.get("DSCE_DIST_BACKEND", "nccl") == "nccl" else None
        info = {}
        counts = allreduce_counts(counts, dev, info)              # the one exchange
        extra["allreduce"] = info
        if a.mse:
            err = allreduce_counts(err, dev)
            pw = allreduce_counts(pw, dev)
        # bits per realisation are a property of the schemes: every rank with work
        # has them (collective on every rank, so a rank with an empty shard too)
        have = np.array([0 if bits is None else 1], dtype=np.int64)
        b = np.zeros((len(names), 2), dtype=np.int64) if bits is None else np.asarray(bits, dtype=np.int64)
        b = allreduce_counts(b, dev)
        have = allreduce_counts(have, dev)
        bits = b // max(1, int(have[0]))
        import torch
        import torch.distributed as dist
        t = torch.tensor([extra["seconds"]], dtype=torch.float64)
        if dev:
            t = t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        extra["seconds"] = float(t.item())
    if a.mse:
        extra["nmse"] = {s: (err[i] / pw[i][:, None]).tolist() for i, s in enumerate(names)}
    extra["realisations_per_s"] = reps / extra["seconds"]
    res = results.make(S, names, counts, bits, reps, a.seed, extra=extra)
    if rank != 0:
        if distributed:
            dist.destroy_process_group()
        return 0
    if a.out:
        results.save(a.out, res, npz=a.npz)
    if a.figures:
        os.makedirs(a.figures, exist_ok=True)
        for f in results.figures(res, a.figures):
            print("wrote", f)
    k = len(S.snr_db) - 1
    summary = {s: {"snr_db": float(S.snr_db[k]),
                   "ber_ic_mmse": float(res["ber"][s]["mmse"]["all"][k][-1]),
                   "ber_onetap_mmse": float(res["ber"][s]["mmse"]["all"][k][0])} for s in names}
    print(json.dumps(summary))
    if distributed:
        dist.destroy_process_group()
    return 0


CHECKPOINT_VERSION = 1


def save_checkpoint(path, key, done, counts, seconds, mse=None):
    """Write the run state atomically (a temporary file, then os.replace): a
    crash while writing leaves the previous checkpoint intact."""
    d = {"version": CHECKPOINT_VERSION, "key": key, "done": int(done), "seconds": float(seconds),
         "counts": np.asarray(counts, dtype=np.int64).ravel().tolist()}
    if mse is not None:
        d["mse_err"] = np.asarray(mse[0]).ravel().tolist()
        d["mse_pow"] = np.asarray(mse[1]).ravel().tolist()
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(d, f)
    os.replace(tmp, path)


def load_checkpoint(path, key):
    """The checkpoint at `path` if it belongs to this run (same configuration,
    schemes, seed, realisation count, shard and rank); anything else is an
    error, never a silent restart or a mixed result."""
    with open(path) as f:
        d = json.load(f)
    if d.get("version") != CHECKPOINT_VERSION:
        raise SystemExit("checkpoint %s: version %r, expected %d" % (path, d.get("version"), CHECKPOINT_VERSION))
    if d.get("key") != key:
        diff = sorted(k for k in set(key) | set(d.get("key", {})) if d.get("key", {}).get(k) != key.get(k))
        raise SystemExit("checkpoint %s belongs to another run (differs in %s)" % (path, ", ".join(diff)))
    if not 0 <= int(d["done"]) <= key["mine"]:
        raise SystemExit("checkpoint %s: realisation count out of range" % path)
    return d


def _snr_subset(S, s0, ns):
    """The setup namespace with SNR points [s0, s0 + ns) only (pn_time, snr_db)."""
    import copy
    T = copy.copy(S)
    T.pn_time = np.asarray(S.pn_time)[s0:s0 + ns]
    T.snr_db = np.asarray(S.snr_db)[s0:s0 + ns]
    return T


def _doubly_flat(a):
    """SimpleVersion_DoublyFlat.m:89-195 (BASELINE config 1) on one GPU."""
    from dsce import results
    from dsce.doubly_flat import DoublyFlatSim

    from dsce.configs import build_doubly_flat_setup
    t0 = time.perf_counter()
    sim = DoublyFlatSim(build_doubly_flat_setup(interpolation=a.interpolation), batch=a.batch)
    setup_s = time.perf_counter() - t0
    S = sim.setup
    reps = a.reps if a.reps is not None else S.n_repetitions    # SimpleVersion_DoublyFlat.m:13, exactly
    if reps < 1:
        raise SystemExit("--reps must be >= 1")
    t0 = time.perf_counter()
    counts = sim.run(a.seed, 0, reps)
    secs = time.perf_counter() - t0
    q = S.schemes["ofdm"].const
    snr_f = np.arange(S.snr_db.min(), S.snr_db.max() + 0.25, 0.5)                     # :180
    theory = _theory(snr_f, q.SymbolMapping, q.BitMapping)
    res = results.doubly_flat_result(sim, counts, reps, a.seed, (snr_f, theory),
                                     extra={"setup_s": setup_s, "seconds": secs,
                                            "realisations_per_s": reps * len(S.snr_db) / secs})
    if a.out:
        results.save(a.out, res)
    if a.figures:
        os.makedirs(a.figures, exist_ok=True)
        print("wrote", results.doubly_flat_figure(res, os.path.join(a.figures, "DoublyFlat.png")))
    print(json.dumps({k: [round(x, 6) for x in v] for k, v in res["ber"].items()}))
    sim.close()
    return 0


def _theory(snr_db, symbols, bitmap):
    """Theory/BitErrorProbabilityDoublyFlatRayleigh.m (host restatement in the
    product package: the plotted reference curve, not a checker)."""
    from dsce.theory import bit_error_probability_doubly_flat_rayleigh
    return bit_error_probability_doubly_flat_rayleigh(snr_db, symbols, bitmap)


if __name__ == "__main__":
    sys.exit(main())
