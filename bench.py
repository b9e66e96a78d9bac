#!/usr/bin/env python3
"""Headline benchmark: Monte-Carlo channel realisations/s at 24 sc x 14 sym.

Workload (BASELINE.json configs[1], "C2"): OFDM 24 subcarriers x 14 symbols,
N = 540 samples, Jakes 500 km/h @ 2.5 GHz, VehicularA, 256-QAM, 16 pilots,
doubly-selective MMSE channel estimation + 4 interference-cancellation
iterations, 7 SNR points (10:5:40 dB).  One realisation = one iteration of
the Monte-Carlo loop body of DoublySelectiveChannelEstimation.m:350-564 for
this scheme: channel draw + TX + perfect-CSI diag(D), then for every SNR point
noise, demodulation, LS, MMSE one-tap, perfect-CSI one-tap and 4 IC iterations
for both, with bit-error counting (with/without edges).  Setup (correlation
matrices, W) is excluded and reported separately.

A "step" = one pass of the hot path over --reps-per-step realisations
(synthetic Philox inputs).  With N GPUs (torch.distributed.run, one rank per
GPU) every rank processes its own contiguous realisation range (weak scaling,
no collective inside the data path); the int64 error counters are summed with
ONE all-reduce (RCCL) at the end of the timed region.

Prints one JSON line (rank 0).  See DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "channel-estimation_amd")]

METRIC = "Monte-Carlo channel realisations/sec at 24sc x 14sym; BER curve match vs ref"
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 matrix/vector peak (AMD spec)
HBM_PEAK_GBS = 8000.0
SEED = 0x5EED0002


def cpu_baseline_leg(seconds):
    """Oracle (literal NumPy restatement of the reference's dense formulation)
    timed on one host core on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import harness
    from dsce.configs import build_setup
    from oracle import refsim
    S = build_setup("default", schemes=("ofdm",))
    sc = S.schemes["ofdm"]
    mm = harness.oracle_mmse(S, sc)                       # setup, untimed
    chan = harness.oracle_chan(S)
    osc = [harness.oracle_scheme(sc)]
    n = 0
    t0 = time.perf_counter()
    while True:
        refsim.simulate(SEED, 10_000_000 + n, 1, chan, osc, S.pn_time, S.n_iter, [mm])
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 2:
            break
    print(json.dumps({"value": n / el, "reps": n, "seconds": el}))


def run_cpu_baseline(seconds):
    env = dict(os.environ)
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "BLIS_NUM_THREADS"):
        env[k] = "1"
    env["HIP_VISIBLE_DEVICES"] = ""
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-leg", "--cpu-seconds",
                          str(seconds)], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return None
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"value": r["value"], "unit": "realisations/s", "cores": 1, "kind": "port",
            "sample": "oracle/refsim.simulate (dense Q'HG, full(W) contraction, brute-force detection, "
                      "NumPy fp64, 1 thread), %d realisations of the C2 workload in %.1f s" % (r["reps"], r["seconds"])}


def latest_pmc_traffic():
    """HBM bytes per k_wcontract launch from the committed rocprofv3 PMC summary
    (profiles/*_pmc_wcontract.json written by tools/pmc_summary.py), or None."""
    d = os.path.join(ROOT, "profiles")
    if not os.path.isdir(d):
        return None
    c = sorted(f for f in os.listdir(d) if f.endswith("_pmc_wcontract.json"))
    if not c:
        return None
    with open(os.path.join(d, c[-1])) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reps-per-step", type=int, default=65536)
    ap.add_argument("--batch", type=int, default=65536, help="realisations per device batch")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-leg", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_baseline_leg:
        cpu_baseline_leg(args.cpu_seconds)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist
        # one rank per GPU; DSCE_DIST_BACKEND=gloo + more ranks than GPUs rehearses
        # the multi-rank path on a single-GPU box (ranks share device local % count)
        device = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        dist.init_process_group(os.environ.get("DSCE_DIST_BACKEND", "nccl"))

    import numpy as np
    from dsce.configs import build_setup
    from dsce.engine import build_engine

    S = build_setup("default", schemes=("ofdm",))
    t_setup = time.perf_counter()
    eng = build_engine(S, device=device, batch=args.batch)
    setup_s = time.perf_counter() - t_setup
    B = args.reps_per_step
    counts = np.zeros(eng.counter_shape(), dtype=np.int64)
    base = rank * (args.steps + args.warmup) * B
    for w in range(args.warmup):
        eng.run(SEED, base + w * B, B)
    eng.enable_timing(True)
    if dist:
        dist.barrier()
        import torch
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        eng.run(SEED, base + (args.warmup + k) * B, B, counts)
    if dist:
        import torch
        ct = torch.from_numpy(counts).cuda()
        dist.all_reduce(ct)                 # the one exchange: BER counters (RCCL)
        torch.cuda.synchronize()
        counts = ct.cpu().numpy()
    el = time.perf_counter() - t0
    if dist:
        import torch
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_reps = B * args.steps * world
    value = total_reps / el

    # roofline of the dominant kernel (MMSE contraction), HIP events on the engine stream
    launches, wc_ms = eng.kernel_time("k_wcontract")
    cmac_per_rep, w_bytes = eng.work_model(0)
    flops = cmac_per_rep * 8.0 * B * args.steps          # this rank's contraction flops in the timed region
    achieved_tf = flops / (wc_ms * 1e-3) / 1e12 if wc_ms > 0 else None
    traffic = latest_pmc_traffic()
    bits = eng.bits_per_rep(0)
    ber = counts[0, :, 0, :, :] / float(bits[0] * total_reps)
    kernels = {}
    for k in ("k_jakes", "tx", "rx_front", "k_pilot_pre", "k_wcontract", "perfect_ic", "k_stage"):
        n, ms = eng.kernel_time(k)
        kernels[k] = {"launches": n, "ms": round(ms, 3)}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu = run_cpu_baseline(args.cpu_seconds)
        except Exception:
            cpu = None
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "realisations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Philox4x32-10 streams, include/dsce.h)",
        "config": {"workload": "C2: OFDM 24sc x 14sym, N=540, Jakes 500 km/h VehA, 256-QAM, 16 pilots, "
                               "7 SNR (10:5:40 dB) x (one-tap + 4 IC) x (MMSE + perfect CSI)",
                   "reps_per_step_per_gpu": B, "engine_batch": args.batch, "parallelism": "dp%d" % world},
        "roofline": {"bound": "mfma", "kernel": "k_wpair3<24,4,fused> (pair-tile MMSE contraction, 3M, with the "
                               "next stage's diag(D_hat) + detection in its epilogue; timed as k_wcontract)",
                     "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": (achieved_tf / FP64_PEAK_TFLOPS) if achieved_tf else None,
                     "traffic": traffic, "launches": launches,
                     "avg_launch_ms": wc_ms / launches if launches else None,
                     "flops_per_launch": flops / launches if launches else None},
        "cpu_baseline": cpu,
        "setup_s": setup_s,
        "kernels_ms": kernels,
        "ber_40dB": {"mmse_ic4": float(ber[0, -1, -1]), "perfect_ic4": float(ber[1, -1, -1]),
                     "mmse_onetap": float(ber[0, -1, 0]), "perfect_onetap": float(ber[1, -1, 0])},
    }
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
