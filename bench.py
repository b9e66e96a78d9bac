#!/usr/bin/env python3
"""Headline benchmark: Monte-Carlo channel realisations/s at 24 sc x 14 sym.

Workload (BASELINE.json configs[1], "C2", the default): OFDM 24 subcarriers x
14 symbols, N = 540 samples, Jakes 500 km/h @ 2.5 GHz, VehicularA, 256-QAM,
16 pilots, doubly-selective MMSE channel estimation + 4 interference-
cancellation iterations, 7 SNR points (10:5:40 dB).  One realisation = one
iteration of the Monte-Carlo loop body of DoublySelectiveChannelEstimation.m:
350-564 for this scheme: channel draw + TX + perfect-CSI diag(D), then for
every SNR point noise, demodulation, LS, MMSE one-tap, perfect-CSI one-tap and
4 IC iterations for both, with bit-error counting (with/without edges).  Setup
(correlation matrices, W) is excluded and reported separately.
``--config c3|c4|c5`` measures the other single-GPU configurations the same
way (FBMC auxiliary / data-spreading 24 x 30; 48 x 30 at SR 720 kHz with the
three schemes and 16 SNR points).

A "step" = one pass of the hot path over --reps-per-step realisations
(synthetic Philox inputs, generated on the device).  With N GPUs (one rank per
GPU, torch.distributed) every rank processes its own contiguous realisation
range (weak scaling, no collective inside the data path); the int64 error
counters are summed with ONE all-reduce (RCCL) after the timed steps.
``--gpus N`` without a launcher starts ``torch.distributed.run`` itself (as a
child process) and forwards rank 0's line.

Prints one JSON line (rank 0).  See DESIGN.md §6.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "channel-estimation_amd")]

METRIC = "Monte-Carlo channel realisations/sec at 24sc x 14sym; BER curve match vs ref"
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 matrix peak (AMD spec) — measured value reported beside it
HBM_PEAK_GBS = 8000.0
SEED = 0x5EED0002

# workload -> (setup name, schemes, default reps per step (= engine batch), description)
WORKLOADS = {
    "c2": ("default", ("ofdm",), 65536,
           "C2: OFDM 24sc x 14sym, N=540, Jakes 500 km/h VehA, 256-QAM, 16 pilots, 7 SNR (10:5:40 dB) x "
           "(one-tap + 4 IC) x (MMSE + perfect CSI)"),
    "c3": ("default", ("fbmc_aux",), 32768,
           "C3: FBMC-OQAM auxiliary-symbol pilots 24sc x 30sym, N=540, PAM-16, 16 pilots + 64 aux, 7 SNR x "
           "(one-tap + 4 IC) x (MMSE + perfect CSI)"),
    "c4": ("default", ("fbmc_cod",), 32768,
           "C4: FBMC-OQAM data-spreading pilots 24sc x 30sym, N=540, PAM-16, 7 SNR x (one-tap + 4 IC) x "
           "(MMSE + perfect CSI)"),
    "c5": ("c5", ("fbmc_aux", "fbmc_cod", "ofdm"), 8192,
           "C5: 48sc x 30sym (OFDM 48x14) at SR 720 kHz, N=1080, 32 pilots, 3 taps, 16 SNR (10:2:40 dB), "
           "3 schemes x (one-tap + 4 IC) x (MMSE + perfect CSI)"),
}


# the roofline object's description of each kernel group (bench line `roofline.kernel`)
KERNEL_DESC = {
    "perfect_ic": ("k_pic_fft: the perfect-CSI branch of every FFT-form OFDM symbol, stage 0 one-tap + the 4 IC "
                   "iterations (script:428-466, :541-561) with u, y / h, 1 / h and the taps in registers: per "
                   "iteration y - (D - diag h) u by IDFT-24 (prime-factor DFT-6 per lane + 4-point network on "
                   "v_mfma_f64_4x4x4f64), the channel's taps, DFT-24, then one-tap, slicer, counts, re-precoding; "
                   "FP64 roofline (f64 VALU and MFMA share the SIMD's issue on gfx950; peak 78.6 TF)"),
    "k_mic_data": ("k_mic_data: every MMSE stage (one-tap + IC iterations) of the OFDM symbols without pilots, "
                   "decisions in registers: per stage the estimated taps H_hat = T_k Z (low-rank operator, Z = Bz hP "
                   "from k_mic_pilot), y - Q'(H_hat (G v)) + diag(D_hat) v by the DFT-24 chain, one-tap + detection; "
                   "FP64 roofline (VALU and MFMA share the issue)"),
    "k_mic_pilot": "k_mic_pilot: every MMSE stage of the pilot symbols, LS pilots and Z = Bz hP per stage",
    "ic_stages": ("the IC group of every FFT-form OFDM symbol (stage 0 + 4 IC iterations, both CSI branches): "
                  "k_pic_fft (perfect CSI, script:428-466 / :541-561) on a second stream beside k_mic_pilot -> "
                  "k_mic_data (MMSE, script:417-537); per stage and symbol the DFT-24 chain (prime-factor DFT-6 "
                  "per lane + the 4-point network on v_mfma_f64_4x4x4f64) with the true or the low-rank estimated "
                  "taps, one-tap, slicer, counts; FP64 roofline (f64 VALU and MFMA share the SIMD's issue, 78.6 TF); "
                  "time = the group's span on the engine's main stream (HIP events: fork before, join after)"),
    "rx_front": ("k_txrx_fft: TX IDFT-24, the doubly-selective channel, and per SNR point the AWGN draw (Philox4x32-10 "
                 "+ table-driven Box-Muller) and the receiver DFT-24"),
    "k_jakes": "k_jakes_grp: the Jakes sum-of-sinusoids taps at the samples the receiver windows read",
    "tx": "k_tx_rows: bits -> Gray -> P [xP; xD]",
}


def source_hash():
    """sha256 over the engine's sources: stamps PMC profiles to the build they measured."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "channel-estimation_amd", "csrc", "*"))) + [
        os.path.join(ROOT, "include", "dsce.h"), os.path.join(ROOT, "channel-estimation_amd", "Makefile")]
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode())
            h.update(fh.read())
    return h.hexdigest()[:16]


# ---------------------------------------------------------------------------
# CPU baseline: the oracle (literal NumPy restatement of the reference's dense
# formulation) on the GPU box's host cores, bounded sample, median of 3
# ---------------------------------------------------------------------------
# the oracle holds full(W) and full(W0) of every SNR point and scheme (complex,
# LK^2 NP each): above this many bytes per process a leg times 1 and 2 SNR
# points and extrapolates (C5: ~100 GB); C2 / C3 / C4 (0.4 / 1.9 / 1.9 GB) are
# timed on the whole workload
ORACLE_W_BYTES_MAX = 8e9


def oracle_w_bytes(S, schemes):
    return sum(2 * len(S.pn_time) * S.schemes[s]["G"].shape[1] ** 2 * len(S.schemes[s]["pilot_pos"]) * 16
               for s in schemes)


def cpu_baseline_leg(seconds, workload, index=0):
    """One process of the CPU baseline: oracle/refsim.simulate on single
    realisations of the whole workload (every SNR point, both CSI branches, all
    IC iterations), 3 timed samples of seconds / 3 each.  Only a workload whose
    full(W) exceeds ORACLE_W_BYTES_MAX per process (C5) times the first 1 and 2
    SNR points and extrapolates: cost(nsnr) = c1 + (nsnr - 1) (c2 - c1) from the
    medians, flagged invalid when the slope is not positive or the samples'
    spread exceeds it."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import harness
    from oracle import refsim
    name, schemes, _, _ = WORKLOADS[workload]
    S = harness.setup(name, schemes=schemes)
    chan = S.chan
    osc = [S.schemes[s] for s in schemes]
    base = 10_000_000 + 1_000_000 * index            # disjoint realisations per pool process
    nsnr = len(S.pn_time)

    def timed(pn, mm, secs):
        refsim.simulate(SEED, base + 900_000, 1, chan, osc, pn, S.n_iter, mm)   # warm-up
        rates, n_total = [], 0
        for _ in range(3):
            n, t0 = 0, time.perf_counter()
            while True:
                refsim.simulate(SEED, base + n_total, 1, chan, osc, pn, S.n_iter, mm)
                n += 1
                n_total += 1
                el = time.perf_counter() - t0
                if el >= secs / 3:
                    break
            rates.append(n / el)
        return rates, n_total

    out = {"snr_points": nsnr}
    if oracle_w_bytes(S, schemes) <= ORACLE_W_BYTES_MAX:
        mm = [harness.oracle_mmse(S, s) for s in schemes]          # setup, untimed
        rates, reps = timed(S.pn_time, mm, seconds)
        out["timed_snr_points"] = nsnr
    else:
        tc = refsim.time_correlation(S.N, chan["dt"], chan["fD"], chan["model"])
        R_vecH = refsim.correlation_matrix(S.N, chan["pdp_norm"], tc)
        cost, reps = {}, 0
        for k in (1, 2):
            pn = S.pn_time[:k]
            mm = [refsim.mmse_setup(R_vecH, S.N, S.schemes[s]["G"], S.schemes[s]["Q"], S.schemes[s]["P"],
                                    S.schemes[s]["pilot_pos"], S.schemes[s]["kappa"], pn, S.zero_threshold)
                  for s in schemes]
            r, n = timed(pn, mm, seconds / 2)
            cost[k] = [1.0 / x for x in r]
            reps += n
            del mm
        c1, c2 = statistics.median(cost[1]), statistics.median(cost[2])
        slope = c2 - c1
        spread = max(max(cost[1]) - min(cost[1]), max(cost[2]) - min(cost[2]))
        ok = slope > 0 and spread < slope
        # one value per sample pairing around the medians' fit: the fit itself
        # and the fits through the extreme samples (a spread, not a median of 3)
        rates = [1.0 / (c1 + (nsnr - 1) * slope)] if ok else []
        if ok:
            lo, hi = min(cost[1]) + (nsnr - 1) * max(slope - spread, 0.0), max(cost[1]) + (nsnr - 1) * (slope + spread)
            rates = [1.0 / hi, rates[0], 1.0 / lo] if lo > 0 else [1.0 / hi, rates[0]]
        out["extrapolated"] = {"snr_points_timed": [1, 2], "snr_points": nsnr, "valid": ok,
                               "cost_1snr_s": cost[1], "cost_2snr_s": cost[2], "slope_s_per_snr": slope,
                               "sample_spread_s": spread,
                               "model": "cost = c1 + (nsnr - 1) (c2 - c1), medians of 3 samples each; invalid when "
                                        "c2 <= c1 or the spread of the samples exceeds c2 - c1"}
    import resource
    out.update({"rates": rates, "reps": reps,
                "maxrss_bytes": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024})
    print(json.dumps(out))


def host_info():
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Thread(s) per core", "Core(s) per socket"):
                info[k.strip()] = v.strip()
    except Exception:
        pass
    return info


def _leg_env(threads=1):
    env = dict(os.environ)
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS", "BLIS_NUM_THREADS"):
        env[k] = str(threads)
    env["HIP_VISIBLE_DEVICES"] = ""
    return env


def progress(msg):
    """A heartbeat on stderr (the GPU runner kills a command silent for 3 minutes)."""
    print("[bench %.0fs] %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


T_START = time.perf_counter()
HOST_MEM_BUDGET = 160e9          # bytes the CPU-baseline pool may hold at once


def _wait_all(procs, timeout):
    t0 = last = time.perf_counter()
    while any(p.poll() is None for p in procs):
        if time.perf_counter() - t0 > timeout:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(1.0)
        if time.perf_counter() - last >= 30.0:
            last = time.perf_counter()
            progress("cpu baseline: %d of %d processes running" % (sum(p.poll() is None for p in procs), len(procs)))


def _spread(x):
    return {"median": statistics.median(x), "min": min(x), "max": max(x), "n": len(x)} if x else None


def run_cpu_baseline(seconds, workload):
    """Two legs of the oracle on the host, each about seconds / 2: one process
    with single-threaded BLAS, and a pool of P such processes running at once
    on disjoint realisations.  P = the CPUs this job may use: the scheduler
    affinity, capped by OMP_NUM_THREADS when it is set (the GPU box exports 16,
    its CPU share, while the affinity mask shows the whole host) and by memory.
    Per-realisation NumPy work is too small for BLAS threading (r02: 16 BLAS
    threads ran slower than one), so the all-core baseline is the process pool:
    its value is the sum of the processes' median rates.  Each leg reports the
    median and the spread (min / max) of its 3 samples."""
    host = host_info()
    aff = host.get("affinity") or host["nproc"]
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    pool = max(1, min(aff, omp) if omp else aff)
    reason = ("OMP_NUM_THREADS=%d (the job's CPU share) within an affinity of %d CPUs" % (omp, aff) if omp and omp < aff
              else "the scheduler affinity (%d CPUs)" % aff)
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-leg", "--cpu-seconds", str(seconds / 2),
           "--config", workload]
    progress("cpu baseline: one process")
    one = subprocess.Popen(cmd, env=_leg_env(), stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    _wait_all([one], 900)
    out1, _ = one.communicate()
    if one.returncode != 0:
        return None
    leg1 = json.loads(out1.strip().splitlines()[-1])
    if not leg1["rates"]:
        return {"value": None, "unit": "realisations/s", "kind": "port", "invalid": leg1.get("extrapolated")}
    # the pool within the host memory one command may use (the GPU box caps it at
    # ~270 GB; C5's oracle setup holds the dense W of three schemes per process)
    pmem = max(1, int(HOST_MEM_BUDGET / max(leg1.get("maxrss_bytes", 1), 1)))
    if pmem < pool:
        reason += ", capped to %d by memory (%.1f GB per process into %.0f GB)" % (
            pmem, leg1.get("maxrss_bytes", 0) / 1e9, HOST_MEM_BUDGET / 1e9)
        pool = pmem
    progress("cpu baseline: %d processes" % pool)
    procs = [subprocess.Popen(cmd + ["--leg-index", str(i + 1)], env=_leg_env(), stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, text=True) for i in range(pool)]
    _wait_all(procs, 900)
    legs = []
    for pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            return None
        legs.append(json.loads(out.strip().splitlines()[-1]))
    if any(not l["rates"] for l in legs):
        return None
    v1 = statistics.median(leg1["rates"])
    vp = sum(statistics.median(l["rates"]) for l in legs)
    # the pool's spread: the sum over processes of each one's min / max sample
    pool_spread = {"median": vp, "min": sum(min(l["rates"]) for l in legs),
                   "max": sum(max(l["rates"]) for l in legs), "n": 3}
    ext = leg1.get("extrapolated")
    timed_all = ext is None
    return {"value": max(v1, vp), "unit": "realisations/s", "cores": pool if vp >= v1 else 1, "kind": "port",
            "value_1t": v1, "value_pool": vp, "pool_processes": pool, "pool_reason": reason,
            "one_process": _spread(leg1["rates"]), "pool": pool_spread,
            "samples_1t": leg1["rates"], "samples_pool": [l["rates"] for l in legs],
            "timed": "the whole workload (every SNR point)" if timed_all else
                     "extrapolated from 1 and 2 SNR points (the oracle's full(W) of all %d exceeds %.0f GB per process)"
                     % (leg1["snr_points"], ORACLE_W_BYTES_MAX / 1e9),
            "extrapolated": ext,
            "label": "CPU restatement of reference algorithm, not MATLAB",
            "sample": "oracle/refsim.simulate (dense Q'HG zgemm, full(W) reshape-and-sum contraction, brute-force "
                      "nearest-neighbour detection, NumPy/OpenBLAS fp64, 1 BLAS thread per process) on %s: one "
                      "process, then %d concurrent processes on disjoint realisations; 3 samples of ~%.0f s per "
                      "process, median; %d + %d realisations"
                      % (workload.upper(), pool, seconds / 6, leg1["reps"], sum(l["reps"] for l in legs)),
            "host": host}


def stored_pmc(kernel_tag, workload):
    """The committed rocprofv3 PMC summary of the dominant kernel
    (profiles/*_pmc_*.json, tools/prof_summary.py: HBM bytes per launch and the
    SQ counters per launch), used only when it was measured on a build of these
    exact sources, this workload and kernel.  Returns (summary or None, source)."""
    src = source_hash()
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_*.json")))
    for f in reversed(cands):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("source_hash") == src and d.get("workload", "c2") == workload and \
                d.get("kernel", "k_wcontract") == kernel_tag:
            return d, "profiles/" + os.path.basename(f)
    return None, "no PMC profile of this source build (%s) for %s under profiles/" % (src, workload)


def dominant_by_time(kernels, roof_kernel):
    """The kernel group with the largest share of the measured step, with its own
    algorithmic rate and limiter (bench line `kernels`), or None when that is the
    roofline kernel itself."""
    if not kernels:
        return None
    k, e = max(kernels.items(), key=lambda kv: kv[1].get("ms_per_step") or 0.0)
    if k == roof_kernel:
        return None
    keys = ("ms_per_step", "share", "tflops", "frac_fp64", "traffic_per_launch", "valu_issue", "mfma_busy", "limiter")
    return dict({"kernel": k}, **{kk: e.get(kk) for kk in keys})


def stored_pmc_all(workload):
    """The committed per-kernel-group PMC summary (profiles/*_pmc_all.json,
    tools/prof_summary.py --all) of THIS source build and workload, or None."""
    src = source_hash()
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_all.json")))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("source_hash") == src and d.get("workload") == workload:
            return d.get("kernels"), "profiles/" + os.path.basename(f)
    return None, "no per-kernel PMC profile of this source build (%s) for %s under profiles/" % (src, workload)


SIMDS = 1024                   # 256 CUs x 4 SIMDs (MI355X)


def derive_limiter(pmc, achieved_tf, avg_ms):
    """What bounds the kernel, from the stamped PMC summary of THIS build (None
    without one).  Kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs,
    MI355X_MICROARCH.md, DVFS note); per SIMD and cycle:
      valu_issue   = SQ_INSTS_VALU x 4 / (SIMDS x cycles)   (a 64-lane FP64 VALU op
                     occupies a 16-lane SIMD 4 cycles)
      mfma_busy    = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDS x cycles)
      waves/SIMD   = SQ_WAVE_CYCLES x 4 / (SIMDS x cycles)  (quad-cycles)
      wait         = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES      (share of wave time stalled on a dependency)
      hbm          = HBM bytes per launch / launch time / 8 TB/s
      fp64         = achieved / 78.6 TF (VALU and MFMA FP64 share that peak)
      issue        = valu_issue + mfma_busy: f64 VALU and f64 MFMA instructions do
                     not overlap on gfx950 (tools/ubench: a 4x4x4 MFMA beside f64
                     FMAs costs the sum of both), so together they are one pipe
    The limiter is the largest single utilisation when it reaches 0.7, else the
    shared FP64 issue when VALU + MFMA reach 0.7, else issue latency."""
    if not pmc:
        return None
    sq = pmc.get("sq_per_launch") or {}
    need = ("GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY")
    if any(sq.get(k) is None for k in need) or not sq["GRBM_GUI_ACTIVE"]:
        return None
    cyc = sq["GRBM_GUI_ACTIVE"] / 8.0
    d = {"valu_issue": sq["SQ_INSTS_VALU"] * 4.0 / (SIMDS * cyc),
         "mfma_busy": sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc),
         "waves_per_simd": sq["SQ_WAVE_CYCLES"] * 4.0 / (SIMDS * cyc),
         "wait_frac": sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"] if sq["SQ_WAVE_CYCLES"] else None,
         "valu_per_mfma": sq["SQ_INSTS_VALU"] / sq["SQ_INSTS_MFMA"] if sq.get("SQ_INSTS_MFMA") else None,
         "eff_clock_ghz": cyc / (pmc["avg_duration_ns_rocprof"] * 1e-9) / 1e9 if pmc.get("avg_duration_ns_rocprof") else None,
         "hbm": (pmc["hbm_bytes_per_launch"] / (avg_ms * 1e-3) / (HBM_PEAK_GBS * 1e9))
         if pmc.get("hbm_bytes_per_launch") and avg_ms else None,
         "fp64": achieved_tf / FP64_PEAK_TFLOPS if achieved_tf else None}
    d["issue"] = d["valu_issue"] + d["mfma_busy"]
    util = {k: d[k] for k in ("valu_issue", "mfma_busy", "hbm") if d[k] is not None}
    top = max(util, key=util.get)
    if util[top] < 0.7 and d["issue"] >= 0.7:
        top, util["issue"] = "issue", d["issue"]      # neither alone, but together they fill the issue
    if util[top] >= 0.7:
        d["limiter"] = {"issue": "FP64 issue: VALU %.2f + matrix cores %.2f of the SIMD's cycles (they share it)" % (
                            d["valu_issue"], d["mfma_busy"]),
                        "valu_issue": "VALU issue", "mfma_busy": "matrix cores", "hbm": "HBM bandwidth"}[top]
    else:
        d["limiter"] = "issue latency (%.1f waves/SIMD, %.0f %% of wave cycles stalled on dependencies)" % (
            d["waves_per_simd"], 100 * (d["wait_frac"] or 0))
    d["source"] = "PMC counters of this build (derive_limiter in bench.py)"
    return {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items()}


# ---------------------------------------------------------------------------
def launch_ranks(args):
    """--gpus N > 1 without a launcher: one rank per GPU via torch.distributed.run,
    started as a child process before anything touches the GPU."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    p = subprocess.run(cmd, capture_output=True, text=True)
    line = None
    for ln in p.stdout.splitlines():
        if ln.startswith("{") and '"metric"' in ln:
            line = ln
    if p.returncode != 0 or line is None:
        sys.stderr.write(p.stdout[-4000:] + p.stderr[-4000:])
        return p.returncode or 1
    print(line)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: C2 100 timed steps after 10 warm-up (about 1 s timed: steady
    # state), the slower configurations 10 after 2
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--reps-per-step", type=int, default=0, help="realisations per step per GPU (0: workload default)")
    ap.add_argument("--batch", type=int, default=0, help="realisations per device batch (0: = reps per step)")
    ap.add_argument("--option", action="append", default=[], help="engine option name=value (dsce_set_option)")
    ap.add_argument("--cpu-seconds", type=float, default=24.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-leg", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--leg-index", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 100 if args.config == "c2" else 10
    if args.warmup is None:
        args.warmup = 10 if args.config == "c2" else 2
    if args.cpu_baseline_leg:
        cpu_baseline_leg(args.cpu_seconds, args.config, args.leg_index)
        return 0

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args)
    world = int(env_world or "1")
    if world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%d\n" % (args.gpus, world))
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local
    # under a launcher (WORLD_SIZE set) the process group and the counters'
    # all-reduce run at every world size, 1 included (the RCCL path exercised)
    if env_world is not None:
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

    setup_name, schemes, default_reps, desc = WORKLOADS[args.config]
    B = args.reps_per_step or default_reps
    batch = args.batch or B
    options = {}
    for kv in args.option:
        k, v = kv.split("=")
        options[k.strip()] = int(v)
    from dsce.engine import gpu_tx
    S = build_setup(setup_name, schemes=schemes, tx=gpu_tx(device))       # G / Q produced on the GPU (row f1)
    t_setup = time.perf_counter()
    eng = build_engine(S, device=device, batch=batch, options=options)
    setup_s = time.perf_counter() - t_setup
    if rank == 0:
        progress("setup done (%.1f s)" % setup_s)
    counts = np.zeros(eng.counter_shape(), dtype=np.int64)
    base = rank * (args.steps + args.warmup) * B
    for w in range(args.warmup):
        eng.run(SEED, base + w * B, B)
    eng.enable_timing(True)
    if dist:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        eng.run(SEED, base + (args.warmup + k) * B, B, counts)
    if dist:
        import torch
        torch.cuda.synchronize()
        dist.barrier()
    el = time.perf_counter() - t0
    if rank == 0:
        progress("%d timed steps: %.3f s" % (args.steps, el))
    allreduce = None
    if dist:
        import torch
        from dsce.parallel import allreduce_counts
        dev = "cuda" if os.environ.get("DSCE_DIST_BACKEND", "nccl") == "nccl" else "cpu"
        allreduce = {}
        counts = allreduce_counts(counts, dev, allreduce)     # the one exchange: BER counters (RCCL)
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_reps = B * args.steps * world
    value = total_reps / el

    # every timed kernel group on its own roofline (dsce_kernel_work: algorithmic
    # flops and compulsory bytes per realisation), plus the step as a whole
    pmc_all, pmc_all_src = stored_pmc_all(args.config)
    kernels = {}
    step_flops = 0.0
    modelled_ms = 0.0
    for k in ("k_jakes", "tx", "rx_front", "k_pilot_pre", "k_wcontract", "k_mic_pilot", "k_mic_data",
              "perfect_ic", "k_stage", "ic_stages"):
        n, ms = eng.kernel_time(k)
        if not n:
            continue
        fr, br = eng.kernel_work(k)
        ent = {"launches": n, "ms_per_step": round(ms / args.steps, 4), "share": None,
               "flops_per_rep": fr or None, "bytes_per_rep": br or None}
        if fr and ms > 0:
            tf = fr * B * args.steps / (ms * 1e-3) / 1e12
            ent["tflops"] = round(tf, 3)
            ent["frac_fp64"] = round(tf / FP64_PEAK_TFLOPS, 4)
            step_flops += fr * B
            modelled_ms += ms
        if br and ms > 0:
            gbs = br * B * args.steps / (ms * 1e-3) / 1e9
            ent["algorithmic_gbs"] = round(gbs, 1)
            ent["frac_hbm_algorithmic"] = round(gbs / HBM_PEAK_GBS, 4)
        kp = (pmc_all or {}).get(k)
        if kp and kp.get("hbm_bytes_per_launch") and ms > 0:
            ent["traffic_per_launch"] = kp["hbm_bytes_per_launch"]
            ent["frac_hbm_measured"] = round(kp["hbm_bytes_per_launch"] * n / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 4)
            if kp.get("sq_per_launch"):
                lk = derive_limiter({"sq_per_launch": kp["sq_per_launch"], "hbm_bytes_per_launch":
                                     kp["hbm_bytes_per_launch"], "avg_duration_ns_rocprof": kp.get("avg_duration_ns_rocprof")},
                                    ent.get("tflops"), ms / n)
                if lk:
                    ent["valu_issue"], ent["mfma_busy"], ent["limiter"] = lk["valu_issue"], lk["mfma_busy"], lk["limiter"]
        kernels[k] = ent
    # the FFT-form OFDM IC group: "ic_stages" spans k_pic_fft -> k_mic_pilot ->
    # k_mic_data on the one stream, so it only repeats its members' sum (not
    # counted twice; r06 retired the overlapping ic_streams variants)
    members = ()
    if "ic_stages" in kernels:
        ent = kernels.pop("ic_stages")
        if ent.get("flops_per_rep"):
            step_flops -= ent["flops_per_rep"] * B
            modelled_ms -= eng.kernel_time("ic_stages")[1]
    tot_ms = sum(eng.kernel_time(k)[1] for k in kernels if k not in members)
    for k in kernels:
        kernels[k]["share"] = round(eng.kernel_time(k)[1] / tot_ms, 4) if tot_ms else None
    step_ms = el / args.steps * 1e3
    step_roof = {"flops_per_step": step_flops, "tflops": step_flops / (step_ms * 1e-3) / 1e12 if step_ms else None,
                 "frac_fp64": step_flops / (step_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS if step_ms else None,
                 "kernel_ms_modelled_share": modelled_ms / tot_ms if tot_ms else None,
                 "note": "algorithmic flops of every modelled kernel group per step / wall time per step / 78.6 TF"}

    # the roofline object: the DOMINANT kernel group by measured time (HIP events
    # on the engine's stream) among those with a work model (C2's
    # perfect-CSI chain k_pic_fft became the largest in r04)
    paths = [eng.path_info(sid) for sid in range(len(schemes))]
    kname = max((k for k in kernels if kernels[k].get("flops_per_rep") and k not in members),
                key=lambda k: kernels[k]["ms_per_step"])
    launches, k_ms = eng.kernel_time(kname)
    avg_ms = k_ms / launches if launches else None
    peak_meas = eng.fp64_mfma_peak()
    contraction = kname == "k_wcontract"
    if contraction:
        # the W contraction: 3M on the matrix cores; the roofline rate counts the
        # flops the matrix cores execute (its 8-flop equivalent exceeds the peak:
        # VERDICT r03 #6), traffic and counters from its own stamped PMC summary
        flops = executed = 0.0
        for sid, p in enumerate(paths):
            if "mic_stages" in p:
                continue
            cmac_per_rep, _ = eng.work_model(sid)
            f = cmac_per_rep * 8.0 * B * args.steps
            flops += f
            executed += f * (0.75 if {"wpair3", "wpair3_fused", "wrow3"} & p else 1.0)
        achieved_tf = flops / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None
        exec_tf = executed / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None
        roof_tf = exec_tf
        pmc, traffic_src = stored_pmc(kname, args.config)
    else:
        # an FFT-form chain kernel group: its dsce_kernel_work flops (8 per complex
        # MAC, 5 n log2 n per DFT) over its time; traffic and counters from the
        # stamped per-kernel-group PMC summary of this build
        flops = kernels[kname]["flops_per_rep"] * B * args.steps
        achieved_tf = exec_tf = roof_tf = flops / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None
        kp = (pmc_all or {}).get(kname)
        pmc = {"sq_per_launch": kp.get("sq_per_launch"), "hbm_bytes_per_launch": kp.get("hbm_bytes_per_launch"),
               "avg_duration_ns_rocprof": kp.get("avg_duration_ns_rocprof")} if kp else None
        if pmc and kname == "ic_stages":
            # a concurrent group: its counters are the members' isolated counts
            # (the --pmc passes serialise dispatches), so the limiter describes
            # the members' mix; the profiler's wall span is the trace's
            pmc["avg_duration_ns_rocprof"] = None
        traffic_src = pmc_all_src
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    lim = derive_limiter(pmc, roof_tf, avg_ms)
    hbm_frac = traffic / (avg_ms * 1e-3) / (HBM_PEAK_GBS * 1e9) if traffic and avg_ms else None
    # the roof the kernel sits closer to: HBM (traffic from the stamped PMC pass)
    # or FP64 compute — the matrix cores alone for the contraction, the SIMD's
    # shared FP64 issue (f64 VALU and f64 MFMA do not overlap on gfx950) for the
    # chain kernels
    if hbm_frac is not None and roof_tf and hbm_frac > roof_tf / FP64_PEAK_TFLOPS:
        bound = "hbm"
    else:
        bound = "mfma" if contraction else "fp64 (VALU+MFMA shared)"
    paths = [sorted(p) for p in paths]
    work = {name: {"cmac_per_rep": eng.work_model(sid)[0],
                   "mmse_kernel": "k_mic_data" if "mic_stages" in paths[sid] else "k_wcontract"}
            for sid, name in enumerate(schemes)}
    ber = {}
    for sid, name in enumerate(schemes):
        bits = eng.bits_per_rep(sid)
        b = counts[sid, :, 0, :, :] / float(bits[0] * total_reps)
        ber[name] = {"snr_db_last": float(S.snr_db[-1]), "mmse_ic4": float(b[0, -1, -1]),
                     "perfect_ic4": float(b[1, -1, -1]), "mmse_onetap": float(b[0, -1, 0]),
                     "perfect_onetap": float(b[1, -1, 0])}

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return 0
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        try:
            cpu = run_cpu_baseline(args.cpu_seconds, args.config)
        except Exception:
            cpu = None
    L = S.L
    line = {
        "metric": METRIC if args.config == "c2" else
        "Monte-Carlo channel realisations/sec at %dsc (%s)" % (L, args.config.upper()),
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
        "config": {"workload": desc, "reps_per_step_per_gpu": B, "engine_batch": batch,
                   "parallelism": "dp%d" % world, "options": options},
        "roofline": {"bound": bound,
                     "kernel": KERNEL_DESC.get(kname, kname),
                     "kernel_group": kname,
                     "achieved": roof_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": (roof_tf / FP64_PEAK_TFLOPS) if roof_tf else None,
                     "achieved_basis": "executed matrix-core flops (3M: 6 per complex MAC)" if contraction else
                                       "algorithmic flops (dsce_kernel_work: 8 per complex MAC, 5 n log2 n per DFT)",
                     "achieved_algorithmic_8flop": achieved_tf, "achieved_executed": exec_tf,
                     "peak_measured": peak_meas,
                     "frac_measured": (roof_tf / peak_meas) if roof_tf and peak_meas else None,
                     # executed matrix-core flops / measured peak (the contraction), or the
                     # SQ_VALU_MFMA_BUSY_CYCLES share of this build's PMC pass (chain kernels)
                     "mfma_busy": ((exec_tf / peak_meas) if exec_tf and peak_meas else None) if contraction else
                     (lim or {}).get("mfma_busy"),
                     "valu_issue": (lim or {}).get("valu_issue"),
                     "hbm_frac": hbm_frac,
                     "traffic": traffic, "traffic_source": traffic_src, "source_hash": source_hash(),
                     "launches": launches, "avg_launch_ms": avg_ms,
                     "flops_per_launch": flops / launches if launches else None,
                     "work_model": ("support-aware: CMACs over W's off-diagonal (row, column) pairs (+ LK x NP for the "
                                    "fused diag(D_hat)); achieved / frac count the executed 6 flops per CMAC of the 3M "
                                    "form, achieved_algorithmic_8flop the 8-flop equivalent; mfma_busy = executed "
                                    "matrix-core flops / measured peak") if contraction else
                                   ("dsce_kernel_work('%s') x realisations per launch; DESIGN.md section 4.0" % kname),
                     "paths": paths,
                     "limiter": lim["limiter"] if lim else None,
                     "counters": lim,
                     # the next largest kernel group, for the record
                     "next_by_time": dominant_by_time({k: v for k, v in kernels.items() if k != kname and k not in members},
                                                      None),
                     "group_members": {m: kernels[m] for m in members if m in kernels} if kname == "ic_stages" else None,
                     "rocprof_span_ms": ((pmc_all or {}).get(kname, {}).get("span_ns_rocprof_trace") or 0) / 1e6 or None},
        "cpu_baseline": cpu,
        "allreduce": allreduce,
        "setup_s": setup_s,
        "kernels": kernels,
        "step_roofline": step_roof,
        "kernels_pmc_source": pmc_all_src,
        "work_per_scheme": work,
        "ber_last_snr": ber,
    }
    print(json.dumps(line))
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
