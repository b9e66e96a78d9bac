"""Results I/O and figures (replaces the plotting block of
DoublySelectiveChannelEstimation.m:570-631).

The engine returns int64 error counts [scheme][csi][edge][snr][stage]
(include/dsce.h).  The reference stores one BER per (SNR, realisation[, IC
step]) and plots `nanmean` over realisations (script:577-631); every
realisation carries the same number of bits, so that mean equals total
errors / total bits, which is what `ber()` returns.

File format (JSON, one object): configuration, SNR grid, per-scheme bit counts,
realisation count, the raw counters and the BER arrays (plus, with
`simulate --mse`, "nmse": [scheme][snr][stage] channel-estimation NMSE, a
build-defined output the reference does not compute); `save(..., npz=True)`
also writes the arrays to a sibling .npz.  `figures()` draws Figures 2-5 with
the script's curve set, colours and markers (matplotlib, optional).
"""
from __future__ import annotations

import json

import numpy as np

CSI = ("mmse", "perfect")
EDGE = ("all", "no_edge")
# script:572-631: which scheme each figure shows
FIGURES = {2: ("ofdm", "OFDM"), 3: ("fbmc_aux", "FBMC Auxiliary Symbols"), 4: ("fbmc_cod", "FBMC Data Spreading")}


def ber(counts, bits, n_rep):
    """BER [scheme][csi][edge][snr][stage] from counters and bits per
    realisation ([scheme][2]: all bits, no-edge bits)."""
    counts = np.asarray(counts, dtype=np.float64)
    bits = np.asarray(bits, dtype=np.float64).reshape(counts.shape[0], 1, 2, 1, 1)
    with np.errstate(invalid="ignore", divide="ignore"):
        return counts / (bits * float(n_rep))


def make(setup, scheme_names, counts, bits, n_rep, seed, extra=None):
    """Result object of one Monte-Carlo run."""
    b = ber(counts, bits, n_rep)
    res = {
        "config": setup.name,
        "N": int(setup.N),
        "snr_db": [float(x) for x in setup.snr_db],
        "n_iter": int(setup.n_iter),
        "plot_snr_db": float(setup.plot_snr_db),
        "n_repetitions": int(n_rep),
        "seed": int(seed),
        "schemes": list(scheme_names),
        "bits_per_rep": {s: [int(x) for x in bits[i]] for i, s in enumerate(scheme_names)},
        "counts": np.asarray(counts, dtype=np.int64).tolist(),
        "ber": {s: {c: {e: b[i, ci, ei].tolist() for ei, e in enumerate(EDGE)} for ci, c in enumerate(CSI)}
                for i, s in enumerate(scheme_names)},
    }
    if extra:
        res.update(extra)
    return res


def save(path, result, npz=False):
    with open(path, "w") as f:
        json.dump(result, f, indent=1)
    if npz:
        base = path[:-5] if path.endswith(".json") else path
        np.savez(base + ".npz", counts=np.asarray(result["counts"], dtype=np.int64),
                 snr_db=np.asarray(result["snr_db"]), n_repetitions=result["n_repetitions"])


def load(path):
    with open(path) as f:
        res = json.load(f)
    res["counts"] = np.asarray(res["counts"], dtype=np.int64)
    return res


def curve(result, scheme, csi, edge, stage=None):
    """BER vs SNR of one curve (stage None = last IC iteration)."""
    a = np.asarray(result["ber"][scheme][csi][edge])
    return a[:, -1 if stage is None else stage]


def figures(result, outdir, theory=None, fmt="png"):
    """Figures 2-5 of the script (one-tap / IC, MMSE / perfect CSI, with and
    without edges).  theory: optional (snr_db, ber) doubly-flat lower bound,
    drawn in grey like script:575.  Returns the written file names."""
    import os

    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    snr = np.asarray(result["snr_db"])
    out = []
    style = [  # (label, csi, edge, stage, fmt, colour) in the script's legend order
        ("Cancellation (Perfect CSI)", "perfect", "all", None, "-x", "black"),
        ("Cancellation", "mmse", "all", None, "-s", "magenta"),
        ("Cancellation (no Edges)", "mmse", "no_edge", None, "-o", "blue"),
        ("One-Tap (Perfect CSI)", "perfect", "all", 0, "-x", (0.7, 0.7, 0.0)),
        ("One-Tap", "mmse", "all", 0, "-s", "red"),
    ]
    for fig, (scheme, title) in FIGURES.items():
        if scheme not in result["ber"]:
            continue
        plt.figure(figsize=(5, 4))
        if theory is not None:
            plt.semilogy(theory[0], theory[1], color=(0.75, 0.75, 0.75), label="Doubly-Flat Theory")
        for label, csi, edge, stage, f, col in style:
            plt.semilogy(snr, curve(result, scheme, csi, edge, stage), f, color=col, markersize=4, label=label)
        plt.ylim(1e-2, 0.5)
        plt.title("%s, %d realisations" % (title, result["n_repetitions"]))
        plt.xlabel("Signal-to-Noise Ratio [dB]")
        plt.ylabel("Bit Error Ratio")
        plt.legend(fontsize=7)
        name = os.path.join(outdir, "Figure%d.%s" % (fig, fmt))
        plt.savefig(name, dpi=120, bbox_inches="tight")
        plt.close()
        out.append(name)
    if "fbmc_aux" in result["ber"]:                     # Figure 5: BER over the IC steps (script:609-631)
        k = list(snr).index(result["plot_snr_db"]) if result["plot_snr_db"] in list(snr) else len(snr) - 1
        it = np.arange(result["n_iter"] + 1)
        plt.figure(figsize=(5, 4))
        for label, csi, edge, stage, f, col in style:
            a = np.asarray(result["ber"]["fbmc_aux"][csi][edge])[k]
            y = np.full(it.shape, a[0]) if stage == 0 else a
            plt.semilogy(it, y, f, color=col, markersize=4, label=label)
        plt.xticks(it)
        plt.title("FBMC Auxiliary Symbols, %g dB" % snr[k])
        plt.xlabel("Iteration Step i")
        plt.ylabel("Bit Error Ratio")
        plt.legend(fontsize=7)
        name = os.path.join(outdir, "Figure5.%s" % fmt)
        plt.savefig(name, dpi=120, bbox_inches="tight")
        plt.close()
        out.append(name)
    return out


def doubly_flat_result(sim, counts, n_rep, seed, theory, extra=None):
    """Result object of the doubly-flat script (SimpleVersion_DoublyFlat.m):
    its five BER curves (mean over realisations, :186-191) and the closed-form
    perfect-CSI BEP it plots (:180-181, ``theory`` on a 0.5 dB grid)."""
    S = sim.setup
    res = {
        "config": "doubly_flat",
        "N": int(S.N),
        "snr_db": [float(x) for x in S.snr_db],
        "n_repetitions": int(n_rep),
        "seed": int(seed),
        "bits_per_rep": [int(x) for x in sim.bits_per_rep()],
        "counts": np.asarray(counts, dtype=np.int64).tolist(),
        "ber": {k: [float(x) for x in v] for k, v in sim.ber(counts, n_rep).items()},
        "theory": {"snr_db": [float(x) for x in theory[0]], "bep": [float(x) for x in theory[1]]},
    }
    if extra:
        res.update(extra)
    return res


def doubly_flat_figure(result, path):
    """The BER/BEP figure of SimpleVersion_DoublyFlat.m:185-195."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    snr = np.asarray(result["snr_db"])
    plt.figure(figsize=(5, 4))
    for label, f, col in (("FBMC Auxiliary", "-o", "red"), ("FBMC Coding", "-o", "blue"), ("OFDM", "-o", "black"),
                          ("FBMC perfect CSI", "-x", "blue"), ("OFDM perfect CSI", "-x", "black")):
        plt.semilogy(snr, result["ber"][label], f, color=col, markersize=4, label="Simulation: " + label)
    plt.semilogy(result["theory"]["snr_db"], result["theory"]["bep"], color="black", label="Theory perfect CSI")
    plt.xlabel("SNR for OFDM (dB)")
    plt.ylabel("BER, BEP")
    plt.title("Doubly-flat, %d realisations" % result["n_repetitions"])
    plt.legend(fontsize=7, loc="lower left")
    plt.savefig(path, dpi=120, bbox_inches="tight")
    plt.close()
    return path
