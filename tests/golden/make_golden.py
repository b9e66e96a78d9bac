#!/usr/bin/env python3
"""Generates the committed golden fixtures of tests/golden/.

* philox_kat.json       — Random123 known-answer vectors of Philox4x32-10
                          (published with Random123's kat_vectors; copied as data).
* theory_4qam.json      — the reference's own closed form of the 4-QAM doubly-flat
                          Rayleigh BEP, SimpleVersion_DoublyFlat.m:179:
                          BEP = 1/2 - 1/(2 sqrt(2 (1 + 10^(-SNR/10)) - 1)).
* oracle_c2_small.json  — regression vectors of the CPU oracle (this repo's
                          restatement, NOT reference output): C2 OFDM, seed
                          0x5EED0002, realisations 0..1, all 7 SNR points —
                          IR samples, R_hP diagonal, error counts.
* setup_<config>.json   — the oracle's setup restatement (oracle/setup.py) of
                          C2-C4 ('default') and C5: per scheme checksums and
                          sampled entries of G, Q, P, the pilot / data positions,
                          no-edge masks, kappa, DPR, SIR.
* oracle_<cN>_small.json — C3 / C4 (FBMC aux / coding, SNR 15 and 35 dB) and C5
                          (OFDM 48 x 14, SNR 20 and 36 dB): 8 realisations of
                          IR samples and D = Q'HG checksums, R_hP, a W slice
                          (sampled entries + non-zero count per SNR and
                          variant) and the int64 error counts of realisations
                          0..1.

Parity of the GPU engine is checked against the live oracle; these files pin
the oracle (and its setup restatement) against silent drift.
usage: python tests/golden/make_golden.py [--only c3,c4,c5,setup,c2,kat]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "channel-estimation_amd"), os.path.join(ROOT, "tests")]

SEED = 0x5EED0002
CFG = {"c3": ("default", "fbmc_aux", [15.0, 35.0]), "c4": ("default", "fbmc_cod", [15.0, 35.0]),
       "c5": ("c5", "ofdm", [20.0, 36.0])}
SAMPLE_ROWS = (0, 1, 100, 333)


def cx(z):
    z = np.asarray(z, dtype=complex)
    return [[float(v.real), float(v.imag)] for v in z.reshape(-1)]


def checksum(A):
    """(sum, sum |.|^2, sum of row-index-weighted entries) — order-sensitive."""
    A = np.asarray(A, dtype=complex)
    w = np.arange(1, A.shape[0] + 1, dtype=float)[:, None] if A.ndim == 2 else np.arange(1, A.size + 1)
    return [cx(A.sum())[0], float(np.sum(np.abs(A) ** 2)), cx((w * A).sum())[0]]


def sample(A, k=12, seed=7):
    A = np.asarray(A)
    rng = np.random.default_rng(seed)
    nz = np.argwhere(np.abs(A) > 0)
    pick = nz[rng.choice(len(nz), size=min(k, len(nz)), replace=False)]
    return [[int(i) for i in p] + cx(A[tuple(p)])[0] for p in pick]


def setup_fixture(name, schemes):
    import harness
    S = harness.setup(name, schemes=schemes)
    out = {"config": name, "N": S.N, "L": S.L, "pdp_norm": [float(x) for x in S.chan["pdp_norm"]],
           "idx_taps": [int(x) for x in S.chan["idx_taps"]], "schemes": {}}
    for k, sc in S.schemes.items():
        d = {f: checksum(sc[f]) for f in ("G", "Q", "P")}
        d.update({f + "_samples": sample(sc[f]) for f in ("G", "Q", "P")})
        d.update(pilot_pos=[int(x) for x in sc["pilot_pos"]], data_pos=[int(x) for x in sc["data_pos"]],
                 considered=[int(x) for x in sc["considered"]], kappa=sc["kappa"], data_div=sc["data_div"],
                 n_data=int(sc["n_data"]))
        if "iic" in sc:
            d.update(DPR=sc["iic"]["DPR"], SIR_dB=[float(x) for x in sc["iic"]["SIR_dB"]])
        out["schemes"][k] = d
    return out


def oracle_fixture(tag):
    import harness
    from oracle import refsim
    name, key, snr = CFG[tag]
    S = harness.setup(name, schemes=(key,), snr_db=snr)
    sc = S.schemes[key]
    ch = S.chan
    mm = harness.oracle_mmse(S, key)
    reps = []
    for rep in range(8):
        ir = refsim.jakes_ir(SEED, rep, S.N, ch["dt"], ch["pdp_norm"], ch["idx_taps"], ch["fD"], ch["paths"])
        H = refsim.conv_matrix(ir, ch["pdp"], S.N)
        D = sc["Q"].conj().T @ (H @ sc["G"])
        reps.append({"rep": rep, "ir": {str(n): cx(ir[n, ch["idx_taps"]]) for n in (0, 1, 100, S.N - 1)},
                     "D": checksum(D), "D_diag": cx(np.diag(D)[list(SAMPLE_ROWS)])})
    LK = sc["G"].shape[1]
    W = {}
    for var in ("W", "W0"):
        for k in range(len(snr)):
            w = mm[var][:, k]
            W["%s_%d" % (var, k)] = {"nnz": int(np.count_nonzero(w)), "checksum": checksum(w),
                                     "samples": sample(w.reshape(-1), k=16, seed=k)}
    res = harness.simulate(S, SEED, 0, 2, [key])
    return {"config": tag, "scheme": key, "seed": SEED, "snr_db": snr, "LK": LK, "reps": reps,
            "R_hP": cx(mm["R_hP"]), "R_est_diag": [cx(np.diag(r)) for r in mm["R_est"]], "W": W,
            "err_reps_0_2": res["err"].tolist(), "nbits": res["nbits"].tolist()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="kat,c2,setup,c3,c4,c5")
    only = set(ap.parse_args().only.split(","))
    if "kat" in only:
        kat = [
            {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
            {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2,
             "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
            {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
             "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
        ]
        json.dump(kat, open(os.path.join(HERE, "philox_kat.json"), "w"), indent=1)
        snr = list(range(0, 41, 5))
        bep = [0.5 - 1.0 / (2.0 * np.sqrt(2.0 * (1.0 + 10.0 ** (-s / 10.0)) - 1.0)) for s in snr]
        json.dump({"snr_db": snr, "bep": bep, "source": "SimpleVersion_DoublyFlat.m:179"},
                  open(os.path.join(HERE, "theory_4qam.json"), "w"), indent=1)
    if "c2" in only:
        import harness
        S = harness.setup("default", schemes=("ofdm",))
        mm = harness.oracle_mmse(S, "ofdm")
        tr = {}
        res = harness.simulate(S, SEED, 0, 2, ["ofdm"], trace=tr)
        ir = tr["ir"][0]
        out = {"seed": SEED, "reps": [0, 2], "config": "C2 ofdm",
               "ir_rep0_samples": {str(n): [ir[n, 0].real, ir[n, 0].imag, ir[n, 1].real, ir[n, 1].imag]
                                   for n in (0, 1, 100, 539)},
               "rhp_diag": [[z.real, z.imag] for z in np.diag(mm["R_hP"])],
               "err": res["err"].tolist(), "nbits": res["nbits"].tolist()}
        json.dump(out, open(os.path.join(HERE, "oracle_c2_small.json"), "w"))
    if "setup" in only:
        json.dump(setup_fixture("default", ("fbmc_aux", "fbmc_cod", "ofdm")),
                  open(os.path.join(HERE, "setup_default.json"), "w"))
        json.dump(setup_fixture("c5", ("fbmc_aux", "fbmc_cod", "ofdm")), open(os.path.join(HERE, "setup_c5.json"), "w"))
    for tag in ("c3", "c4", "c5"):
        if tag in only:
            json.dump(oracle_fixture(tag), open(os.path.join(HERE, "oracle_%s_small.json" % tag), "w"))
            print(tag, "written", flush=True)
    print("golden fixtures written")


if __name__ == "__main__":
    main()
