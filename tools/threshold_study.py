#!/usr/bin/env python3
"""CPU study of the reference's two 1e-8 sparsifications (R_Dij,hP at
script:263-264, W / W0 at script:287-289 / :306-308) against the unthresholded
estimator W_s = R_Dij,hP pinv(R), which is what a structured form
D_hat = Q' H_hat G computes.

For a scheme it reports, per (variant, SNR) slice:
* the structural support of W (pairs (r, c) where Q' M_p G is not identically
  zero for some pilot p: the time overlap of Q's row and G's column through the
  channel taps), and the band the product keeps after the threshold (the pairs
  with a non-zero thresholded entry);
* how many entries the thresholds change (W_thr != W_s beyond rounding), split
  into entries zeroed by the W threshold (|W_s| < thr) and entries moved by the
  R_Dij threshold propagating through pinv(R), and their share of the kept band;
* the largest |W_thr - W_s| relative to max |W|, and the magnitude histogram of
  W_s inside the support (which ZeroThreshold values drop non-rounding entries).

Uses oracle/ (test infrastructure) as the model of the reference: this is a
study tool, not part of the product.  Output: one JSON object on stdout.

  python tools/threshold_study.py --config default --scheme ofdm
  python tools/threshold_study.py --config default --scheme fbmc_aux --snr 0 6
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "channel-estimation_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="default")
    ap.add_argument("--scheme", default="ofdm")
    ap.add_argument("--snr", type=int, nargs="*", default=None, help="SNR indices (default: all)")
    ap.add_argument("--threshold", type=float, default=None)
    args = ap.parse_args()

    import harness
    from oracle import refsim

    S = harness.setup(args.config, schemes=(args.scheme,))
    thr = S.zero_threshold if args.threshold is None else args.threshold
    sc = S.schemes[args.scheme]
    ch = S.chan
    tc = refsim.time_correlation(S.N, ch["dt"], ch["fD"], ch["model"])
    R_vecH = refsim.correlation_matrix(S.N, ch["pdp_norm"], tc)
    G, Q, P = sc["G"], sc["Q"], sc["P"]
    LK = G.shape[1]
    NP = len(sc["pilot_pos"])
    # unthresholded R_Dij (threshold 0) and the script's
    base = refsim.mmse_setup(R_vecH, S.N, G, Q, P, sc["pilot_pos"], sc["kappa"], S.pn_time, 0.0, want_W=False)
    Rd0 = base["R_Dij"]
    Rdt = Rd0.copy()
    Rdt[np.abs(Rdt) < thr] = 0
    # structural support: Q row r and G column c overlap in time through the taps
    taps = np.flatnonzero(np.asarray(ch["pdp_norm"]) > 0)
    qs = np.abs(Q) > 0
    gs = np.abs(G) > 0
    gsh = np.zeros_like(gs)
    for d in taps:
        gsh[d:] |= gs[:S.N - d]
    struct = (qs.T.astype(np.int32) @ gsh.astype(np.int32)) > 0          # [r, c]
    struct_flat = struct.reshape(-1, order="F")                            # index r + LK c
    hist_edges = [0, 1e-14, 1e-12, 1e-10, 1e-9, 1e-8, 1e-7, 1e-6, 1e-5, 1e-4, 1e-2, np.inf]
    out = {"config": args.config, "scheme": args.scheme, "threshold": thr, "LK": LK, "NP": NP,
           "struct_pairs": int(struct.sum()), "pairs_total": LK * LK,
           "rdij_entries_zeroed_in_support": int(((np.abs(Rd0) < thr) & (Rd0 != 0)).sum()),
           "rdij_entries_support": int((Rd0 != 0).sum()), "slices": []}
    snrs = range(len(S.pn_time)) if args.snr is None else args.snr
    for s in snrs:
        for var, R in (("W", base["R_est"][s]), ("W0", base["R_noI"][s])):
            Pi = np.linalg.pinv(R)
            Ws = (Rd0 @ Pi)                                # LK^2 x NP
            Wt = Rdt @ Pi
            Wt[np.abs(Wt) < thr] = 0
            mx = np.abs(Ws).max()
            kept = (np.abs(Wt) > 0).any(axis=1)            # pairs with any non-zero thresholded entry
            d = np.abs(Wt - Ws)
            rnd = 1e-12 * mx
            changed = d > rnd
            by_w = changed & (Wt == 0)                     # zeroed by the W threshold
            by_r = changed & (Wt != 0)                     # moved by the propagated R_Dij threshold
            ch_pairs = changed.any(axis=1)
            mag = np.abs(Ws[struct_flat]).ravel()
            h = np.histogram(mag, bins=hist_edges)[0]
            out["slices"].append({
                "snr_index": int(s), "snr_db": float(S.snr_db[s]), "variant": var, "cond_R": float(np.linalg.cond(R)),
                "max_abs_W": float(mx),
                "kept_pairs": int(kept.sum()), "kept_over_struct": float(kept.sum() / max(struct.sum(), 1)),
                "changed_entries": int(changed.sum()), "changed_by_W_threshold": int(by_w.sum()),
                "changed_by_Rdij_threshold": int(by_r.sum()),
                "changed_pairs": int(ch_pairs.sum()),
                "changed_pairs_inside_kept": int((ch_pairs & kept).sum()),
                "changed_pairs_over_kept": float((ch_pairs & kept).sum() / max(kept.sum(), 1)),
                "changed_pairs_outside_kept_in_struct": int((ch_pairs & ~kept & struct_flat).sum()),
                "max_dev_rel": float(d.max() / mx), "max_dev_abs": float(d.max()),
                "max_dev_abs_inside_kept": float(d[kept].max()) if kept.any() else 0.0,
                "hist_edges": [str(e) for e in hist_edges], "hist_abs_Ws_in_struct": [int(x) for x in h]})
            print("snr %d %s: kept %d / struct %d pairs, changed pairs %d (inside kept %d = %.3f), "
                  "max dev %.3g abs (%.3g rel)" % (s, var, kept.sum(), struct.sum(), ch_pairs.sum(),
                                                   (ch_pairs & kept).sum(), (ch_pairs & kept).sum() / max(kept.sum(), 1),
                                                   d.max(), d.max() / mx), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
