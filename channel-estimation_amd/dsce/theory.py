"""``Theory/BitErrorProbabilityDoublyFlatRayleigh.m`` (:10-130): closed-form
bit-error probability of a rectangular-grid constellation over a doubly-flat
Rayleigh channel with perfect CSI (Nissel & Rupp, IEEE Comm. Letters 2017).

Host-side, part of the reference's API surface (the curve
SimpleVersion_DoublyFlat.m:180-181 and DoublySelectiveChannelEstimation.m:575
plot).  Vectorised over SNR points, transmitted symbols and decision regions
at once; the test suite checks it against the oracle's literal restatement.
"""
from __future__ import annotations

import numpy as np


def gaussian_ratio_cdf(a, b, zR, zI):
    """Pr(Re(y/h) < zR, Im(y/h) < zI) for complex Gaussians with
    alpha = E{y h*}/E{|h|^2} = a and beta = E{|y|^2}/E{|h|^2} = b (:85-130);
    zR / zI may be +-inf.  Broadcasts over all arguments."""
    a, b, zR, zI = np.broadcast_arrays(np.asarray(a, dtype=complex), np.asarray(b, dtype=float),
                                       np.asarray(zR, dtype=float), np.asarray(zI, dtype=float))
    v = b - np.abs(a) ** 2
    dr = zR - a.real
    di = zI - a.imag
    with np.errstate(invalid="ignore", divide="ignore"):
        sr = np.sqrt(dr ** 2 + v)
        si = np.sqrt(di ** 2 + v)
        normal = 0.25 + dr * (2 * np.arctan(di / sr) + np.pi) / (4 * np.pi * sr) \
            + di * (2 * np.arctan(dr / si) + np.pi) / (4 * np.pi * si)
        real_only = 0.5 + dr / (2 * sr)                 # zI = +inf (:105-107)
        imag_only = 0.5 + di / (2 * si)                 # zR = +inf (:109-111)
    out = np.where(np.isfinite(zR) & np.isfinite(zI), normal, np.nan)
    out = np.where(np.isfinite(zR) & (zI == np.inf), real_only, out)
    out = np.where(np.isfinite(zI) & (zR == np.inf), imag_only, out)
    out = np.where((zR == np.inf) & (zI == np.inf), 1.0, out)
    out = np.where((zR == -np.inf) | (zI == -np.inf), 0.0, out)
    return out


def bit_error_probability_doubly_flat_rayleigh(snr_db, symbol_mapping, bit_mapping):
    """BitErrorProbabilityDoublyFlatRayleigh(SNR_dB, SymbolMapping, BitMapping):
    one value per SNR point (the SNR of the complex domain; for FBMC-OQAM use
    SNR_OFDM - 3 dB, :11)."""
    x = np.asarray(symbol_mapping, dtype=complex).reshape(-1)
    bm = np.asarray(bit_mapping).reshape(x.size, -1).astype(bool)
    half = np.min(np.abs(x.real))                                           # :19-31
    lo_r = np.where(x.real == x.real.min(), -np.inf, x.real - half)
    hi_r = np.where(x.real == x.real.max(), np.inf, x.real + half)
    lo_i = np.where(x.imag == x.imag.min(), -np.inf, x.imag - half)
    hi_i = np.where(x.imag == x.imag.max(), np.inf, x.imag + half)
    pn = 10.0 ** (-np.atleast_1d(np.asarray(snr_db, dtype=float)) / 10)
    # [snr, region m, sent symbol i]: Pr(y/h in region m | x_i), :39-45, :64-74
    a = x[None, None, :]
    b = (np.abs(x) ** 2)[None, None, :] + pn[:, None, None]
    R = lambda zr, zi: gaussian_ratio_cdf(a, b, zr[None, :, None], zi[None, :, None])
    Pm = R(hi_r, hi_i) + R(lo_r, lo_i) - R(lo_r, hi_i) - R(hi_r, lo_i)
    # per bit and sent value: mean over sent symbols of the mass of the wrong regions (:46-52)
    ep = []
    for k in range(bm.shape[1]):
        for v in (False, True):
            sent = bm[:, k] == v
            ep.append(Pm[:, ~sent, :][:, :, sent].sum(axis=1).mean(axis=1))
    return np.mean(np.stack(ep, axis=1), axis=1)
