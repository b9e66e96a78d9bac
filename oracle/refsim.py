"""ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never by the product path).

CPU restatement (NumPy/SciPy fp64) of the reference's doubly-selective hot
path, written to follow the MATLAB line by line — including its explicit-matrix
formulation, which is also what makes it the CPU baseline:

* Jakes channel realisation          FastFading.m:222-238
* discrete-Doppler / time-invariant  FastFading.m:153-177, :203-221, :241-246
* doubly-flat loop (config 1)        SimpleVersion_DoublyFlat.m:89-170
* time-variant convolution matrix    FastFading.m:133-144, :186-190, :276-295
* R_vecH = E{vec(H) vec(H)^H}         FastFading.m:321-340, :366-407 (literal
  sparse build, including the tau>=2 wrap-around quirk of :377)
* R_hP / R_hP,est / R_Dij,hP / W     DoublySelectiveChannelEstimation.m:208-313
* Monte-Carlo body                   DoublySelectiveChannelEstimation.m:350-564
* detection                          SignalConstellation.m:76-101 (brute force,
  first minimum wins)

Randomness comes from ``oracle.philox`` (spec in include/dsce.h) instead of
MATLAB's global generator; draw shapes and order follow SURVEY.md appendix A3.

Pinning status: no MATLAB/Octave exists in this container, the reference has no
tests, fixtures or golden data for this path, so the
restatement is pinned only by (i) the Random123 Philox known-answer vectors,
(ii) the closed-form known answers of Theory/BitErrorProbabilityDoublyFlatRayleigh.m
(the reference's own commented 4-QAM formula, SimpleVersion_DoublyFlat.m:179),
(iii) the structural invariants stated in the reference's comments (Q'G = I,
real(D) = I for OQAM, PDP normalisation, Hermitian R_hP) and (iv) statistical
agreement with the published Figure 3/5 points.  Bit-level parity against
MATLAB itself is therefore "parity unpinned" (see DESIGN.md §Oracle).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from scipy.special import j0

from . import philox


def _col(x):
    return np.asarray(x).reshape(-1, order="F")


# ---------------------------------------------------------------------------
# channel
# ---------------------------------------------------------------------------
def jakes_ir(seed, rep, N, dt, pdp_norm, idx_taps, fD, paths, model="Jakes"):
    """ImpulseResponse (N x Ltap) of one realisation, FastFading.m:222-238."""
    nt = len(idx_taps)
    th = philox.uniforms(seed, rep, philox.STREAM_THETA, 0, nt * paths).reshape(nt, paths, order="F")
    ph = philox.uniforms(seed, rep, philox.STREAM_PHI, 0, nt * paths).reshape(nt, paths, order="F")
    if model == "Jakes":
        ds = np.cos(th * 2 * np.pi) * fD
    else:
        ds = 2 * (th - 0.5) * fD
    t = np.arange(N) * dt
    ir_tmp = np.zeros((len(pdp_norm), N), dtype=complex)
    for i, tap in enumerate(idx_taps):
        x = ph[i][:, None] + ds[i][:, None] * t[None, :]          # Paths x N
        ir_tmp[tap, :] = np.exp(1j * (2 * np.pi * x)).sum(axis=0) / np.sqrt(paths)
    return (np.sqrt(np.asarray(pdp_norm))[:, None] * ir_tmp).T


def static_ir(seed, rep, N, pdp_norm, idx_taps):
    """MaximumDopplerShift == 0 (FastFading.m:241-246): one impulse response
    1/sqrt(2) sqrt(PDPn) (randn + j randn) per realisation; returned repeated
    over the N samples as GetConvolutionMatrix uses it (:288-291)."""
    pdp_norm = np.asarray(pdp_norm, dtype=float)
    taps = np.asarray(idx_taps)
    re, im = philox.normal_pairs(seed, rep, philox.STREAM_THETA, 0, np.arange(taps.size))
    row = np.zeros(pdp_norm.size, dtype=complex)
    row[taps] = 1 / np.sqrt(2) * np.sqrt(pdp_norm[taps]) * (re + 1j * im)
    return np.repeat(row[None, :], N, axis=0)


def discrete_doppler_spectrum(N, SR, fD, model):
    """FastFading.m:158-177; returns (nd, S) with S over the bins f = -nd..nd,
    or (0, None) when fD/df <= 0.5 sets the velocity to zero (:153-156)."""
    df = SR / N
    if fD / df <= 0.5:
        return 0, None
    nd = int(np.ceil(fD / df))
    ip = df * (np.arange(-nd - 1, nd + 1) + 0.5)
    ip[ip <= -fD] = -fD
    ip[ip >= fD] = fD
    if model == "Discrete-Jakes":
        S = np.arcsin(ip[1:] / fD) - np.arcsin(ip[:-1] / fD)
    else:
        S = ip[1:] - ip[:-1]
    return nd, S / S.sum()


def discrete_ir(seed, rep, N, SR, pdp_norm, idx_taps, fD, model):
    """UseDiscreteDopplerSpectrum branch of NewRealization (FastFading.m:203-221),
    literally: ifft of [sqrt(S(nd+1:end)).*G1; zeros; sqrt(S(1:nd)).*G2] with
    G = N/sqrt(2) (randn + j randn) sqrt(PDPn)."""
    pdp_norm = np.asarray(pdp_norm, dtype=float)
    taps = np.asarray(idx_taps)
    nt = taps.size
    nd, S = discrete_doppler_spectrum(N, SR, fD, model)
    if S is None:
        return static_ir(seed, rep, N, pdp_norm, idx_taps)
    nb = 2 * nd + 1
    re, im = philox.normal_pairs(seed, rep, philox.STREAM_THETA, 1, np.arange(nb * nt))
    Z = (re + 1j * im).reshape(nb, nt, order="F")                 # row = f + nd
    g1 = N / np.sqrt(2) * Z[nd:, :]                                # f = 0..nd
    g2 = N / np.sqrt(2) * Z[:nd, :]                                # f = -nd..-1
    sp_ = np.sqrt(pdp_norm[taps])[None, :]
    g1 = g1 * sp_
    g2 = g2 * sp_
    Sm = np.repeat(S[:, None], nt, axis=1)
    X = np.concatenate([np.sqrt(Sm[nd:, :]) * g1, np.zeros((N - 2 * nd - 1, nt)), np.sqrt(Sm[:nd, :]) * g2])
    ir = np.zeros((N, pdp_norm.size), dtype=complex)
    ir[:, taps] = np.fft.ifft(X, axis=0)
    return ir


def conv_matrix(ir, pdp, N):
    """GetConvolutionMatrix{1} (FastFading.m:133-144, :186-190, :276-295)."""
    ltap = len(pdp)
    maps = []
    for i in range(1, ltap + 1):
        n = np.arange(i, N + 1)
        maps.append(np.stack([-i + 1 + n, n], axis=1))
    mapping = np.concatenate(maps)
    fast = mapping.copy()
    off = 0
    for i in range(1, ltap + 1):
        cnt = N - i + 1
        if pdp[i - 1] == 0:
            fast[off:off + cnt, :] = -1
        off += cnt
    fast = fast[fast[:, 0] != -1]
    cancel = np.ones((N, ltap), dtype=bool)                    # FastFading.m:186-189
    for i in range(1, ltap):
        cancel[i - 1, i:] = False                              # (end-Ltap+1+i):end, 1-based
    taps = np.flatnonzero(np.asarray(pdp))
    vals = _col(ir[:, taps])[_col(cancel[:, taps])]
    return sp.csc_matrix((vals, (fast[:, 1] - 1, fast[:, 0] - 1)), shape=(N, N))


def time_correlation(N, dt, fD, model="Jakes"):
    t = dt * np.arange(-(N - 1), N)
    if model == "Jakes":
        return j0(np.pi * 2 * fD * t)
    return np.sinc(2 * fD * t)


def correlation_matrix(N, pdp_norm, timecorr):
    """R_vecH, FastFading.m:366-407 (single-chunk branch, then cropped)."""
    ltap = len(pdp_norm)
    a = np.arange(N)
    itc = (N - 1) + a[:, None] - a[None, :]                   # 0-based IndexTimeCorrelation
    tcm = timecorr[itc]
    ordered = np.concatenate([p * tcm for p in pdp_norm], axis=0)   # (Ltap*N) x N
    icmc = (np.arange(0, N * N, N + 1))[:, None] + np.arange(ltap)[None, :]   # 0-based
    row = np.tile(_col(icmc), N)
    col = _col(np.kron(icmc.T, np.ones((N, 1), dtype=np.int64)))
    vals = _col(ordered)
    keep = (vals != 0) & (row < N * N) & (col < N * N)
    return sp.csr_matrix((vals[keep], (row[keep], col[keep])), shape=(N * N, N * N))


# ---------------------------------------------------------------------------
# correlation matrices and MMSE estimator (script:208-313)
# ---------------------------------------------------------------------------
def mmse_setup(R_vecH, N, G, Q, P, pilot_pos, kappa, pn_time, threshold=1e-8, want_W=True):
    """Returns R_hP, R_est (nsnr x NP x NP), R_noI, R_Dij (LK^2 x NP, thresholded),
    W, W0 (LK^2*NP x nsnr, thresholded)."""
    GP = G[:, pilot_pos]
    QP = Q[:, pilot_pos]
    NP = len(pilot_pos)
    LK = G.shape[1]
    Ms = []
    R_hP = np.empty((NP, NP), dtype=complex)
    for j in range(NP):
        v = _col(np.outer(QP[:, j], np.conj(GP[:, j])))       # kron(g.', q')' (script:213)
        M = (R_vecH @ v).reshape(N, N, order="F")
        Ms.append(M)
        R_hP[:, j] = np.sum((QP.conj().T @ M) * GP.T, axis=1)
    Gp = G @ P
    noN = R_hP.copy()
    for i in range(NP):                                        # script:222-234
        Temp = sp.kron(sp.eye(N), sp.csr_matrix(QP[:, i].conj()[None, :])) / np.sqrt(kappa)
        C = (Temp @ R_vecH @ Temp.conj().T).toarray()
        noN[i, i] = np.abs(np.sum((Gp.T @ C) * Gp.conj().T))
    nsnr = len(pn_time)
    R_est = np.repeat(noN[None], nsnr, axis=0)
    for s, pn in enumerate(pn_time):                           # script:241-249
        for i in range(NP):
            R_est[s, i, i] = noN[i, i] + pn * (QP[:, i].conj() @ QP[:, i]) / kappa
    R_noI = R_est - (noN - R_hP)[None]                         # script:251-253
    out = dict(R_hP=R_hP, R_est_noNoise=noN, R_est=R_est, R_noI=R_noI)
    R_Dij = np.empty((LK * LK, NP), dtype=complex)
    for i in range(NP):                                        # script:259-268
        t = _col(Q.conj().T @ Ms[i] @ G)
        t[np.abs(t) < threshold] = 0
        R_Dij[:, i] = t
    out["R_Dij"] = R_Dij
    if want_W:
        W = np.empty((LK * LK * NP, nsnr), dtype=complex)
        W0 = np.empty_like(W)
        for s in range(nsnr):                                  # script:282-313
            w = _col(R_Dij @ np.linalg.pinv(R_est[s]))
            w[np.abs(w) < threshold] = 0
            W[:, s] = w
            w0 = _col(R_Dij @ np.linalg.pinv(R_noI[s]))
            w0[np.abs(w0) < threshold] = 0
            W0[:, s] = w0
        out["W"] = W
        out["W0"] = W0
    return out


# ---------------------------------------------------------------------------
# detection (SignalConstellation.m:83-101)
# ---------------------------------------------------------------------------
def nearest(x, symbols):
    d = np.abs(_col(x)[:, None] - symbols[None, :])
    idx = np.argmin(d, axis=1)
    srt = np.sort(d, axis=1)
    margin = srt[:, 1] - srt[:, 0] if symbols.size > 1 else np.full(idx.shape, np.inf)
    return idx, margin


# ---------------------------------------------------------------------------
# Monte-Carlo loop (script:350-564)
# ---------------------------------------------------------------------------
def simulate(seed, first_rep, n_rep, chan, schemes, pn_time, n_iter, mmse, margin_eps=1e-9, trace=None,
             w_sparse=False):
    """Literal restatement of the Monte-Carlo body.

    ``chan``: dict(N, dt, pdp, pdp_norm, idx_taps, fD, paths, model).
    ``schemes``: list of dicts with G, Q, P, pilot_pos, data_pos, despread,
    real_detect, data_div, kappa, symbols (constellation, sorted), bits_per_symbol,
    considered (per data symbol), bits_slot, pilot_slot.
    ``mmse``: per scheme the dict from :func:`mmse_setup`.

    Returns dict(err=int64[ns, 2 csi, 2 edge, nsnr, 1+n_iter], borderline=int64[ns],
    nbits=int64[ns, 2 edge], mse_err=float[ns, nsnr, 1+n_iter], mse_pow=float[ns, nsnr]).
    The MSE sums (|h_hat - h|^2 per stage, |h|^2, h = diag(D)) are build-defined
    (the reference computes none): the checker of dsce_get_mse.

    ``w_sparse``: form D_hat = reshape(W hP) (script:417-425, :493-511) as a
    sparse (LK^2 x NP) product over W's stored non-zeros instead of the
    literal full(W) .* hP summed over the third dimension.  Same terms, same
    thresholded W; only the summation order over p differs (rounding level).
    Used for the C5 FBMC schemes, where full(W) is 1 GB per evaluation.
    """
    ns = len(schemes)
    nsnr = len(pn_time)
    N = chan["N"]
    err = np.zeros((ns, 2, 2, nsnr, 1 + n_iter), dtype=np.int64)
    mse_err = np.zeros((ns, nsnr, 1 + n_iter))
    mse_pow = np.zeros((ns, nsnr))
    border = np.zeros(ns, dtype=np.int64)
    nbits = np.zeros((ns, 2), dtype=np.int64)
    for si, sc in enumerate(schemes):
        m = sc["bits_per_symbol"]
        nbits[si, 0] = sc["n_data"] * m * n_rep
        nbits[si, 1] = int(np.sum(sc["considered"])) * m * n_rep
    wsp = {}
    if w_sparse:
        for si, sc in enumerate(schemes):
            LK, NP = sc["G"].shape[1], len(sc["pilot_pos"])
            for key in ("W", "W0"):
                for isnr in range(len(pn_time)):
                    wsp[si, key, isnr] = sp.csr_matrix(mmse[si][key][:, isnr].reshape(LK * LK, NP, order="F"))

    def d_hat(si, key, isnr, hp, LK, NP):
        if w_sparse:
            return (wsp[si, key, isnr] @ hp).reshape(LK, LK, order="F")
        return (mmse[si][key][:, isnr].reshape(LK, LK, NP, order="F") * hp[None, None, :]).sum(axis=2)

    for rep in range(first_rep, first_rep + n_rep):
        ir = jakes_ir(seed, rep, N, chan["dt"], chan["pdp_norm"], chan["idx_taps"], chan["fD"],
                      chan["paths"], chan.get("model", "Jakes"))
        H = conv_matrix(ir, chan["pdp"], N)
        if trace is not None:
            trace.setdefault("ir", []).append(ir)
        for si, sc in enumerate(schemes):
            G, Q, P = sc["G"], sc["Q"], sc["P"]
            symbols = sc["symbols"]
            bitmap = sc["bitmap"]
            M = symbols.size
            mbit = sc["bits_per_symbol"]
            nd = sc["n_data"]
            NP = len(sc["pilot_pos"])
            LK = G.shape[1]
            b = philox.bits(seed, rep, sc["bits_slot"], nd * mbit)               # script:355-357
            xD = symbols[(b.reshape(nd, mbit).astype(np.int64) << np.arange(mbit)).sum(axis=1)]
            pidx = philox.indices(seed, rep, sc["pilot_slot"], NP, M)            # script:365-368
            xP = symbols[pidx]
            xP = xP / np.abs(xP)
            x = P @ np.concatenate([xP, xD])                                     # script:371-373
            s = G @ x                                                            # script:376-378
            r0 = H @ s                                                           # script:383-385
            D = (Q.conj().T @ (H @ G))                                           # script:388-389
            h = np.diag(D).copy()
            cons_bits = np.repeat(sc["considered"], mbit)
            Dnd = D - np.diag(h)

            def detect(xhat):
                if sc["despread"]:
                    z = P.conj().T @ xhat
                    z = z[NP:]
                else:
                    z = xhat[sc["data_pos"]]
                if sc["real_detect"]:
                    z = np.real(z / sc["data_div"]) if not sc["despread"] else np.real(z) / sc["data_div"]
                else:
                    z = z / sc["data_div"]
                idx, margin = nearest(z, symbols)
                return z, idx, margin

            def count(idx, margin):
                det = bitmap[idx, :].reshape(-1)
                e = det != b
                border[si] += int(np.sum(margin < margin_eps))
                return int(e.sum()), int(e[cons_bits].sum())

            for isnr, pn in enumerate(pn_time):
                nre, nim = philox.complex_normals(seed, rep, isnr, N)             # script:399
                noise = np.sqrt(pn / 2) * (nre + 1j * nim)
                r = r0 + noise
                y = Q.conj().T @ r                                               # script:406-409
                hP = y[sc["pilot_pos"]] / xP / np.sqrt(sc["kappa"])              # script:412-414
                Dest = d_hat(si, "W", isnr, hP, LK, NP)
                hest = np.diag(Dest).copy()
                mse_err[si, isnr, 0] += np.sum(np.abs(hest - h) ** 2)
                mse_pow[si, isnr] += np.sum(np.abs(h) ** 2)
                # one-tap, estimated (script:428-447)
                _, idx, mg = detect(y / hest)
                e = count(idx, mg)
                err[si, 0, 0, isnr, 0] += e[0]
                err[si, 0, 1, isnr, 0] += e[1]
                zD_est = symbols[idx]
                # one-tap, perfect (script:450-466)
                _, idxp, mgp = detect(y / h)
                e = count(idxp, mgp)
                err[si, 1, 0, isnr, 0] += e[0]
                err[si, 1, 1, isnr, 0] += e[1]
                zD_perf = symbols[idxp]
                if trace is not None:
                    trace.setdefault("y", []).append(y)
                    trace.setdefault("hP0", []).append(hP)
                    trace.setdefault("hest0", []).append(hest)
                    trace.setdefault("hp_stages", []).append([hP])
                    trace.setdefault("hest_stages", []).append([hest])
                    # per (rep, SNR) unit, every stage: the quantities dsce_trace_unit_ex returns
                    unit = dict(rep=rep, snr=isnr, y=y, h=h, hp=[hP], hest=[hest], yest=[y], yperf=[y],
                                dec_e=[idx], dec_p=[idxp], margin_e=[mg], margin_p=[mgp])
                    trace.setdefault("units", []).append(unit)
                Dt = Dest
                ht = hest
                for it in range(1, n_iter + 1):
                    v = P @ np.concatenate([xP, zD_est])                           # script:482-484
                    yic = y - (Dt - np.diag(ht)) @ v
                    hPt = yic[sc["pilot_pos"]] / xP / np.sqrt(sc["kappa"])         # script:487-489
                    Dt = d_hat(si, "W" if it <= n_iter / 2 else "W0", isnr, hPt, LK, NP)   # script:492

                    ht = np.diag(Dt).copy()
                    mse_err[si, isnr, it] += np.sum(np.abs(ht - h) ** 2)
                    _, idx, mg = detect(yic / ht)                                  # script:519-537
                    e = count(idx, mg)
                    err[si, 0, 0, isnr, it] += e[0]
                    err[si, 0, 1, isnr, it] += e[1]
                    zD_est = symbols[idx]
                    vp = P @ np.concatenate([xP, zD_perf])                          # script:541-561
                    ypc = y - Dnd @ vp
                    _, idxp, mgp = detect(ypc / h)
                    e = count(idxp, mgp)
                    err[si, 1, 0, isnr, it] += e[0]
                    err[si, 1, 1, isnr, it] += e[1]
                    zD_perf = symbols[idxp]
                    if trace is not None:
                        trace.setdefault("yic", []).append(yic)
                        trace.setdefault("ypc", []).append(ypc)
                        trace["hp_stages"][-1].append(hPt)
                        trace["hest_stages"][-1].append(ht)
                        for key, val in (("hp", hPt), ("hest", ht), ("yest", yic), ("yperf", ypc), ("dec_e", idx),
                                         ("dec_p", idxp), ("margin_e", mg), ("margin_p", mgp)):
                            unit[key].append(val)
    return dict(err=err, borderline=border, nbits=nbits, mse_err=mse_err, mse_pow=mse_pow)


# ---------------------------------------------------------------------------
# SimpleVersion_DoublyFlat.m:89-170 (BASELINE config 1)
# ---------------------------------------------------------------------------
def snr_seed(seed, k):
    """Philox key of SNR point k of the doubly-flat loop: seed + k * 2^32."""
    return (int(seed) + (int(k) << 32)) & ((1 << 64) - 1)


def simulate_doubly_flat(seed, first_rep, n_rep, N, schemes, pn_time, margin_eps=1e-9):
    """Literal restatement of the doubly-flat Monte-Carlo loop.

    ``schemes``: oracle scheme dicts (see :func:`simulate`) plus ``noise_slot``
    and ``interp`` (the LK x NP PilotSymbolAidedChannelEstimation weights,
    ChannelInterpolation = interp @ LS, PSACE.m:115-121).  Every random
    quantity is drawn per (realisation, SNR point) with key snr_seed(seed, k)
    (:90-126).  Returns dict(err=int64[ns, 2 csi, nsnr], borderline=int64[ns]).
    """
    ns = len(schemes)
    err = np.zeros((ns, 2, len(pn_time)), dtype=np.int64)
    border = np.zeros(ns, dtype=np.int64)
    for rep in range(first_rep, first_rep + n_rep):
        for k, pn in enumerate(pn_time):
            sk = snr_seed(seed, k)
            h = static_ir(sk, rep, N, [1.0], [0])[0, 0]                     # :123
            noise = {}
            for si, sc in enumerate(schemes):
                P, G, Q = sc["P"], sc["G"], sc["Q"]
                symbols, bitmap = sc["symbols"], sc["bitmap"]
                M = symbols.size
                mbit = sc["bits_per_symbol"]
                nd = sc["n_data"]
                NP = len(sc["pilot_pos"])
                b = philox.bits(sk, rep, sc["bits_slot"], nd * mbit)          # :95-97
                xD = symbols[(b.reshape(nd, mbit).astype(np.int64) << np.arange(mbit)).sum(axis=1)]   # :100-102
                xP = symbols[philox.indices(sk, rep, sc["pilot_slot"], NP, M)]   # :105-108
                xP = xP / np.abs(xP)
                x = P @ np.concatenate([xP, xD])                               # :111-115
                s = G @ x                                                      # :118-120
                slot = sc["noise_slot"]
                if slot not in noise:                                          # :125-126
                    nre, nim = philox.complex_normals(sk, rep, 256 * slot, N)
                    noise[slot] = np.sqrt(pn / 2) * (nre + 1j * nim)
                r = h * s + noise[slot]                                        # :128-130
                y = Q.conj().T @ r                                             # :133-135
                LS = y[sc["pilot_pos"]] / xP / np.sqrt(sc["kappa"])            # :138-140
                hest = sc["interp"] @ LS                                       # :143-145
                for csi, hh in ((0, hest), (1, h)):                            # :148-161
                    xhat = y / hh
                    if sc["despread"]:
                        z = np.real(P[:, NP:].conj().T @ xhat) / sc["data_div"]
                    elif sc["real_detect"]:
                        z = np.real(xhat[sc["data_pos"]] / sc["data_div"])
                    else:
                        z = xhat[sc["data_pos"]] / sc["data_div"]
                    idx, margin = nearest(z, symbols)
                    det = bitmap[idx, :].reshape(-1)
                    err[si, csi, k] += int(np.sum(det != b))                   # :164-169
                    border[si] += int(np.sum(margin < margin_eps))
    return dict(err=err, borderline=border)


# ---------------------------------------------------------------------------
# Theory/BitErrorProbabilityDoublyFlatRayleigh.m:10-130
# ---------------------------------------------------------------------------
def _gauss_ratio_cdf(Ey2, Eh2, Eyh, zR, zI):
    a = Eyh / Eh2
    b = Ey2 / Eh2
    zR = np.asarray(zR, dtype=float)
    zI = np.asarray(zI, dtype=float)
    out = np.full(zR.shape, np.nan)
    i0 = (zR == -np.inf) | (zI == -np.inf)
    i1 = (zR == np.inf) & (zI == np.inf)
    ir = (zI == np.inf) & np.isfinite(zR)
    ii = (zR == np.inf) & np.isfinite(zI)
    inn = np.isfinite(zR) & np.isfinite(zI)
    out[i0] = 0
    out[i1] = 1
    out[ir] = 0.5 - (a.real - zR[ir]) / (2 * np.sqrt((a.real - zR[ir]) ** 2 + b - abs(a) ** 2))
    out[ii] = 0.5 - (a.imag - zI[ii]) / (2 * np.sqrt((a.imag - zI[ii]) ** 2 + b - abs(a) ** 2))
    r, q = zR[inn], zI[inn]
    out[inn] = (0.25 + (r - a.real) * (2 * np.arctan((q - a.imag) / np.sqrt((r - a.real) ** 2 + b - abs(a) ** 2))
                                       + np.pi) / (4 * np.pi * np.sqrt((r - a.real) ** 2 + b - abs(a) ** 2))
                + (q - a.imag) * (2 * np.arctan((r - a.real) / np.sqrt((q - a.imag) ** 2 + b - abs(a) ** 2))
                                  + np.pi) / (4 * np.pi * np.sqrt((q - a.imag) ** 2 + b - abs(a) ** 2)))
    return out


def bit_error_probability_doubly_flat_rayleigh(snr_db, symbols, bitmap):
    symbols = np.asarray(symbols, dtype=complex)
    bitmap = np.asarray(bitmap, dtype=np.int64)
    half = np.min(np.abs(symbols.real))
    dr = np.stack([symbols.real - half, symbols.real + half, symbols.imag - half, symbols.imag + half], axis=1)
    dr[symbols.real == symbols.real.min(), 0] = -np.inf
    dr[symbols.real == symbols.real.max(), 1] = np.inf
    dr[symbols.imag == symbols.imag.min(), 2] = -np.inf
    dr[symbols.imag == symbols.imag.max(), 3] = np.inf
    out = np.empty(len(snr_db))
    for k, snr in enumerate(np.atleast_1d(snr_db)):
        pn = 10 ** (-snr / 10)
        PM = np.empty((symbols.size, symbols.size))
        for i, x in enumerate(symbols):
            Ey2 = abs(x) ** 2 + pn
            cdf = lambda zr, zi: _gauss_ratio_cdf(Ey2, 1.0, x, zr, zi)
            PM[:, i] = cdf(dr[:, 1], dr[:, 3]) + cdf(dr[:, 0], dr[:, 2]) - cdf(dr[:, 0], dr[:, 3]) - cdf(dr[:, 1], dr[:, 2])
        ep = np.empty((2, bitmap.shape[1]))
        for ib in range(bitmap.shape[1]):
            for v in (0, 1):
                ix = bitmap[:, ib] == v
                ep[v, ib] = np.mean(np.sum(PM[np.ix_(~ix, ix)], axis=0))
        out[k] = np.mean(ep)
    return out
