"""CPU: the structure behind the low-rank MMSE IC tap operator (DESIGN.md
§2.0c, build_mic_lr in dsce_api.hip), checked on the ORACLE's own C2 OFDM
operators (oracle/setup.py) — independent of the GPU fit it justifies.

The estimated taps of the structured MMSE IC are hhat[q][n] = sum_p Bv[q][n][p]
hP_p with Bv = m pinv(R) and m = the J0-Toeplitz coefficients of the pilot
columns (script:213 / :260 restricted to the convolution matrix's band).  For
OFDM, Q[b + d_q, j] conj(G[b, j]) is constant over pilot j's FFT window, so
m[j][q][n - d_q] = kappa_qj T_k(j)[n] with T_k the J0 kernel summed over pilot
symbol k's window: Bv = T Bz with only 4 real columns T_k.  The engine fits Bz
to its GPU-built Bv and requires the fit to reproduce Bv within 1e-13 relative;
here the same fit on the oracle's Bv reaches rounding level."""
import numpy as np

import harness


def test_bv_is_rank_four_in_the_window_kernels():
    from oracle import refsim
    S = harness.setup("default", schemes=("ofdm",))
    sc = S.schemes["ofdm"]
    G, Q, pil = sc["G"], sc["Q"], sc["pilot_pos"]
    N, LK, NP = G.shape[0], G.shape[1], len(pil)
    ch = S.chan
    j0 = refsim.time_correlation(N, ch["dt"], ch["fD"], ch["model"])        # index lag + N - 1
    pdp = np.asarray(ch["pdp_norm"])
    taps = [(d, pdp[d]) for d in range(len(pdp)) if pdp[d] > 0]
    L = S.L
    # FFT window of each OFDM symbol: the support of its Q columns (CP rows zeroed, OFDM.m:216-217)
    win = [np.flatnonzero(np.abs(Q[:, k * L:(k + 1) * L]).sum(axis=1) > 0) for k in range(LK // L)]
    assert all(w.size == 24 for w in win)
    psym = sorted({int(p) // L for p in pil})
    assert len(psym) == 4
    J = j0[(np.arange(N)[:, None] - np.arange(N)[None, :]) + N - 1]            # J0(n - b)
    T = np.stack([J[:, win[k]].sum(axis=1) for k in psym], axis=1)           # N x 4, real
    mm = harness.oracle_mmse(S, "ofdm")
    rows = np.concatenate(win)
    worst = 0.0
    for s in range(len(S.pn_time)):
        for R in (mm["R_est"][s], mm["R_noI"][s]):
            rinv = np.linalg.pinv(R)
            # the engine's bar (build_mic_lr): max(1e-13, 4e-16 ||R||_1 ||pinv(R)||_1) max|Bv|
            k1 = max(np.abs(R).sum(0).max(), np.abs(R).sum(1).max()) * \
                max(np.abs(rinv).sum(0).max(), np.abs(rinv).sum(1).max())
            tol = max(1e-13, 4e-16 * k1)
            dev = mx = 0.0
            for d, pw in taps:
                # m[j][q][n - d] = PDP_q sum_b J0(n - d - b) Q[b + d, j] conj(G[b, j])
                m = np.zeros((N, NP), dtype=complex)
                for jj, col in enumerate(pil):
                    w = np.zeros(N, dtype=complex)
                    w[:N - d] = Q[d:, col] * np.conj(G[:N - d, col])     # indexed by b
                    mb = pw * (J @ w)                                     # m at column a = n - d
                    m[d:, jj] = mb[:N - d]
                bv = m @ rinv                                             # N x NP
                z, *_ = np.linalg.lstsq(T[rows], bv[rows], rcond=None)
                dev = max(dev, np.abs(T[rows] @ z - bv[rows]).max())
                mx = max(mx, np.abs(bv[rows]).max())
            worst = max(worst, dev / (tol * mx))
            assert dev / mx < 1e-11, (s, dev / mx)
    assert worst < 0.2, worst           # rounding level: well inside the engine's bar
