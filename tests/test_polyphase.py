"""CPU: the polyphase form behind the perfect-CSI IC passes of FBMC and C5 OFDM
(build_poly / k_poly_syn / k_poly_chan / k_poly_ana), checked
on the ORACLE's own G and Q (oracle/setup.py, FBMC.m:255-354, OFDM.m:153-218).

Every symbol's columns are one real window times the subcarrier tones,
G[n, l + L k] = A_k[n] w^(l n) C[l][k] (w = e^(2 pi i / L)), and likewise Q, so
D u = Q^H H G u (script:541-543) is an IDFT-L per symbol, window sums per sample,
the channel, window sums per residue n mod L and a DFT-L per symbol.  Here a
NumPy restatement of exactly that sequence (same factorisation rule as
poly_factor, same residue-major window tables) equals the dense product to
rounding, for C3 / C4 and for C5's FBMC and OFDM schemes."""
import numpy as np
import pytest

import harness


def _factor(M, L, K):
    """poly_factor (dsce_api.hip): A_k = column (0, k) with the phase of its
    largest entry removed, C[l][k] from that entry; returns A (K x N), C (K x L)
    and the largest |M - A w C| / max|M|."""
    N = M.shape[0]
    n = np.arange(N)
    A = np.zeros((K, N))
    C = np.zeros((K, L), complex)
    mmax = np.abs(M).max()
    worst = 0.0
    for k in range(K):
        c0 = M[:, L * k]
        ns = int(np.argmax(np.abs(c0)))
        g = abs(c0[ns])
        a = c0 * np.conj(c0[ns]) / g
        assert np.abs(a.imag).max() <= 1e-12 * mmax
        A[k] = a.real
        lv = np.arange(L)
        C[k] = M[ns, L * k + lv] * np.exp(-2j * np.pi * ((lv * ns) % L) / L) / g
        f = A[k][:, None] * np.exp(2j * np.pi * ((np.outer(n, lv)) % L) / L) * C[k][None, :]
        worst = max(worst, np.abs(M[:, L * k:L * (k + 1)] - f).max() / mmax)
    return A, C, worst


def _poly_apply(A, C, B, E, ir, delays, u, L):
    """Q^H H G u by the three kernels' sequence (one unit)."""
    K, N = A.shape
    V = np.fft.ifft(C * u.reshape(K, L), axis=1) * L              # V_k[m] = sum_l C u w^(l m)
    t = np.zeros(N, complex)
    for k in range(K):
        t += A[k] * V[k][np.arange(N) % L]                         # k_poly_chan, synthesis
    r0 = np.zeros(N, complex)
    for q, d in enumerate(delays):
        r0[d:] += ir[q][d:] * t[:N - d]                            # FastFading.m:284
    fold = np.zeros((K, L), complex)
    for k in range(K):
        np.add.at(fold[k], np.arange(N) % L, B[k] * r0)            # window sums per residue
    return (E * np.fft.fft(fold, axis=1)).reshape(-1)              # k_poly_ana: E DFT(fold)


@pytest.mark.parametrize("cfg,name", [("default", "fbmc_aux"), ("default", "fbmc_cod"),
                                      ("c5", "fbmc_aux"), ("c5", "ofdm")])
def test_polyphase_chain_equals_dense_operator(cfg, name):
    S = harness.setup(cfg, schemes=(name,), snr_db=[20.0])
    sc = S.schemes[name]
    G, Q = sc["G"], sc["Q"]
    N, LK = G.shape
    L = S.L
    K = LK // L
    assert L in (24, 48) and L * K == LK
    A, C, rg = _factor(G, L, K)
    B, Cq, rq = _factor(Q, L, K)
    assert rg < 1e-13 and rq < 1e-13, (rg, rq)
    E = np.conj(Cq)
    ch = S.chan
    pdp = np.asarray(ch["pdp_norm"])
    delays = [d for d in range(len(pdp)) if pdp[d] > 0]
    assert max(delays) < L
    rng = np.random.default_rng(7)
    ir = [rng.standard_normal(N) + 1j * rng.standard_normal(N) for _ in delays]
    H = np.zeros((N, N), complex)
    for q, d in enumerate(delays):
        H[np.arange(d, N), np.arange(N - d)] = ir[q][d:]
    D = Q.conj().T @ H @ G
    for _ in range(3):
        u = rng.standard_normal(LK) + 1j * rng.standard_normal(LK)
        ref = D @ u
        got = _poly_apply(A, C, B, E, ir, delays, u, L)
        assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()
    # the windows are real and short: FBMC 8 (C3) periods of L, OFDM one symbol + CP
    sup = [(np.flatnonzero(A[k]).min(), np.flatnonzero(A[k]).max()) for k in range(K)]
    span = {b - a + 1 for a, b in sup}
    assert len(span) <= 2 and max(span) <= 8 * L
    # residue tables of the kernels hold every sample: ceil(N / L) <= POLY_NI = 24
    assert -(-N // L) <= 24
