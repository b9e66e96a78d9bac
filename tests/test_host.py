"""CPU: host-side mirror of the reference's setup classes (dsce.modulation /
estimation / configs) against the structural statements of the reference."""
import numpy as np
import pytest

import harness  # noqa: F401
from dsce.channel import quantise_pdp
from dsce.configs import build_setup
from dsce.modulation import FBMC, OFDM, SignalConstellation


def test_vehicular_a_pdp_on_sample_grid():
    """FastFading.m:77-80/:111-129 at SR = 360 kHz."""
    _, n = quantise_pdp("VehicularA", 360e3)
    np.testing.assert_allclose(n, [0.979813, 0.020187], atol=1e-6)
    assert n.sum() == pytest.approx(1.0)
    _, n5 = quantise_pdp("VehicularA", 720e3)
    assert n5.size == 3 and np.all(n5 > 0)


@pytest.mark.parametrize("name,N,LKf,LKo,NP", [("default", 540, 720, 336, 16), ("c5", 1080, 1440, 672, 32)])
def test_derived_sizes(name, N, LKf, LKo, NP):
    """SURVEY.md appendix A1."""
    S = build_setup(name, schemes=("ofdm",))
    assert S.N == N
    sc = S.schemes["ofdm"]
    assert sc.LK == LKo and sc.n_pilots == NP and sc.n_data == LKo - NP
    fb = FBMC(S.L, 30, 15e3, S.SR, 0, False, "Hermite-OQAM", 8, 0, True)
    assert fb.Nr.SamplesTotal == N and fb.Nr.Subcarriers * fb.Nr.MCSymbols == LKf


def test_paper_config_sizes():
    fb = FBMC(24, 60, 15e3, 15e3 * 14 * 14, 0, False, "Hermite-OQAM", 8, 0, True)
    assert fb.Nr.SamplesTotal == 7350 and fb.Implementation.TimeSpacing == 98


def test_tx_rx_matrices_reproduce_modulation():
    """G x == Modulation(x), Q' r == Demodulation(r) (FBMC.m:319-320, :344-345;
    OFDM.m:185-186, :206-207)."""
    rng = np.random.default_rng(1)
    for mod in (FBMC(24, 30, 15e3, 360e3, 0, False, "Hermite-OQAM", 8, 0, True),
                OFDM(24, 14, 15e3, 360e3, 0, False, 1 / 15e3 / 14, 88 / 360e3)):
        L, K = mod.Nr.Subcarriers, mod.Nr.MCSymbols
        x = rng.standard_normal((L, K)) + 1j * rng.standard_normal((L, K))
        G = mod.GetTXMatrix()
        np.testing.assert_allclose(G @ x.reshape(-1, order="F"), mod.Modulation(x), atol=1e-12)
        r = rng.standard_normal(mod.Nr.SamplesTotal) + 1j * rng.standard_normal(mod.Nr.SamplesTotal)
        np.testing.assert_allclose(mod.GetRXMatrix() @ r, mod.Demodulation(r).reshape(-1, order="F"), atol=1e-11)


def test_fbmc_oqam_transmission_matrix():
    """Real part of D = Q'G is the identity, the rest is imaginary interference
    (FBMC.m:1-14, :371-377); GetFBMCMatrix == Demod(Mod(.)) (FBMC.m:356-357)."""
    fb = FBMC(24, 30, 15e3, 360e3, 0, False, "Hermite-OQAM", 8, 0, True)
    D = fb.GetRXMatrix() @ fb.GetTXMatrix()
    np.testing.assert_allclose(D.real, np.eye(D.shape[0]), atol=1e-6)
    Df = fb.GetFBMCMatrix()
    for col in (0, 100, 359, 719):
        e = np.zeros(720)
        e[col] = 1
        np.testing.assert_allclose(Df[:, col], fb.Demodulation(fb.Modulation(e)).reshape(-1, order="F"), atol=1e-10)


@pytest.mark.parametrize("M,kind", [(4, "QAM"), (16, "QAM"), (256, "QAM"), (16, "PAM"), (4, "PAM")])
def test_constellation_gray_and_order(M, kind):
    c = SignalConstellation(M, kind)
    lab = (c.BitMapping.astype(int) << np.arange(c.BitsPerSymbol)).sum(axis=1)
    assert np.array_equal(lab, np.arange(M))                      # sorted by bi2de (SignalConstellation.m:64-66)
    assert np.mean(np.abs(c.SymbolMapping) ** 2) == pytest.approx(1.0)
    d = np.abs(c.SymbolMapping[:, None] - c.SymbolMapping[None, :])
    dmin = d[d > 0].min()
    for i in range(M):                                            # Gray: nearest neighbours differ in one bit
        for k in np.flatnonzero(np.abs(d[i] - dmin) < 1e-12):
            assert bin(i ^ k).count("1") == 1
    bits = np.random.default_rng(0).integers(0, 2, c.BitsPerSymbol * 50).astype(np.uint8)
    assert np.array_equal(c.Symbol2Bit(c.Bit2Symbol(bits)), bits)


def test_precoders_cancel_pilot_interference():
    """IIC.m:92-96 / :203-207: high SIR at the pilots, DPR normalisation."""
    S = build_setup("default", schemes=("fbmc_aux", "fbmc_cod", "ofdm"))
    aux = S.schemes["fbmc_aux"].extras["iic"]
    cod = S.schemes["fbmc_cod"].extras["iic"]
    assert aux.SIR_dB.min() > 30 and cod.SIR_dB.min() > 20
    for iic in (aux, cod):
        P = iic.PrecodingMatrix
        assert np.sum(np.abs(P) ** 2) == pytest.approx(P.shape[0])     # numel / DPR scaling
    assert aux.NrDataSymbols == 640 and cod.NrDataSymbols == 688 and aux.NrAuxiliarySymbols == 64
    o = S.schemes["ofdm"]
    assert o.kappa == pytest.approx(2 * o.dpr) and o.dpr == pytest.approx(336 / (16 * 2 + 320))


def test_psace_scattered_interpolation():
    """Config-1 plumbing: 'linear' scatteredInterpolant on the
    pilot grid is exact for affine channels inside and outside the pilot hull
    (SimpleVersion_DoublyFlat.m:47-66 uses Diamond pilots + 'linear'); 'nearest'
    returns the closest pilot's LS value."""
    from dsce.estimation import PilotSymbolAidedChannelEstimation as PSACE
    for pattern, params in (("Diamond", [[12, 4], [15, 4]]), ("Rectangular", [[24, 6], [14, 7]])):
        est = PSACE(pattern, params, "linear")
        PM = est.PilotMatrix
        nL, nK = PM.shape
        f, t = np.meshgrid(np.arange(1, nL + 1), np.arange(1, nK + 1), indexing="ij")
        H = (0.3 - 0.2j) + (0.05 + 0.01j) * f - (0.02 - 0.03j) * t
        ls = H.reshape(-1, order="F")[PM.reshape(-1, order="F") == 1]
        np.testing.assert_allclose(est.ChannelInterpolation(ls), H, rtol=0, atol=1e-12)
        near = PSACE(pattern, params, "nearest").ChannelInterpolation(ls)
        np.testing.assert_allclose(near[PM == 1], H[PM == 1], rtol=0, atol=1e-15)
        pr, pc = np.nonzero(PM)
        for (r, c) in ((0, 0), (nL - 1, nK - 1), (nL // 2, nK // 3)):
            d = (pr - r) ** 2 + (pc - c) ** 2
            assert np.isclose(d[np.argmin(d)], ((pr - r) ** 2 + (pc - c) ** 2)[
                np.argmin(np.abs(H[pr, pc] - near[r, c]))])


def test_psace_linear_weights_match_scipy_inside_hull():
    """PSACE 'linear' weights equal scipy's LinearNDInterpolator (an independent
    Delaunay/barycentric implementation) at every grid point inside the pilot
    hull; every row sums to one (affine fields are reproduced)."""
    from scipy.interpolate import LinearNDInterpolator

    from dsce.estimation import PilotSymbolAidedChannelEstimation as PSACE
    ce = PSACE("Diamond", [[12, 6], [30, 8]], "linear")
    W = ce.GetInterpolationWeights()
    NP = ce.NrPilotSymbols
    assert W.shape == (12 * 30, NP) and np.allclose(W.sum(axis=1), 1.0)
    rows, cols = np.nonzero(ce.PilotMatrix.T)
    pts = np.stack([cols + 1.0, rows + 1.0], axis=1)
    rng = np.random.default_rng(0)
    v = rng.standard_normal(NP) + 1j * rng.standard_normal(NP)
    f = LinearNDInterpolator(pts, v)
    ll, kk = np.meshgrid(np.arange(1, 13.0), np.arange(1, 31.0), indexing="ij")
    ref = f(ll.reshape(-1, order="F"), kk.reshape(-1, order="F"))
    inside = ~np.isnan(ref)
    assert inside.sum() > 100
    assert np.max(np.abs((W @ v)[inside] - ref[inside])) < 1e-12
    got = ce.ChannelInterpolation(v)
    assert np.allclose(got.reshape(-1, order="F"), W @ v)


def test_psace_natural_neighbour_weights():
    """PSACE 'natural' (PSACE.m:74-76, :118-121; scatteredInterpolant 'natural'
    = Sibson coordinates, 'linear' extrapolation).  Checked by properties that
    do not depend on the construction: rows sum to one, non-negative inside the
    hull, affine fields reproduced everywhere (Sibson's linear precision), LS
    values reproduced at the pilots, smooth weights that differ from 'linear';
    and at interior points against a brute-force raster of the definition (the
    share of x's Voronoi cell that each pilot's cell would lose)."""
    from dsce.estimation import PilotSymbolAidedChannelEstimation as PSACE
    from dsce.estimation import _sibson
    parity = "parity unpinned: MATLAB's scatteredInterpolant is absent; property + definition checks"
    for pattern, params in (("Diamond", [[12, 4], [15, 4]]), ("Rectangular", [[24, 6], [14, 7]]),
                            ("Diamond", [[12, 6], [30, 8]])):
        ce = PSACE(pattern, params, "natural")
        W = ce.GetInterpolationWeights()
        PM = ce.PilotMatrix
        nL, nK = PM.shape
        assert W.shape == (nL * nK, ce.NrPilotSymbols)
        np.testing.assert_allclose(W.sum(axis=1), 1.0, rtol=0, atol=1e-12, err_msg=parity)
        f, t = np.meshgrid(np.arange(1, nL + 1), np.arange(1, nK + 1), indexing="ij")
        H = (0.3 - 0.2j) + (0.05 + 0.01j) * f - (0.02 - 0.03j) * t
        ls = H.reshape(-1, order="F")[PM.reshape(-1, order="F") == 1]
        np.testing.assert_allclose(ce.ChannelInterpolation(ls), H, rtol=0, atol=1e-12)
        lin = PSACE(pattern, params, "linear").GetInterpolationWeights()
        assert np.abs(W - lin).max() > 1e-3            # not the linear weights
        piv = PM.reshape(-1, order="F") == 1
        np.testing.assert_allclose(W[piv], np.eye(ce.NrPilotSymbols), atol=1e-12)
    # the definition, by raster, at interior points off the lattice symmetry
    ce = PSACE("Diamond", [[12, 6], [30, 8]], "natural")
    rows, cols = np.nonzero(ce.PilotMatrix.T)
    pts = np.stack([cols + 1.0, rows + 1.0], axis=1)
    h = 0.01
    for x in (np.array([6.3, 14.7]), np.array([5.0, 17.0]), np.array([8.2, 11.1])):
        w = _sibson(pts, x)
        assert w is not None and (w >= -1e-15).all()
        g = np.arange(-7.0, 7.0, h) + h / 2
        px, py = np.meshgrid(x[0] + g, x[1] + g, indexing="ij")
        P = np.stack([px.ravel(), py.ravel()], axis=1)
        d = ((P[:, None, :] - pts[None, :, :]) ** 2).sum(-1)
        near = d.argmin(axis=1)
        mine = ((P - x) ** 2).sum(-1) < d.min(axis=1)
        est = np.bincount(near[mine], minlength=pts.shape[0]) / mine.sum()
        assert np.abs(est - w).max() < 0.01, (x, np.abs(est - w).max())
        np.testing.assert_allclose(w @ pts, x, atol=1e-12)


def test_doubly_flat_setup_matches_script():
    """SimpleVersion_DoublyFlat.m:16-82: sizes, pilots, kappa, noise slots."""
    from dsce.configs import build_doubly_flat_setup
    S = build_doubly_flat_setup()
    assert S.N == 3780 and S.n_iter == 0 and S.channel.MaximumDopplerShift == 0
    assert np.allclose(S.pn_time, 14 * 10 ** (-np.arange(0, 31, 5) / 10))
    a, c, o = (S.schemes[k] for k in ("fbmc_aux", "fbmc_cod", "ofdm"))
    assert (a.LK, c.LK, o.LK) == (360, 360, 180) and a.n_pilots == c.n_pilots == o.n_pilots == 8
    assert o.n_data == 172 and o.kappa == 1.0 and c.kappa == 2.0
    assert (a.extras["noise_slot"], c.extras["noise_slot"], o.extras["noise_slot"]) == (0, 0, 1)
    assert (a.pilot_slot, c.pilot_slot, o.pilot_slot) == (0, 0, 1)
    assert len({a.bits_slot, c.bits_slot, o.bits_slot}) == 3
    # OFDM pilots / data mapped by a permutation (:113-115)
    assert np.allclose(np.abs(o.P).sum(axis=0), 1) and np.allclose(np.abs(o.P).sum(axis=1), 1)


@pytest.mark.parametrize("M,kind", [(4, "QAM"), (16, "QAM"), (256, "QAM"), (4, "PAM"), (16, "PAM")])
def test_theory_module_matches_oracle(M, kind):
    """dsce.theory (vectorised, plotted by the doubly-flat run) against the
    oracle's literal restatement of Theory/BitErrorProbabilityDoublyFlatRayleigh.m."""
    from dsce.modulation import SignalConstellation
    from dsce.theory import bit_error_probability_doubly_flat_rayleigh as bep
    from oracle import refsim
    c = SignalConstellation(M, kind)
    snr = np.arange(-5, 41, 2.5)
    a = bep(snr, c.SymbolMapping, c.BitMapping)
    b = refsim.bit_error_probability_doubly_flat_rayleigh(snr, c.SymbolMapping, c.BitMapping)
    assert np.max(np.abs(a / b - 1)) < 1e-10


def test_psace_patterns_use_matlab_round():
    """PSACE.m:48 rounds half away from zero: Rectangular [[24, 6], [14, 7]]
    puts pilots on rows 4, 10, 16, 22 (1-based) — mod(23, 6) / 2 = 2.5 -> 3 —
    and columns 4, 11; Diamond with an odd spacing (sf = 5, :57-60) offsets the
    second lattice by round(2.5) = 3 and the fourth by round(7.5) = 8."""
    from dsce.estimation import PilotSymbolAidedChannelEstimation as PSACE
    from dsce.estimation import mround
    assert mround(2.5) == 3 and mround(-2.5) == -3 and mround(7.5) == 8
    r = PSACE("Rectangular", [[24, 6], [14, 7]], "linear")
    rows, cols = np.nonzero(r.PilotMatrix)
    assert sorted(set(rows + 1)) == [4, 10, 16, 22] and sorted(set(cols + 1)) == [4, 11]
    d = PSACE("Diamond", [[24, 5], [14, 4]], "linear")
    # FrequencyPositionShift = floor((24 - max(1:10:24, 3.5:10:24, 6:10:24, 8.5:10:24)) / 2) + 1 = 1,
    # TimePositionShift = floor((14 - max(1:8:14, 5:8:14)) / 2) + 1 = 1
    f, t = 1, 1
    want = set()
    for f0, t0 in ((f, t), (f + 3, t + 4), (f + 5, t), (f + 8, t + 4)):
        for a in range(f0, 25, 10):
            for b in range(t0, 15, 8):
                want.add((a - 1, b - 1))
    got = set(zip(*np.nonzero(d.PilotMatrix)))
    assert got == want, sorted(got ^ want)
