"""CPU: the oracle pinned against every known answer available offline
(Random123 KATs, the reference's own closed-form BEP, structural invariants
stated in the reference) and against its committed regression vectors."""
import json
import os

import numpy as np
import pytest

import harness  # noqa: F401
from oracle import philox, refsim

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_philox_known_answers():
    for v in json.load(open(os.path.join(GOLD, "philox_kat.json"))):
        out = philox.philox4x32_10(*[np.uint32(c) for c in v["ctr"]], *v["key"])
        assert [int(x) for x in out] == v["out"]


def test_stream_layout():
    # bits: bit i = bit (i&31) of word ((i>>5)&3) of counter i>>7
    b = philox.bits(7, 3, 2, 300)
    w = philox._block(7, 3, philox.STREAM_BITS, 2, np.arange(3, dtype=np.uint32))
    words = np.stack(w, axis=1).reshape(-1)
    for i in (0, 31, 32, 127, 128, 299):
        assert b[i] == (int(words[i >> 5]) >> (i & 31)) & 1
    u = philox.uniforms(7, 3, philox.STREAM_THETA, 0, 5)
    assert np.all((u >= 0) & (u < 1))
    assert not np.array_equal(philox.uniforms(7, 4, 1, 0, 8), philox.uniforms(7, 3, 1, 0, 8))
    re, im = philox.complex_normals(9, 1, 0, 200000)
    assert abs(re.mean()) < 0.01 and abs(im.std() - 1) < 0.01 and abs(np.mean(re * im)) < 0.01
    idx = philox.indices(1, 2, 0, 4000, 16)
    assert idx.min() == 0 and idx.max() == 15


def test_theory_bep_closed_form_4qam():
    """Theory/BitErrorProbabilityDoublyFlatRayleigh.m vs the reference's own
    closed form for 4-QAM (SimpleVersion_DoublyFlat.m:179)."""
    from dsce.modulation import SignalConstellation
    g = json.load(open(os.path.join(GOLD, "theory_4qam.json")))
    q = SignalConstellation(4, "QAM")
    got = refsim.bit_error_probability_doubly_flat_rayleigh(g["snr_db"], q.SymbolMapping, q.BitMapping)
    np.testing.assert_allclose(got, g["bep"], rtol=1e-10, atol=1e-15)   # 0.5 - x cancellation at high SNR


def test_theory_bep_256qam_lower_bound_of_figure5():
    """The grey 'doubly-flat theory' line of png/Figure5.png is ~0.0129 at 32 dB."""
    from dsce.modulation import SignalConstellation
    q = SignalConstellation(256, "QAM")
    b = refsim.bit_error_probability_doubly_flat_rayleigh([32.0], q.SymbolMapping, q.BitMapping)[0]
    assert abs(b - 0.0129) < 0.0004


def test_jakes_statistics():
    """Sum of sinusoids: E|h_tau|^2 = PDPn[tau], E{h(n) h*(n+k)} ~ J0(2 pi fD k dt)."""
    S = harness.setup("default", schemes=())
    ch = S.chan
    irs = np.stack([refsim.jakes_ir(3, r, S.N, ch["dt"], ch["pdp_norm"], ch["idx_taps"], ch["fD"], ch["paths"])
                    for r in range(300)])
    p = np.mean(np.abs(irs) ** 2, axis=(0, 1))
    np.testing.assert_allclose(p, ch["pdp_norm"], rtol=0.12)
    lag = 200
    c = np.mean(irs[:, :-lag, 0] * np.conj(irs[:, lag:, 0])) / ch["pdp_norm"][0]
    tc = refsim.time_correlation(S.N, ch["dt"], ch["fD"])[S.N - 1 + lag]
    assert abs(c.real - tc) < 0.12


def test_convolution_matrix_structure():
    """GetConvolutionMatrix: H[n, n - tau] = IR[n, tau], zero elsewhere."""
    N = 40
    pdp = np.array([0.5, 0.0, 0.3, 0.2])
    ir = (np.arange(N)[:, None] + 1j * np.arange(4)[None, :]) * (pdp > 0)
    H = refsim.conv_matrix(ir, pdp, N).toarray()
    ref = np.zeros((N, N), dtype=complex)
    for tau in np.flatnonzero(pdp):
        for n in range(tau, N):
            ref[n, n - tau] = ir[n, tau]
    np.testing.assert_array_equal(H, ref)


def test_correlation_matrix_literal_structure():
    """R_vecH[vec(H[a+tau,a]), vec(H[b+tau,b])] = PDPn[tau] J0(a-b), including the
    column wrap of FastFading.m:377 for tau >= 2 (entries with a+tau >= N land in
    row a+tau-N of column a+1 and survive the crop at N^2)."""
    N = 12
    pdp = np.array([0.6, 0.3, 0.1])
    tc = refsim.time_correlation(N, 1 / 720e3, 1158.18)
    R = refsim.correlation_matrix(N, pdp, tc).toarray()
    f = lambda a, t: a * (N + 1) + t
    for t in range(3):
        for a in range(N):
            for b in range(N):
                if f(a, t) < N * N and f(b, t) < N * N:
                    assert R[f(a, t), f(b, t)] == pytest.approx(pdp[t] * tc[N - 1 + a - b], abs=1e-15)
    assert R[f(N - 2, 2), f(N - 2, 2)] != 0          # the wrapped entry (row 0, column N-1)
    assert np.count_nonzero(R) == sum(min(N, (N * N - t + N) // (N + 1)) ** 2 for t in range(3))


@pytest.fixture(scope="module")
def c2():
    S = harness.setup("default", schemes=("ofdm",))
    return S, harness.oracle_mmse(S, "ofdm")


def test_correlation_invariants(c2):
    S, mm = c2
    R = mm["R_hP"]
    np.testing.assert_allclose(R, R.conj().T, atol=1e-14)
    assert np.linalg.eigvalsh(R).min() > -1e-12
    for k in range(len(S.pn_time)):
        assert np.all(np.real(np.diag(mm["R_est"][k])) >= np.real(np.diag(R)) - 1e-12)
    w = mm["W"]
    nz = np.abs(w[w != 0])
    assert nz.min() >= 1e-8                               # script:287-289 threshold
    # block-diagonal OFDM estimator: only same-symbol (r, c) pairs survive
    LK = S.schemes["ofdm"]["G"].shape[1]
    W3 = w[:, 0].reshape(LK, LK, -1, order="F")
    r, c = np.nonzero(np.abs(W3).sum(axis=2))
    assert np.all(r // 24 == c // 24)


def test_oracle_regression_vectors(c2):
    S, mm = c2
    g = json.load(open(os.path.join(GOLD, "oracle_c2_small.json")))
    tr = {}
    res = harness.simulate(S, g["seed"], 0, 2, ["ofdm"], trace=tr)
    ir = tr["ir"][0]
    for n, v in g["ir_rep0_samples"].items():
        n = int(n)
        np.testing.assert_allclose([ir[n, 0].real, ir[n, 0].imag, ir[n, 1].real, ir[n, 1].imag], v, atol=1e-13)
    np.testing.assert_allclose([[z.real, z.imag] for z in np.diag(mm["R_hP"])], g["rhp_diag"], atol=1e-13)
    assert res["err"].tolist() == g["err"]
    assert res["nbits"].tolist() == g["nbits"]


# ---------------------------------------------------------------------------
# FastFading's other realisation branches and the doubly-flat loop (config 1)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("model", ["Discrete-Jakes", "Discrete-Uniform"])
def test_discrete_ir_direct_sum_equals_ifft(model):
    """The literal IFFT of FastFading.m:203-221 equals the direct sum over the
    2 nd + 1 Doppler bins that k_discrete evaluates."""
    N, SR, fD = 540, 360e3, 500 / 3.6 * 2.5e9 / 2.998e8
    pdp = np.array([0.979813, 0.020187])
    ir = refsim.discrete_ir(11, 5, N, SR, pdp, [0, 1], fD, model)
    nd, S = refsim.discrete_doppler_spectrum(N, SR, fD, model)
    assert nd == 2 and abs(S.sum() - 1) < 1e-15
    nb = 2 * nd + 1
    re, im = philox.normal_pairs(11, 5, philox.STREAM_THETA, 1, np.arange(2 * nb))
    z = (re + 1j * im).reshape(nb, 2, order="F")
    n = np.arange(N)
    for q in range(2):
        c = np.sqrt(S) * np.sqrt(pdp[q]) / np.sqrt(2) * z[:, q]
        direct = (c[:, None] * np.exp(2j * np.pi * np.outer(np.arange(-nd, nd + 1), n) / N)).sum(axis=0)
        assert np.max(np.abs(direct - ir[:, q])) < 1e-14


def test_discrete_low_velocity_is_time_invariant():
    """fD/df <= 0.5 sets the velocity to zero (FastFading.m:153-156)."""
    ir = refsim.discrete_ir(3, 1, 540, 360e3, [1.0], [0], 300.0, "Discrete-Jakes")
    assert np.all(ir == ir[0]) and ir[0, 0] == refsim.static_ir(3, 1, 540, [1.0], [0])[0, 0]


def test_static_and_discrete_channel_power():
    """E|IR[n, tau]|^2 = PDPn[tau] for the time-invariant (:244) and the discrete
    Doppler (:207-221, spectrum normalised to 1) branches."""
    pdp = np.array([0.7, 0.0, 0.3])
    st = np.array([refsim.static_ir(1, r, 8, pdp, [0, 2])[0] for r in range(4000)])
    assert np.allclose(np.mean(np.abs(st) ** 2, axis=0), pdp, atol=0.03)
    dj = np.array([refsim.discrete_ir(2, r, 64, 64e3, pdp, [0, 2], 3e3, "Discrete-Jakes")[::16] for r in range(2000)])
    assert np.allclose(np.mean(np.abs(dj) ** 2, axis=(0, 1)), pdp, atol=0.03)


def test_doubly_flat_oracle_vs_theory_low_snr():
    """SimpleVersion_DoublyFlat.m restated: OFDM with perfect CSI against the
    reference's own closed-form BEP (Theory/..., script :181) at 0 and 5 dB
    (where 150 realisations resolve it; the GPU test covers the full curve)."""
    from dsce.configs import build_doubly_flat_setup
    S = build_doubly_flat_setup(snr_db=[0.0, 5.0])
    sc = S.schemes["ofdm"]
    d = harness.product_scheme_dict(sc)
    d.update(noise_slot=sc.extras["noise_slot"], interp=sc.extras["interp"])
    n = 150
    r = refsim.simulate_doubly_flat(0x5EED0001, 0, n, S.N, [d], S.pn_time)
    ber = r["err"][0] / (sc.n_bits * n)
    th = refsim.bit_error_probability_doubly_flat_rayleigh(S.snr_db, sc.const.SymbolMapping, sc.const.BitMapping)
    assert np.all(np.abs(ber[1] / th - 1) < 0.15), (ber[1], th)
    assert np.all(ber[0] > ber[1])                 # interpolated channel is worse than perfect CSI


# ---------------------------------------------------------------------------
# SURVEY §8(c)-4 fixtures: the oracle and its setup restatement recomputed and
# compared with the committed vectors of tests/golden/make_golden.py
# ---------------------------------------------------------------------------
def _golden():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _same(a, b, path="", rtol=1e-10):
    if isinstance(a, dict):
        assert set(a) == set(b), path
        for k in a:
            _same(a[k], b[k], path + "/" + str(k), rtol)
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _same(x, y, "%s[%d]" % (path, i), rtol)
    elif isinstance(a, float) or isinstance(b, float):
        assert abs(a - b) <= rtol * max(1.0, abs(a), abs(b)), (path, a, b)
    else:
        assert a == b, (path, a, b)


@pytest.mark.parametrize("name,fname,schemes", [("default", "setup_default.json", ("fbmc_aux", "fbmc_cod", "ofdm")),
                                                ("c5", "setup_c5.json", ("fbmc_aux", "fbmc_cod", "ofdm"))])
def test_setup_fixtures(name, fname, schemes):
    got = json.loads(json.dumps(_golden().setup_fixture(name, schemes)))
    _same(got, json.load(open(os.path.join(GOLD, fname))))


@pytest.mark.parametrize("tag", ["c3", "c4", "c5"])
def test_oracle_fixtures(tag):
    """8 realisations of IR / D = Q'HG, R_hP, W slices and int64 counts (C3, C4:
    FBMC auxiliary / coding 24 x 30; C5: OFDM 48 x 14 at 720 kHz)."""
    got = json.loads(json.dumps(_golden().oracle_fixture(tag)))
    ref = json.load(open(os.path.join(GOLD, "oracle_%s_small.json" % tag)))
    assert got["err_reps_0_2"] == ref["err_reps_0_2"] and got["nbits"] == ref["nbits"]
    _same(got, ref, rtol=1e-9)


def test_sparse_w_contraction_equals_literal_full_w():
    """refsim.simulate(w_sparse=True) forms D_hat = reshape(W hP) from W's stored
    non-zeros (used for the C5 FBMC parity tests, where full(W) is 1 GB per
    evaluation) instead of the literal full(W) .* hP summed over the third
    dimension (script:417-425, :493-511): identical counts, traces equal to
    summation-order rounding.  C4 (FBMC data spreading), 2 realisations."""
    import harness
    from oracle import refsim
    S = harness.setup("default", schemes=("fbmc_cod",), snr_db=[35.0])
    mm = harness.oracle_mmse(S, "fbmc_cod")
    sc = S.schemes["fbmc_cod"]
    ta, tb = {}, {}
    a = refsim.simulate(0x5EED0004, 3, 2, S.chan, [sc], S.pn_time, S.n_iter, [mm], trace=ta)
    b = refsim.simulate(0x5EED0004, 3, 2, S.chan, [sc], S.pn_time, S.n_iter, [mm], trace=tb, w_sparse=True)
    np.testing.assert_array_equal(a["err"], b["err"])
    np.testing.assert_allclose(a["mse_err"], b["mse_err"], rtol=1e-12)
    for ua, ub in zip(ta["units"], tb["units"]):
        for key in ("hp", "hest", "yest", "yperf"):
            np.testing.assert_allclose(np.array(ub[key]), np.array(ua[key]), rtol=0, atol=1e-12)
