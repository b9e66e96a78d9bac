"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on the
same Philox streams.  Floating-point quantities: |gpu - oracle| within the
stated fp64 tolerances; bit-error counts: identical, up to the number of
decisions the oracle flags as borderline (distance margin < 1e-9)."""
import numpy as np
import pytest

import harness  # noqa: F401  (sys.path)
from dsce.configs import build_setup
from oracle import refsim

pytestmark = pytest.mark.gpu

SEED = 0x5EED0002


@pytest.fixture(scope="module")
def ofdm():
    from dsce.engine import build_engine
    S = build_setup("default", schemes=("ofdm",))
    eng = build_engine(S, batch=256)
    mm = harness.oracle_mmse(S, S.schemes["ofdm"])
    yield S, eng, mm
    eng.close()


def test_jakes_ir_matches_oracle(ofdm):
    S, eng, _ = ofdm
    ch = S.channel
    # rep % 8 is the realisation's lane in its batch (dsce_channel_realise): 1 and
    # 77 sit in the second half-wave of k_jakes's two-realisations-per-wave mapping
    for rep in (0, 1, 6, 77, 1 << 33):
        ir_g = eng.channel_impulse_response(SEED, rep)
        ir_o = refsim.jakes_ir(SEED, rep, S.N, ch.dt, ch.PowerDelayProfileNormalized, ch.IndexDelayTaps,
                               ch.MaximumDopplerShift, ch.Paths)
        assert ir_g.shape == ir_o.shape
        np.testing.assert_allclose(ir_g, ir_o, rtol=0, atol=1e-12)


def test_correlation_matrices_match_oracle(ofdm):
    S, eng, mm = ofdm
    rhp, rest, rnoi = eng.correlation(0)
    scale = np.abs(mm["R_hP"]).max()
    np.testing.assert_allclose(rhp, mm["R_hP"], rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(rest, mm["R_est"], rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(rnoi, mm["R_noI"], rtol=0, atol=1e-12 * scale)


def test_mmse_estimator_matches_oracle(ofdm):
    """W = R_Dij pinv(R): the tolerance is fp64 rounding amplified by the
    condition number of R (pinv/inverse of an ill-conditioned pilot
    correlation at high SNR) and growing with its dimension NP,
    tol = 1e-14 * cond(R) * max(1, NP/16) * max|W|."""
    S, eng, mm = ofdm
    for k in range(len(S.pn_time)):
        for var, key, R in ((0, "W", mm["R_est"][k]), (1, "W0", mm["R_noI"][k])):
            wg = eng.W(0, k, var)
            wo = mm[key][:, k]
            scale = np.abs(wo).max()
            tol = max(1e-14 * np.linalg.cond(R) * max(1, R.shape[0] / 16), 1e-12) * scale
            diff = np.abs(wg - wo)
            # entries within tol of the 1e-8 zero threshold may legitimately flip to 0
            border = np.abs(np.abs(wo) - 1e-8) <= tol
            assert np.all((diff <= tol) | border), (k, var, diff.max() / scale, np.linalg.cond(R))


def test_unit_trace_matches_oracle(ofdm):
    S, eng, mm = ofdm
    sc = S.schemes["ofdm"]
    tr = {}
    rep, k = 5, 3
    refsim.simulate(SEED, rep, 1, harness.oracle_chan(S), [harness.oracle_scheme(sc)], S.pn_time, S.n_iter, [mm],
                    trace=tr)
    g = eng.trace_unit(0, SEED, rep, k)
    np.testing.assert_allclose(g["y"], tr["y"][k], rtol=0, atol=1e-10)
    np.testing.assert_allclose(g["h"], np.diag(sc.Q.conj().T @ (np.asarray(
        refsim.conv_matrix(tr["ir"][0], S.channel.PowerDelayProfile, S.N).todense()) @ sc.G)), rtol=0, atol=1e-10)
    # every stage: LS pilot estimates and diag(D_hat) after the MMSE contraction
    # (stage s >= 1 depends on y_est of the k_wcontract kernel).  Decisions
    # are identical here, so the trajectories agree to fp64 rounding.
    for st in range(S.n_iter + 1):
        np.testing.assert_allclose(g["hp"][st], tr["hp_stages"][k][st], rtol=0, atol=1e-9)
        np.testing.assert_allclose(g["hest"][st], tr["hest_stages"][k][st], rtol=0, atol=1e-9)


def test_error_counts_match_oracle(ofdm):
    S, eng, mm = ofdm
    sc = S.schemes["ofdm"]
    n = 64
    eng.enable_mse()
    cg = eng.run(SEED, 0, n)
    res = refsim.simulate(SEED, 0, n, harness.oracle_chan(S), [harness.oracle_scheme(sc)], S.pn_time, S.n_iter, [mm])
    co = res["err"]
    diff = np.abs(cg - co).sum()
    assert diff <= 8 * res["borderline"].sum(), (cg - co)
    _check_mse(eng, res)
    eng.enable_mse(False)
    b = eng.bits_per_rep(0)
    assert b[0] == sc.n_bits and b[1] == sc.considered_symbols.sum() * sc.bits_per_symbol


# ---------------------------------------------------------------------------
# C3 / C4: FBMC-OQAM with auxiliary-symbol and data-spreading precoders
# (two SNR points keep the literal oracle's run time in check)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module", params=["fbmc_aux", "fbmc_cod"])
def fbmc(request):
    from dsce.engine import build_engine
    S = build_setup("default", schemes=(request.param,), snr_db=[15.0, 35.0])
    eng = build_engine(S, batch=256)
    mm = harness.oracle_mmse(S, S.schemes[request.param])
    yield request.param, S, eng, mm
    eng.close()


def test_fbmc_estimator_and_trace(fbmc):
    name, S, eng, mm = fbmc
    sc = S.schemes[name]
    for k in range(2):
        for var, key, R in ((0, "W", mm["R_est"][k]), (1, "W0", mm["R_noI"][k])):
            wg = eng.W(0, k, var)
            wo = mm[key][:, k]
            scale = np.abs(wo).max()
            tol = max(1e-14 * np.linalg.cond(R) * max(1, R.shape[0] / 16), 1e-12) * scale
            border = np.abs(np.abs(wo) - 1e-8) <= tol
            assert np.all((np.abs(wg - wo) <= tol) | border), (name, k, var)
    tr = {}
    refsim.simulate(SEED, 9, 1, harness.oracle_chan(S), [harness.oracle_scheme(sc)], S.pn_time, S.n_iter, [mm],
                    trace=tr)
    for k in range(2):
        g = eng.trace_unit(0, SEED, 9, k)
        np.testing.assert_allclose(g["y"], tr["y"][k], rtol=0, atol=1e-10)
        for st in range(S.n_iter + 1):
            np.testing.assert_allclose(g["hp"][st], tr["hp_stages"][k][st], rtol=0, atol=1e-9)
            np.testing.assert_allclose(g["hest"][st], tr["hest_stages"][k][st], rtol=0, atol=1e-9)


def test_fbmc_error_counts(fbmc):
    name, S, eng, mm = fbmc
    sc = S.schemes[name]
    eng.enable_mse()
    cg = eng.run(SEED, 64, 64)
    res = refsim.simulate(SEED, 64, 64, harness.oracle_chan(S), [harness.oracle_scheme(sc)], S.pn_time, S.n_iter,
                          [mm])
    assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), (name, cg - res["err"])
    _check_mse(eng, res)
    eng.enable_mse(False)


def _check_mse(eng, res):
    """dsce_get_mse (build-defined channel-estimation MSE, parity unpinned vs
    MATLAB) against the oracle's sums: fp64 sums of O(1e4) terms, 1e-9
    relative; and a sane NMSE (below 1, decreasing with SNR at stage 0)."""
    err, pw = eng.mse()
    np.testing.assert_allclose(err, res["mse_err"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(pw, res["mse_pow"], rtol=1e-12, atol=0)
    nmse = err[..., 0] / pw
    assert np.all(nmse < 1) and np.all(np.diff(nmse, axis=-1) < 0)


def test_three_schemes_share_channel_and_noise():
    """script:350-403: one channel draw and one noise draw per (rep, SNR) feed
    all three schemes; a joint engine equals three single-scheme engines."""
    from dsce.engine import build_engine
    S = build_setup("default", snr_db=[25.0])
    joint = build_engine(S, batch=128)
    cj = joint.run(SEED, 0, 128)
    joint.close()
    for i, name in enumerate(S.schemes):
        e = build_engine(S, schemes=(name,), batch=128)
        np.testing.assert_array_equal(e.run(SEED, 0, 128)[0], cj[i])
        e.close()


def test_counts_are_additive_and_batch_invariant(ofdm):
    """Size-independent properties at any scale: [0,2B) = [0,B) + [B,2B), and the
    device batch size does not change a single count."""
    S, eng, _ = ofdm
    a = eng.run(SEED, 0, 512)
    b = eng.run(SEED, 0, 256) + eng.run(SEED, 256, 256)
    np.testing.assert_array_equal(a, b)
    eng.set_batch(64)
    c = eng.run(SEED, 0, 512)
    eng.set_batch(256)
    np.testing.assert_array_equal(a, c)


def test_psace_mmse_plugin(ofdm):
    """The 'MMSE' method of PilotSymbolAidedChannelEstimation (a stub in the
    reference, PSACE.m:110-111/:128-129) served by the engine equals
    diag(sum_p W_p hP_p) of script:417-428."""
    from dsce.estimation import PilotSymbolAidedChannelEstimation
    S, eng, mm = ofdm
    sc = S.schemes["ofdm"]
    pm = sc.extras["pilot_matrix"]
    est = PilotSymbolAidedChannelEstimation("Custom", pm, "MMSE")
    est.set_mmse_engine(eng, 0, 3)
    rng = np.random.default_rng(4)
    ls = rng.standard_normal(16) + 1j * rng.standard_normal(16)
    got = est.ChannelInterpolation(ls)
    W3 = mm["W"][:, 3].reshape(sc.LK, sc.LK, 16, order="F")
    ref = np.diag((W3 * ls[None, None, :]).sum(axis=2))
    np.testing.assert_allclose(got.reshape(-1, order="F"), ref, rtol=0, atol=1e-11 * np.abs(ref).max())


def test_w_band_trim_is_bit_exact(monkeypatch):
    """Trimming W to its non-zero column extent (after the 1e-8 threshold) skips
    exact zeros only: counts are bit-identical and the contracted work shrinks."""
    from dsce.engine import build_engine
    S = build_setup("default", schemes=("fbmc_aux",), snr_db=[20.0, 40.0])
    monkeypatch.setenv("DSCE_WTRIM", "0")
    full = build_engine(S, batch=128)
    monkeypatch.setenv("DSCE_WTRIM", "1")
    trim = build_engine(S, batch=128)
    np.testing.assert_array_equal(full.run(SEED, 0, 128), trim.run(SEED, 0, 128))
    for k in range(2):
        np.testing.assert_array_equal(full.W(0, k, 0), trim.W(0, k, 0))
    assert trim.work_model(0)[0] < 0.7 * full.work_model(0)[0]
    full.close()
    trim.close()


@pytest.mark.parametrize("name", ["ofdm", "fbmc_aux"])
def test_stage_variants_agree(monkeypatch, name):
    """The fused select-mode stage (k_ls + k_stage_fused, any row-block size,
    perfect-CSI branch fused into perfect_ic or not, any work order) and the
    3-kernel split path (k_ls_hest, k_detect, k_precode) differ only in rounding
    of the one-tap quotient: identical counts on 1024 realisations."""
    from dsce.engine import build_engine
    S = build_setup("default", schemes=(name,), snr_db=[10.0, 25.0, 40.0])
    eng = build_engine(S, batch=512)
    monkeypatch.setenv("DSCE_STAGE", "split")
    ref = eng.run(SEED, 0, 1024)
    monkeypatch.setenv("DSCE_STAGE", "fused")
    for rb in ("4", "8", "16"):
        monkeypatch.setenv("DSCE_STAGE_RB", rb)
        np.testing.assert_array_equal(eng.run(SEED, 0, 1024), ref, err_msg=rb)
    # perfect-CSI detection fused into perfect_ic (OFDM) on/off, XCD-aware
    # work order on/off, SNR-chunked receiver, two streams instead of one, the
    # one-pass perfect-CSI IC (k_pic) instead of the two passes, 4-MFMA instead of
    # 3M complex products, 32-row contraction tiles instead of pairs, the MMSE
    # stage as its own kernels instead of fused into the contraction, the
    # perfect-CSI chain as per-iteration passes / VALU chain instead of k_pic_mfma,
    # the fused epilogue's diag(D_hat) with 4 real MFMAs instead of 3M, one
    # realisation per Jakes wave (17- vs 9-sample recurrence chunks), the fused
    # contraction held to 3 waves/SIMD
    variants = ({"DSCE_PFUSE": "0"}, {"DSCE_XCD": "0"}, {"DSCE_SNR_CHUNK": "2"}, {"DSCE_STREAMS": "2"},
                {"DSCE_PIC": "1", "DSCE_PIC_CHAIN": "0"}, {"DSCE_WPAIR_3M": "0"}, {"DSCE_WCONTRACT": "mfma"},
                {"DSCE_FUSE_STAGE": "0"}, {"DSCE_PIC_CHAIN": "0"}, {"DSCE_PIC_CHAIN": "1"},
                {"DSCE_STREAMS": "2", "DSCE_FUSE_STAGE": "0"}, {"DSCE_NOISE_FUSE": "0"}, {"DSCE_WDA_3M": "0"},
                {"DSCE_JAKES_RPW": "1"}, {"DSCE_WPAIR_3W": "1"}, {"DSCE_WPAIR_3W": "1", "DSCE_WDA_3M": "0"})
    for env in variants:
        for var, val in env.items():
            monkeypatch.setenv(var, val)
        np.testing.assert_array_equal(eng.run(SEED, 0, 1024), ref, err_msg=str(env))
        for var in env:
            monkeypatch.delenv(var)
    eng.close()


def test_w3_layouts_agree(monkeypatch):
    """W's 3M planes packed two k-steps per 16-byte lane load (default) or one
    double per lane (DSCE_W3_X4=0, chosen when the estimator is built): the
    contraction reads the same values, counts are identical, fused and unfused."""
    from dsce.engine import build_engine
    S = build_setup("default", schemes=("ofdm",), snr_db=[10.0, 25.0, 40.0])
    x4 = build_engine(S, batch=512)
    monkeypatch.setenv("DSCE_W3_X4", "0")
    x2 = build_engine(S, batch=512)
    monkeypatch.delenv("DSCE_W3_X4")
    for fuse in ("1", "0"):
        monkeypatch.setenv("DSCE_FUSE_STAGE", fuse)
        np.testing.assert_array_equal(x4.run(SEED, 0, 1024), x2.run(SEED, 0, 1024), err_msg=fuse)
    x4.close()
    x2.close()


@pytest.mark.parametrize("name", ["default", "c5", "paper"])
def test_tx_matrices_on_gpu_match_host_mirror(name):
    """Row f1: G and Q = GetRXMatrix' produced on the GPU in closed form equal
    the host mirror's L Modulation() calls (OFDM.m:184-218, FBMC.m:318-354)."""
    from dsce.engine import Engine
    from dsce.configs import build_setup
    S = build_setup(name, schemes=("fbmc_aux", "ofdm"))
    eng = Engine()
    for key in ("fbmc_aux", "ofdm"):
        sc = S.schemes[key]
        G, Q = eng.tx_matrices(sc.extras["modulation"])
        scale = np.abs(sc.G).max()
        np.testing.assert_allclose(G, sc.G, rtol=0, atol=1e-13 * scale, err_msg=key)
        np.testing.assert_allclose(Q, sc.Q, rtol=0, atol=1e-13 * np.abs(sc.Q).max(), err_msg=key)
    eng.close()
