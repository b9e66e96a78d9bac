"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on the
same Philox streams and the same, independently produced setup (the oracle's
own restatement oracle/setup.py, handed to the engine as data; tests/harness.py).
Floating-point quantities: |gpu - oracle| within the stated fp64 tolerances;
bit-error counts: identical, up to the number of decisions the oracle flags as
borderline (distance margin < 1e-9)."""
import numpy as np
import pytest

import harness
from oracle import refsim

pytestmark = pytest.mark.gpu

SEED = 0x5EED0002


@pytest.fixture(scope="module")
def ofdm():
    S = harness.setup("default", schemes=("ofdm",))
    eng = harness.engine(S, batch=256)
    mm = harness.oracle_mmse(S, "ofdm")
    yield S, eng, mm
    eng.close()


def test_jakes_ir_matches_oracle(ofdm):
    S, eng, _ = ofdm
    ch = S.chan
    # rep % 8 is the realisation's lane in its batch (dsce_channel_realise): 1 and
    # 77 sit in the second half-wave of k_jakes's two-realisations-per-wave mapping
    for rep in (0, 1, 6, 77, 1 << 33):
        ir_g = eng.channel_impulse_response(SEED, rep)
        ir_o = refsim.jakes_ir(SEED, rep, S.N, ch["dt"], ch["pdp_norm"], ch["idx_taps"], ch["fD"], ch["paths"])
        assert ir_g.shape == ir_o.shape
        np.testing.assert_allclose(ir_g, ir_o, rtol=0, atol=1e-12)


@pytest.mark.parametrize("mom,grp2", [(2, 1), (2, 0), (1, 1), (0, 1)])
def test_jakes_window_kernels_match_oracle(ofdm, mom, grp2):
    """The run's Jakes kernels (only the samples the Q^H windows read):
    k_jakes_grp2 (Taylor anchors over runs of windows, both taps per wave; the
    default for two-tap channels since r06), k_jakes_grp (one tap per block),
    k_jakes_mom (one anchor per window) and the recurrence, each against the
    oracle's per-sample sum of sinusoids at the window samples, 1e-12."""
    S, eng, _ = ofdm
    ch = S.chan
    eng.set_option("realise_win", 1)
    eng.set_option("jakes_mom", mom)
    eng.set_option("jakes_grp2", grp2)
    try:
        for rep in (0, 1, 6, 77, 1 << 33):
            ir_g = eng.channel_impulse_response(SEED, rep)
            ir_o = refsim.jakes_ir(SEED, rep, S.N, ch["dt"], ch["pdp_norm"], ch["idx_taps"], ch["fD"], ch["paths"])
            mask = ir_g != 0
            # every tap's window samples: C2 reads 14 windows of 24
            assert mask.sum() >= 14 * 24 * len(ch["idx_taps"]), mask.sum()
            np.testing.assert_allclose(ir_g[mask], ir_o[mask], rtol=0, atol=1e-12, err_msg=str((mom, rep)))
    finally:
        eng.set_option("realise_win", 0)
        eng.set_option("jakes_mom", 2)
        eng.set_option("jakes_grp2", 1)


@pytest.mark.parametrize("mom", [2, 1, 0])
def test_teardown_is_clean_after_window_realisations(mom):
    """Regression for the r04 double free (fixed in 5b14aa2): dsce_channel_realise
    with realise_win 1 allocates the Jakes window tables behind its scratch; the
    scratch is freed by pointer and dsce_destroy (ABI 6: returns a status,
    Engine.close raises on it) must then free every buffer exactly once.  A run
    between the realisations puts the batch buffers in the list too."""
    S = harness.setup("default", schemes=("ofdm",))
    eng = harness.engine(S, batch=64)
    eng.set_option("realise_win", 1)
    eng.set_option("jakes_mom", mom)
    eng.channel_impulse_response(SEED, 3)
    eng.run(SEED, 0, 64)
    eng.channel_impulse_response(SEED, 77)
    eng.close()          # raises DsceError on a failed teardown call


def test_correlation_matrices_match_oracle(ofdm):
    S, eng, mm = ofdm
    rhp, rest, rnoi = eng.correlation(0)
    scale = np.abs(mm["R_hP"]).max()
    np.testing.assert_allclose(rhp, mm["R_hP"], rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(rest, mm["R_est"], rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(rnoi, mm["R_noI"], rtol=0, atol=1e-12 * scale)


def _check_W(eng, mm, nsnr):
    """W = R_Dij pinv(R): the tolerance is fp64 rounding amplified by the
    condition number of R (pinv/inverse of an ill-conditioned pilot
    correlation at high SNR) and growing with its dimension NP,
    tol = 1e-14 * cond(R) * max(1, NP/16) * max|W|; entries within tol of the
    1e-8 zero threshold (script:287-289) may legitimately flip to 0."""
    for k in range(nsnr):
        for var, key, R in ((0, "W", mm["R_est"][k]), (1, "W0", mm["R_noI"][k])):
            wg = eng.W(0, k, var)
            wo = mm[key][:, k]
            scale = np.abs(wo).max()
            tol = max(1e-14 * np.linalg.cond(R) * max(1, R.shape[0] / 16), 1e-12) * scale
            diff = np.abs(wg - wo)
            border = np.abs(np.abs(wo) - 1e-8) <= tol
            assert np.all((diff <= tol) | border), (k, var, diff.max() / scale, np.linalg.cond(R))


def test_mmse_estimator_matches_oracle(ofdm):
    S, eng, mm = ofdm
    _check_W(eng, mm, len(S.pn_time))


# ---------------------------------------------------------------------------
# The benchmarked kernels under direct oracle parity (bench path = C2 OFDM:
# k_txrx_fft for TX / channel / noisy receiver front, k_pic_fft for the whole
# perfect-CSI branch (stage 0 + IC chain), k_mic_pilot + k_mic_data for every
# stage of the MMSE branch (Q' H_hat G by FFT)), and the W contraction
# (k_pilot_pre + fused k_wpair3 epilogue, mmse_ic 0) alongside.
# ---------------------------------------------------------------------------
BENCH_BASE = {"mic_fft", "mic_stages", "pic_fft", "noise_fused", "txrx_fft"}


def bench_path(eng):
    """The bench path's kernels; the low-rank tap operator (k_mic_pilot /
    k_mic_data LR) when the engine's mic_lr option is on (its default)."""
    return BENCH_BASE | ({"mic_lr"} if eng.get_option("mic_lr") else set())


W_PATH = {"wpair3_fused", "pic_fft", "stage_fused", "noise_fused", "txrx_fft"}


def _check_trace(g, u, name, tol=1e-9):
    """Per element, per stage: |gpu - oracle| <= 1e-9 for y, h = diag(D), hP,
    diag(D_hat) and y_est (all rows); decisions identical except where the
    oracle's nearest-point margin is below 1e-9 (borderline, none expected)."""
    ns = len(u["hp"])
    np.testing.assert_allclose(g["y"], u["y"], rtol=0, atol=1e-10, err_msg=name)
    np.testing.assert_allclose(g["h"], u["h"], rtol=0, atol=1e-10, err_msg=name)
    for st in range(ns):
        np.testing.assert_allclose(g["hp"][st], u["hp"][st], rtol=0, atol=tol, err_msg="%s hp %d" % (name, st))
        np.testing.assert_allclose(g["hest"][st], u["hest"][st], rtol=0, atol=tol, err_msg="%s hest %d" % (name, st))
        np.testing.assert_allclose(g["yest"][st], u["yest"][st], rtol=0, atol=tol, err_msg="%s yest %d" % (name, st))
        for key, mk in (("dec_e", "margin_e"), ("dec_p", "margin_p")):
            ok = (g[key][st] == u[key][st]) | (u[mk][st] < 1e-9)
            assert ok.all(), (name, key, st, np.flatnonzero(~ok)[:8])
    return ns


def test_bench_kernels_trace_matches_oracle(ofdm):
    """dsce_trace_unit_ex runs the same kernels as dsce_run (asserted through
    dsce_path_info) and every intermediate of every stage of a unit matches the
    oracle (literal W of script:493-511): k_mic_pilot / k_mic_data's y_est,
    LS pilots and diag(D_hat) of every stage, k_pic_fft's y_perf (data rows:
    the chain forms only those) and both branches' decisions; the same for the
    fused W contraction (mmse_ic 0: k_pilot_pre + k_wpair3 epilogue, stage 0
    from k_stage_fused, k_pic_fft without its stage 0)."""
    S, eng, mm = ofdm
    rows = S.schemes["ofdm"]["data_pos"]
    for mic, path in ((1, bench_path(eng)), (0, W_PATH)):
        eng.set_option("mmse_ic", mic)
        for rep in (5, 70):
            tr = {}
            harness.simulate(S, SEED, rep, 1, ["ofdm"], trace=tr)
            for k in range(len(S.pn_time)):
                g = eng.trace_unit(0, SEED, rep, k)
                assert path <= eng.path_info(0), eng.path_info(0)
                u = tr["units"][k]
                ns = _check_trace(g, u, "mmse_ic %d rep %d snr %d" % (mic, rep, k))
                for st in range(1, ns):
                    np.testing.assert_allclose(g["yperf"][st][rows], u["yperf"][st][rows], rtol=0, atol=1e-9)
    eng.set_option("mmse_ic", 1)


def test_nonuniform_row_precoder_matches_oracle():
    """A row-local precoder whose data rows carry different unit-modulus
    factors (SchemeK::pv_uni 0): the non-uniform re-precode branch of k_pic_fft
    and k_mic_data (row value x the staged constellation, the constant rows
    from the lane's LDS slot, r05) against the oracle on the same P: counts
    within the borderline bar, the FFT-form kernels ran (asserted)."""
    import copy
    from types import SimpleNamespace
    S0 = harness.setup("default", schemes=("ofdm",))
    S = SimpleNamespace(**vars(S0))
    S.name = "default_pv_rotated"          # its own oracle_mmse cache entry
    S.schemes = copy.deepcopy(S0.schemes)
    sc = S.schemes["ofdm"]
    NP = len(sc["pilot_pos"])
    P = sc["P"].copy()
    ph = np.exp(1j * np.pi / 4 * (np.arange(P.shape[1] - NP) % 3))
    P[:, NP:] = P[:, NP:] * ph[None, :]
    sc["P"] = P
    eng = harness.engine(S, batch=256)
    try:
        cg = eng.run(SEED, 0, 64)
        assert {"pic_fft", "mic_stages"} <= eng.path_info(0), eng.path_info(0)
        res = harness.simulate(S, SEED, 0, 64, ["ofdm"])
        assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), cg - res["err"]
        assert res["err"].sum() > 0
    finally:
        eng.close()


def test_error_counts_match_oracle(ofdm):
    """Error counts and MSE sums through the bench path, 64 realisations x 7 SNR
    points (7 x 14 perfect-CSI chain blocks: not a multiple of the 8 XCDs) and
    128 x 7; the bench kernels ran (asserted)."""
    S, eng, mm = ofdm
    sc = S.schemes["ofdm"]
    eng.enable_mse()
    for first, n in ((0, 64), (128, 128)):
        eng.set_batch(n)
        cg = eng.run(SEED, first, n)
        assert bench_path(eng) <= eng.path_info(0), eng.path_info(0)
        res = harness.simulate(S, SEED, first, n, ["ofdm"])
        assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), (first, cg - res["err"])
        if first == 0:
            _check_mse(eng, res)
            eng.enable_mse(False)
    eng.set_option("mmse_ic", 0)        # the W contraction on the same realisations
    cw = eng.run(SEED, 128, 128)
    assert W_PATH <= eng.path_info(0), eng.path_info(0)
    assert np.abs(cw - res["err"]).sum() <= 8 * res["borderline"].sum(), cw - res["err"]
    eng.set_option("mmse_ic", 1)
    eng.set_batch(256)
    b = eng.bits_per_rep(0)
    assert b[0] == sc["n_data"] * sc["bits_per_symbol"] and b[1] == sc["considered"].sum() * sc["bits_per_symbol"]


@pytest.mark.parametrize("first", [(1 << 32) - 30, (1 << 40) + 3])
def test_counts_at_far_realisation_indices_match_oracle(ofdm, first):
    """Realisations far from 0: the Philox counter carries the realisation index
    as two 32-bit words, so 2^32 - 30 .. 2^32 + 33 crosses the low word's wrap
    inside one wave (a 32-bit index anywhere on the path would alias rep 0..33),
    and 2^40 + 3 sits past it; every stream (bits, pilots, THETA / PHI, noise)
    against the oracle, through the bench kernels."""
    S, eng, mm = ofdm
    eng.set_batch(64)
    try:
        cg = eng.run(SEED, first, 64)
        assert bench_path(eng) <= eng.path_info(0), eng.path_info(0)
        res = harness.simulate(S, SEED, first, 64, ["ofdm"])
        assert res["err"].sum() > 0
        assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), cg - res["err"]
        # the oracle keys every stream by the 64-bit index, so this also shows
        # the counts are not those of the low word's realisations
        if first >> 32:
            assert not np.array_equal(cg, eng.run(SEED, first & 0xFFFFFFFF, 64))
    finally:
        eng.set_batch(256)


@pytest.mark.parametrize("n_iter", [1, 2, 3, 6])
def test_ic_iteration_counts_match_oracle(n_iter):
    """Other IC iteration counts (script:479 `NrIterations`): the estimator
    variant switch (W0 up to niter / 2, script:497-501) against the oracle
    through the bench kernels and the W contraction, counts of every stage, and
    one unit traced per element."""
    S = harness.setup("default", schemes=("ofdm",), snr_db=[15.0, 35.0], n_iter=n_iter)
    eng = harness.engine(S, batch=64)
    cg = eng.run(SEED, 0, 64)
    path = eng.path_info(0)
    assert bench_path(eng) <= path, path
    eng.set_option("mmse_ic", 0)                # the W contraction, per-stage launches
    assert np.array_equal(eng.run(SEED, 0, 64), cg)
    assert W_PATH <= eng.path_info(0), eng.path_info(0)
    eng.set_option("mmse_ic", 1)
    res = harness.simulate(S, SEED, 0, 64, ["ofdm"])
    assert cg.shape == res["err"].shape
    assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), cg - res["err"]
    tr = {}
    harness.simulate(S, SEED, 3, 1, ["ofdm"], trace=tr)
    for k in range(2):
        assert _check_trace(eng.trace_unit(0, SEED, 3, k), tr["units"][k], "niter %d snr %d" % (n_iter, k)) == n_iter + 1
    eng.close()


# ---------------------------------------------------------------------------
# C3 / C4: FBMC-OQAM with auxiliary-symbol and data-spreading precoders
# (two SNR points keep the literal oracle's run time in check)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module", params=["fbmc_aux", "fbmc_cod"])
def fbmc(request):
    S = harness.setup("default", schemes=(request.param,), snr_db=[15.0, 35.0])
    eng = harness.engine(S, batch=256)
    mm = harness.oracle_mmse(S, request.param)
    yield request.param, S, eng, mm
    eng.close()


def test_fbmc_estimator_and_trace(fbmc):
    name, S, eng, mm = fbmc
    _check_W(eng, mm, 2)
    tr = {}
    harness.simulate(S, SEED, 9, 1, [name], trace=tr)
    for k in range(2):
        g = eng.trace_unit(0, SEED, 9, k)
        u = tr["units"][k]
        ns = _check_trace(g, u, "%s snr %d" % (name, k))
        for st in range(1, ns):        # unfused perfect-CSI passes: y_perf of every row
            np.testing.assert_allclose(g["yperf"][st], u["yperf"][st], rtol=0, atol=1e-9)
    # the row-tile GEMM contraction and the polyphase perfect-CSI passes ran
    assert {"wrow3", "pic_poly"} <= eng.path_info(0), eng.path_info(0)


def test_fbmc_error_counts(fbmc):
    name, S, eng, mm = fbmc
    eng.enable_mse()
    cg = eng.run(SEED, 64, 64)
    res = harness.simulate(S, SEED, 64, 64, [name])
    assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), (name, cg - res["err"])
    _check_mse(eng, res)
    err64, pw64 = eng.mse()
    # ragged runs (padding lanes of a partial wave count nothing, neither in the
    # counters nor in the MSE sums of any FBMC stage kernel): the same 64
    # realisations as 25 + 39, and as 1 + 63
    for a, b in ((25, 39), (1, 63)):
        eng.enable_mse()                                # resets the sums
        np.testing.assert_array_equal(eng.run(SEED, 64, a) + eng.run(SEED, 64 + a, b), cg)
        err, pw = eng.mse()
        np.testing.assert_allclose(err, err64, rtol=1e-12, atol=0)
        np.testing.assert_allclose(pw, pw64, rtol=1e-12, atol=0)
    eng.enable_mse(False)


def test_fbmc_counts_across_the_counter_word_wrap(fbmc):
    """FBMC's kernels (TX precoding, polyphase perfect-CSI passes, the W
    contraction) at realisations 2^32 - 30 .. 2^32 + 33 against the oracle:
    the realisation index crosses the Philox counter's low-word wrap."""
    name, S, eng, mm = fbmc
    first = (1 << 32) - 30
    cg = eng.run(SEED, first, 64)
    res = harness.simulate(S, SEED, first, 64, [name])
    assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), (name, cg - res["err"])


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
    S = harness.setup("default", snr_db=[25.0])
    joint = harness.engine(S, batch=128)
    cj = joint.run(SEED, 0, 128)
    joint.close()
    for i, name in enumerate(S.schemes):
        e = harness.engine(S, schemes=(name,), batch=128)
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


def test_batch_invariance_at_full_and_largest_batches():
    """The bench's own batch (65 536 realisations x 7 SNR points) and larger:
    every count of [0, 262144) is the same at device batch 131 072, 65 536 and
    8 192 through the bench kernels.  At 262 144 the realisation-major tap
    buffer (ntap N R x 16 B) passes 4 GB, past k_pic_fft's 32-bit buffer view,
    so the engine falls back to the W contraction and the banded perfect-CSI
    passes (pic_fft_ok / mmse_stages_ok) instead of overflowing; that path
    gives the same counts up to the oracle's borderline decisions (none
    expected)."""
    S = harness.setup("default", schemes=("ofdm",))
    n = 262144
    ref = None
    for batch in (131072, 65536, 8192, 262144):
        eng = harness.engine(S, batch=batch)
        try:
            c = eng.run(SEED, 0, n)
            path = eng.path_info(0)
        finally:
            eng.close()
        assert c.sum() > 0
        if batch == 262144:
            assert "pic_fft" not in path and "mic_stages" not in path and "wpair3_fused" in path, path
            d = np.abs(c - ref)
            assert d.sum() <= 8, (int(d.sum()), int(ref.sum()))
            continue
        assert BENCH_BASE | {"mic_lr"} <= path, (batch, path)
        if ref is None:
            ref = c
        else:
            np.testing.assert_array_equal(c, ref, err_msg=str(batch))


def test_any_repetition_count(ofdm):
    """dsce_run takes the script's own NrRepetitions as is — 25 (script:19) and
    1000 (the paper's, script:44) — not only multiples of one wavefront: the
    padding realisations of a partial wave are simulated but counted nowhere.
    25 realisations against the oracle (counts and MSE sums); 1000 against
    every split and batch size; 0 realisations add nothing."""
    S, eng, _ = ofdm
    eng.enable_mse()
    c25 = eng.run(SEED, 0, 25)
    assert bench_path(eng) <= eng.path_info(0), eng.path_info(0)
    res = harness.simulate(S, SEED, 0, 25, ["ofdm"])
    assert np.abs(c25 - res["err"]).sum() <= 8 * res["borderline"].sum(), c25 - res["err"]
    _check_mse(eng, res)
    eng.enable_mse(False)
    assert not eng.run(SEED, 0, 0).any()
    a = eng.run(SEED, 0, 1000)
    np.testing.assert_array_equal(eng.run(SEED, 0, 25) + eng.run(SEED, 25, 975), a)
    np.testing.assert_array_equal(eng.run(SEED, 0, 999) + eng.run(SEED, 999, 1), a)
    eng.set_batch(64)
    np.testing.assert_array_equal(sum(eng.run(SEED, 25 * k, 25) for k in range(40)), a)
    np.testing.assert_array_equal(eng.run(SEED, 0, 1000), a)
    eng.set_batch(256)
    # the W-contraction path of the same scheme masks its padding lanes too
    eng.set_option("mmse_ic", 0)
    np.testing.assert_array_equal(eng.run(SEED, 0, 25) + eng.run(SEED, 25, 975), eng.run(SEED, 0, 1000))
    c25w = eng.run(SEED, 0, 25)
    eng.set_option("mmse_ic", 1)
    assert np.abs(c25w - res["err"]).sum() <= 8 * res["borderline"].sum()


def test_structured_ofdm_guard_rejects_what_the_threshold_changes():
    """build_mic keeps the structured MMSE IC (k_mic_pilot / k_mic_data: D_hat = Q' H_hat G)
    only if Q' H_hat G reproduces EVERY entry of the thresholded W — the
    off-diagonal entries the IC subtraction uses (script:482-484), not just
    diag(D_hat).  At ZeroThreshold 1e-5 (instead of the script's 1e-8,
    script:34) the diagonal still agrees (oracle: 0 x tolerance) but the
    entries the threshold drops off the diagonal do not (1.04 x): the engine
    must fall back to the W contraction and still equal the oracle's literal
    thresholded W."""
    from types import SimpleNamespace
    S = SimpleNamespace(**vars(harness.setup("default", schemes=("ofdm",))))
    S.zero_threshold = 1e-5
    eng = harness.engine(S, batch=64)
    cg = eng.run(SEED, 0, 64)
    path = eng.path_info(0)
    assert "mic_fft" not in path and "wpair3_fused" in path, path
    res = harness.simulate(S, SEED, 0, 64, ["ofdm"])
    assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), cg - res["err"]
    eng.close()
    # the script's threshold keeps the structured path: Q' H_hat G equals the
    # thresholded W to rounding (oracle, tools/threshold_study.py: <= 7e-13
    # absolute at max|W| 0.41-0.59)
    S.zero_threshold = 1e-8
    eng = harness.engine(S, batch=64, options={"mic_lr": 1})
    eng.run(SEED, 0, 64)
    assert "mic_fft" in eng.path_info(0)
    chk = eng.structured_check(0)
    # the bar is rounding level: max(1e-11, 4e-16 kappa(R)) max|W| per slice (GPU, C2:
    # dev 5.9e-12 at max|W| 0.59, kappa ~1e5: bars of 1e-11 .. 5e-11; capped at 1e-9)
    assert 0.0 <= chk["ratio"] <= 1.0 and chk["dev"] <= chk["rtol"] * chk["wmax"], chk
    assert 1e-11 <= chk["rtol"] <= 1e-9, chk
    # the low-rank form of the tap operator reproduces Bv to rounding and is used
    assert chk["lr"] and 0.0 <= chk["lr_ratio"] <= 1.0 and 0.0 <= chk["lr_resid"] < 1e-10, chk
    assert "mic_lr" in eng.path_info(0)
    eng.close()


def test_structured_ofdm_guard_is_at_rounding_level():
    """a guard at the threshold (r02-r03: thr + 1e-9 max|W|)
    accepts any geometry whose only deviation is the W threshold itself, since a
    zeroed entry has |W_s| < thr by definition.  At ZeroThreshold 1e-6 the
    thresholds of script:287-289 / :306-308 zero C2 entries of magnitude
    1e-7..1e-6 (oracle: max |W_thr - W_s| = 0.94 thr, tools/threshold_study.py),
    which the old guard accepted (deviation < thr) and the rounding-level guard
    (min(1e-9, max(1e-11, 4e-16 kappa(R))) max|W| per slice, dsce_structured_check) must
    reject: the W contraction runs and
    the counts equal the oracle's literal thresholded W."""
    from types import SimpleNamespace
    S = SimpleNamespace(**vars(harness.setup("default", schemes=("ofdm",))))
    S.zero_threshold = 1e-6
    eng = harness.engine(S, batch=64)
    chk = eng.structured_check(0)
    # the old guard would have accepted: every deviation is below the threshold
    assert 0.0 < chk["dev"] < S.zero_threshold, chk
    # ... but it is far above rounding
    assert chk["ratio"] > 1e2 and 1e-11 <= chk["rtol"] <= 1e-9, chk
    cg = eng.run(SEED, 0, 64)
    path = eng.path_info(0)
    assert "mic_fft" not in path and "wpair3_fused" in path, path
    res = harness.simulate(S, SEED, 0, 64, ["ofdm"])
    assert np.abs(cg - res["err"]).sum() <= 8 * res["borderline"].sum(), cg - res["err"]
    eng.close()


def test_psace_mmse_plugin(ofdm):
    """The 'MMSE' method of PilotSymbolAidedChannelEstimation (a stub in the
    reference, PSACE.m:110-111/:128-129) served by the engine equals
    diag(sum_p W_p hP_p) of script:417-428."""
    from dsce.estimation import PilotSymbolAidedChannelEstimation
    S, eng, mm = ofdm
    sc = S.schemes["ofdm"]
    LK = sc["G"].shape[1]
    pm = np.zeros(LK)
    pm[sc["pilot_pos"]] = 1
    est = PilotSymbolAidedChannelEstimation("Custom", pm.reshape(S.L, LK // S.L, order="F"), "MMSE")
    est.set_mmse_engine(eng, 0, 3)
    rng = np.random.default_rng(4)
    ls = rng.standard_normal(16) + 1j * rng.standard_normal(16)
    got = est.ChannelInterpolation(ls)
    W3 = mm["W"][:, 3].reshape(LK, LK, 16, order="F")
    ref = np.diag((W3 * ls[None, None, :]).sum(axis=2))
    np.testing.assert_allclose(got.reshape(-1, order="F"), ref, rtol=0, atol=1e-11 * np.abs(ref).max())


def test_w_band_trim_is_bit_exact():
    """Trimming W to its non-zero column extent (after the 1e-8 threshold) skips
    exact zeros only: counts are bit-identical and the contracted work shrinks."""
    S = harness.setup("default", schemes=("fbmc_aux",), snr_db=[20.0, 40.0])
    full = harness.engine(S, batch=128, options={"wtrim": 0})
    trim = harness.engine(S, batch=128)
    np.testing.assert_array_equal(full.run(SEED, 0, 128), trim.run(SEED, 0, 128))
    for k in range(2):
        np.testing.assert_array_equal(full.W(0, k, 0), trim.W(0, k, 0))
    assert trim.work_model(0)[0] < 0.7 * full.work_model(0)[0]
    full.close()
    trim.close()


@pytest.mark.parametrize("name", ["ofdm", "fbmc_aux"])
def test_stage_variants_agree(name):
    """Every kernel option (dsce_set_option) gives identical counts on 1024
    realisations: the fused select-mode stage vs the 3-kernel split path (any
    row-block size), perfect-CSI detection fused into the second pass or not,
    XCD-aware work order on/off, SNR-chunked receiver, the VALU contraction
    (the fallback without pair tiles), the MMSE stage as its own kernels
    instead of fused into the contraction, the perfect-CSI chain as
    per-iteration passes instead of k_pic_fft, one realisation per Jakes wave,
    the W contraction instead of the structured MMSE IC (k_mic_pilot /
    k_mic_data), the Jakes taps at every sample instead of only where a Q^H row
    reads them (and the anchor / moment fallbacks), TX / channel / noisy Q^H as
    banded passes instead of k_txrx_fft, the TX symbols one realisation per
    lane (k_tx_symbols, the fallback for non-row-local precoders), k_pic_fft's
    4-point network by DPP instead of on the matrix cores (and k_mic_pilot /
    k_mic_data's, with the tap GEMM's exchange by ds_bpermute), the tap GEMM
    Bv hP instead of the low-rank operator T_k Z (mic_lr 0), the perfect-CSI
    passes banded instead of polyphase (pic_poly 0; FBMC) and polyphase for
    OFDM too (pic_poly 1 with pic_chain 0: OFDM's chain is otherwise
    k_pic_fft), the FBMC contraction as k_wpair3's pair tiles instead of
    k_wrow3's row-tile GEMM (wrow 0).  (pic_skip and ic_streams 2 / 3, measured
    neutral, were retired in r06.)"""
    S = harness.setup("default", schemes=(name,), snr_db=[10.0, 25.0, 40.0])
    eng = harness.engine(S, batch=512)
    eng.set_option("stage_split", 1)
    ref = eng.run(SEED, 0, 1024)
    assert "stage_split" in eng.path_info(0)
    eng.set_option("stage_split", 0)
    for rb in (4, 8, 16):
        eng.set_option("stage_rb", rb)
        np.testing.assert_array_equal(eng.run(SEED, 0, 1024), ref, err_msg=str(rb))
    eng.set_option("stage_rb", 8)
    variants = ({"pfuse": 0}, {"xcd": 0}, {"snr_chunk": 2},
                {"wcontract_valu": 1}, {"fuse_stage": 0}, {"pic_chain": 0},
                {"noise_fuse": 0}, {"jakes_rpw": 1}, {"mmse_ic": 0},
                {"jakes_win": 0}, {"txrx_fft": 0}, {"mmse_ic": 0, "fuse_stage": 0, "pic_chain": 0},
                {"jakes_mom": 1}, {"jakes_mom": 0}, {"tx_rows": 0}, {"pic_net": 0},
                {"pic_net": 0, "mmse_ic": 0}, {"mic_net": 0}, {"mic_net": 2}, {"mic_net": 3},
                {"mic_net": 0, "pic_net": 0}, {"mic_lr": 0}, {"mic_lr": 0, "mic_net": 3},
                {"pic_poly": 0}, {"pic_poly": 1, "pic_chain": 0}, {"wrow": 0}, {"jakes_grp2": 0})
    for env in variants:
        old = {k: eng.get_option(k) for k in env}
        for k, v in env.items():
            eng.set_option(k, v)
        np.testing.assert_array_equal(eng.run(SEED, 0, 1024), ref, err_msg=str(env))
        for k, v in old.items():
            eng.set_option(k, v)
    eng.close()


def test_options_are_validated():
    from dsce.engine import DsceError, Engine
    eng = Engine()
    with pytest.raises(DsceError):
        eng.set_option("no_such_option", 1)
    with pytest.raises(DsceError):
        eng.set_option("stage_rb", 5)
    for retired in (1, 2):                      # k_pic_chain / k_pic_mfma, retired in r03
        with pytest.raises(DsceError):
            eng.set_option("pic_chain", retired)
    # the r01-r02 variants pruned in r03 (4M k_wpair, the per-stage k_mic_fft
    # path, the second stream): their options are gone
    for name in ("wpair_3m", "wda_3m", "streams", "qidx", "stage0_fft", "mic_mfma", "pilot_fft", "mic_yic",
                 "pilot_fuse", "mic2", "pic_skip", "ic_streams"):         # the last two retired in r06
        with pytest.raises(DsceError):
            eng.set_option(name, 0)
    assert eng.get_option("fuse_stage") == 1
    eng.close()


@pytest.mark.parametrize("name", ["default", "c5", "paper"])
def test_tx_matrices_on_gpu_match_host_mirror(name):
    """Row f1: G and Q = GetRXMatrix' produced on the GPU in closed form equal
    the host mirror's L Modulation() calls (OFDM.m:184-218, FBMC.m:318-354)
    and the oracle's own restatement (oracle/setup.py)."""
    from dsce.configs import build_setup
    from dsce.engine import Engine
    S = build_setup(name, schemes=("fbmc_aux", "ofdm"))
    O = harness.setup(name, schemes=("ofdm",))
    eng = Engine()
    for key in ("fbmc_aux", "ofdm"):
        sc = S.schemes[key]
        G, Q = eng.tx_matrices(sc.extras["modulation"])
        scale = np.abs(sc.G).max()
        np.testing.assert_allclose(G, sc.G, rtol=0, atol=1e-13 * scale, err_msg=key)
        np.testing.assert_allclose(Q, sc.Q, rtol=0, atol=1e-13 * np.abs(sc.Q).max(), err_msg=key)
        if key == "ofdm":
            np.testing.assert_allclose(G, O.schemes["ofdm"]["G"], rtol=0, atol=1e-13 * scale)
    eng.close()


def test_setup_with_gpu_tx_matrices_gives_the_same_counts():
    """Row f1 wired into the setup: build_setup(tx=gpu_tx()) takes G and Q from
    dsce_tx_matrices; the engine built from it counts exactly like the one
    built from the host mirror's G / Q (C2 OFDM and FBMC auxiliary, 256
    realisations, 2 SNR points)."""
    from dsce.configs import build_setup
    from dsce.engine import build_engine, gpu_tx
    for sc in ("ofdm", "fbmc_aux"):
        a = build_setup("default", schemes=(sc,), snr_db=[15.0, 35.0])
        b = build_setup("default", schemes=(sc,), snr_db=[15.0, 35.0], tx=gpu_tx())
        np.testing.assert_allclose(b.schemes[sc].G, a.schemes[sc].G, rtol=0, atol=1e-13 * np.abs(a.schemes[sc].G).max())
        ea, eb = build_engine(a, batch=256), build_engine(b, batch=256)
        np.testing.assert_array_equal(ea.run(SEED, 0, 256), eb.run(SEED, 0, 256))
        ea.close()
        eb.close()


def test_transmission_matrix_probe_matches_oracle():
    """SURVEY §8(b)'s probe dsce_transmission_matrix: D = Q' H G of one
    realisation (script:381-393) from the engine's operators and the run's
    Jakes realisation equals the oracle's literal product (sparse
    GetConvolutionMatrix H, refsim.conv_matrix) to 1e-12 max|D|, for OFDM and
    FBMC and realisations at several lanes of the Jakes batch; its diagonal is
    the perfect-CSI one-tap channel h the hot path forms without D
    (dsce_trace_unit_ex's h_perfect)."""
    S = harness.setup("default", schemes=("ofdm", "fbmc_aux"), snr_db=[25.0])
    eng = harness.engine(S, batch=256)
    ch = S.chan
    try:
        for sid, name in enumerate(S.schemes):                 # harness.engine's scheme order
            sc = S.schemes[name]
            for rep in (3, 64, 1 << 33):
                D = eng.transmission_matrix(sid, SEED, rep)
                ir = refsim.jakes_ir(SEED, rep, S.N, ch["dt"], ch["pdp_norm"], ch["idx_taps"], ch["fD"], ch["paths"])
                H = refsim.conv_matrix(ir, ch["pdp"], S.N)
                Do = sc["Q"].conj().T @ (H @ sc["G"])
                scale = np.abs(Do).max()
                np.testing.assert_allclose(D, Do, rtol=0, atol=1e-12 * scale, err_msg="%s rep %d" % (name, rep))
                h = eng.trace_unit(sid, SEED, rep, 0)["h"]
                np.testing.assert_allclose(h, np.diag(D), rtol=0, atol=1e-12 * scale, err_msg=name)
    finally:
        eng.close()
