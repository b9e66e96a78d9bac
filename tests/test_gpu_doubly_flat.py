"""GPU parity for FastFading's other realisation branches and for the
doubly-flat script (SimpleVersion_DoublyFlat.m, BASELINE config 1): the HIP
engine through the C-ABI against the CPU oracle on the same Philox streams,
and the perfect-CSI OFDM curve against the reference's own closed-form BEP
(Theory/BitErrorProbabilityDoublyFlatRayleigh.m, plotted by the script at
:180-192)."""
import numpy as np
import pytest

import harness  # noqa: F401  (sys.path)
from dsce.channel import FastFading
from dsce.engine import Engine
from oracle import refsim

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001
FD = 500 / 3.6 * 2.5e9 / 2.998e8


def _channel_engine(ff):
    eng = Engine(0)
    eng.set_channel(ff)
    return eng


@pytest.mark.parametrize("model", ["Discrete-Jakes", "Discrete-Uniform"])
def test_discrete_doppler_ir_matches_oracle(model):
    """k_discrete (direct sum over the Doppler bins) vs the literal IFFT of
    FastFading.m:203-221, C2 grid (N = 540, nd = 2) and the paper grid
    (N = 7350, SR = 2.94 MHz, six taps)."""
    for sr, n, pdp in ((360e3, 540, "VehicularA"), (2.94e6, 7350, "VehicularA")):
        ff = FastFading(sr, pdp, n, FD, model, 200)
        assert ff.UseDiscreteDopplerSpectrum
        eng = _channel_engine(ff)
        try:
            for rep in (0, 3, 1 << 33):
                g = eng.channel_impulse_response(SEED, rep)
                o = refsim.discrete_ir(SEED, rep, n, sr, ff.PowerDelayProfileNormalized, ff.IndexDelayTaps, FD, model)
                np.testing.assert_allclose(g, o, rtol=0, atol=1e-12)
        finally:
            eng.close()


def test_time_invariant_ir_matches_oracle():
    """MaximumDopplerShift = 0 (FastFading.m:241-246): one tap set per
    realisation, repeated over the samples; also the discrete model at a
    velocity below half a Doppler bin (:153-156)."""
    for ff in (FastFading(360e3, "VehicularA", 540, 0.0, "Jakes", 200),
               FastFading(360e3, "Flat", 3780, 0.0, "Jakes", 1),
               FastFading(360e3, "VehicularA", 540, 200.0, "Discrete-Jakes", 200)):
        assert ff.MaximumDopplerShift == 0
        eng = _channel_engine(ff)
        try:
            for rep in (0, 5, 999):
                g = eng.channel_impulse_response(SEED, rep)
                o = refsim.static_ir(SEED, rep, ff.SamplesTotal, ff.PowerDelayProfileNormalized, ff.IndexDelayTaps)
                np.testing.assert_allclose(g, o, rtol=0, atol=1e-13)
        finally:
            eng.close()


def test_mmse_refuses_discrete_doppler():
    """The reference has no TimeCorrelation for 'Discrete-*' (FastFading.m:321-336)."""
    from dsce.configs import build_setup
    from dsce.engine import DsceError
    S = build_setup("default", schemes=("ofdm",))
    ff = FastFading(S.SR, "VehicularA", S.N, FD, "Discrete-Jakes", 200)
    eng = Engine(0)
    try:
        eng.set_channel(ff)
        eng.set_snr(S.pn_time, 4)
        eng.add_scheme(S.schemes["ofdm"])
        with pytest.raises(DsceError, match="discrete Doppler"):
            eng.build_mmse()
    finally:
        eng.close()


@pytest.fixture(scope="module")
def flat():
    from dsce.doubly_flat import DoublyFlatSim
    sim = DoublyFlatSim(batch=8192)
    yield sim
    sim.close()


def _oracle_schemes(S):
    out = []
    for n in ("fbmc_aux", "fbmc_cod", "ofdm"):
        sc = S.schemes[n]
        d = harness.product_scheme_dict(sc)
        d.update(noise_slot=sc.extras["noise_slot"], interp=sc.extras["interp"])
        out.append(d)
    return out


def test_doubly_flat_counts_match_oracle(flat):
    """All three schemes, interpolated and perfect CSI, 7 SNR points, 64
    realisations: identical bit-error counts up to borderline decisions."""
    S = flat.setup
    got = flat.run(SEED, 0, 64)
    ref = refsim.simulate_doubly_flat(SEED, 0, 64, S.N, _oracle_schemes(S), S.pn_time)
    diff = np.abs(got - ref["err"]).sum(axis=(1, 2))
    allowed = 8 * ref["borderline"]
    assert np.all(diff <= allowed), (got, ref["err"], ref["borderline"])
    assert got.sum() > 1000


def test_doubly_flat_counts_across_the_counter_word_wrap(flat):
    """The doubly-flat kernels at realisations 2^32 - 30 .. 2^32 + 33 (the
    Philox counter's realisation low word wraps inside the wave) against the
    oracle."""
    S = flat.setup
    first = (1 << 32) - 30
    got = flat.run(SEED, first, 64)
    ref = refsim.simulate_doubly_flat(SEED, first, 64, S.N, _oracle_schemes(S), S.pn_time)
    diff = np.abs(got - ref["err"]).sum(axis=(1, 2))
    assert np.all(diff <= 8 * ref["borderline"]), (got, ref["err"], ref["borderline"])
    assert got.sum() > 1000


@pytest.mark.parametrize("method", ["natural", "nearest"])
def test_doubly_flat_other_interpolations_match_oracle(method):
    """PSACE's other scatteredInterpolant methods (PSACE.m:74-76) on the same
    kernels: counts identical to the oracle with the same weights, 64
    realisations x 7 SNR points, all three schemes."""
    from dsce.configs import build_doubly_flat_setup
    from dsce.doubly_flat import DoublyFlatSim
    sim = DoublyFlatSim(build_doubly_flat_setup(interpolation=method), batch=64)
    try:
        S = sim.setup
        got = sim.run(SEED, 0, 64)
        ref = refsim.simulate_doubly_flat(SEED, 0, 64, S.N, _oracle_schemes(S), S.pn_time)
        diff = np.abs(got - ref["err"]).sum(axis=(1, 2))
        assert np.all(diff <= 8 * ref["borderline"]), (got, ref["err"])
        ls = np.random.default_rng(2).standard_normal(S.schemes["ofdm"].n_pilots) + 0j
        g = sim.engine.mmse_onetap(sim.sid["ofdm"], 0, ls)
        np.testing.assert_allclose(g, S.schemes["ofdm"].extras["psace"].ChannelInterpolation(ls).reshape(-1, order="F"),
                                   rtol=0, atol=1e-13)
    finally:
        sim.close()


def test_doubly_flat_interpolation_onetap_matches_psace(flat):
    """dsce_mmse_onetap on an interpolation scheme = PSACE.ChannelInterpolation."""
    S = flat.setup
    rng = np.random.default_rng(1)
    for name in ("fbmc_aux", "ofdm"):
        sc = S.schemes[name]
        ls = rng.standard_normal(sc.n_pilots) + 1j * rng.standard_normal(sc.n_pilots)
        g = flat.engine.mmse_onetap(flat.sid[name], 0, ls)
        ref = sc.extras["psace"].ChannelInterpolation(ls).reshape(-1, order="F")
        np.testing.assert_allclose(g, ref, rtol=0, atol=1e-13)


def test_doubly_flat_perfect_csi_matches_theory(flat):
    """OFDM 16-QAM with perfect CSI over the doubly-flat Rayleigh channel
    reproduces the closed-form BEP the script plots (:180-181) at 65536
    realisations per SNR point (statistical tolerance 4 %)."""
    S = flat.setup
    n = 65536
    counts = flat.run(SEED + 1, 0, n)
    ber = flat.ber(counts, n)
    q = S.schemes["ofdm"].const
    th = refsim.bit_error_probability_doubly_flat_rayleigh(S.snr_db, q.SymbolMapping, q.BitMapping)
    rel = np.abs(ber["OFDM perfect CSI"] / th - 1)
    assert np.all(rel < 0.04), (ber["OFDM perfect CSI"], th)
    # interpolated estimates lose against perfect CSI at every SNR point
    assert np.all(ber["OFDM"] > ber["OFDM perfect CSI"])
    assert np.all(ber["FBMC Coding"] > ber["FBMC perfect CSI"])
