"""GPU: the polyphase perfect-CSI IC passes (option pic_poly; k_poly_syn /
k_poly_chan / k_poly_ana) against the CPU oracle and against
the banded passes they replace, for C3 / C4 (FBMC 24 x 30, StorePerfectIC
epilogue) and C5 (FBMC 48 x 30 and OFDM 48 x 14, whose row-local precoder
takes the StorePerfectDetect epilogue).  y_perf of every row and stage of a
traced unit within 1e-9 of the oracle's literal Q' H G (script:541-543), error
counts within the oracle's borderline decisions, and the two device paths on
the same realisations."""
import numpy as np
import pytest

import harness

pytestmark = pytest.mark.gpu

SEED = 0x5EED0006


def _trace_yperf(S, name, eng, rep, snrs, w_sparse=False):
    tr = {}
    harness.simulate(S, SEED, rep, 1, [name], trace=tr, w_sparse=w_sparse)
    for k in snrs:
        g = eng.trace_unit(0, SEED, rep, k)
        u = tr["units"][k]
        for st in range(1, S.n_iter + 1):
            rows = slice(None) if name != "ofdm" else S.schemes[name]["data_pos"]
            np.testing.assert_allclose(g["yperf"][st][rows], u["yperf"][st][rows], rtol=0, atol=1e-9,
                                       err_msg="%s snr %d stage %d" % (name, k, st))
            ok = (g["dec_p"][st] == u["dec_p"][st]) | (u["margin_p"][st] < 1e-9)
            assert ok.all(), (name, k, st)


@pytest.mark.parametrize("cfg,name", [("default", "fbmc_aux"), ("default", "fbmc_cod"), ("c5", "fbmc_aux"),
                                      ("c5", "ofdm")])
def test_poly_passes_match_oracle(cfg, name):
    snr = [15.0, 35.0] if cfg == "default" else [36.0]
    S = harness.setup(cfg, schemes=(name,), snr_db=snr)
    ws = cfg == "c5" and name != "ofdm"
    poly = harness.engine(S, batch=64, options={"pic_poly": 1})
    band = harness.engine(S, batch=64, options={"pic_poly": 0})
    cp = poly.run(SEED, 0, 64)
    assert "pic_poly" in poly.path_info(0) and "pic_passes" not in poly.path_info(0), poly.path_info(0)
    cb = band.run(SEED, 0, 64)
    assert "pic_passes" in band.path_info(0) and "pic_poly" not in band.path_info(0)
    res = harness.simulate(S, SEED, 0, 64, [name], w_sparse=ws)
    border = 8 * res["borderline"].sum()
    assert np.abs(cp - res["err"]).sum() <= border, (name, cp - res["err"])
    assert np.abs(cp - cb).sum() <= border, (name, cp - cb)
    _trace_yperf(S, name, poly, 5, range(len(snr)), w_sparse=ws)
    poly.close()
    band.close()


def test_poly_and_band_agree_at_scale():
    """C3 at the script's 7 SNR points, 2048 realisations: the polyphase and
    banded passes give the same counts up to decisions within rounding of a
    boundary (none expected at this size; at most 1e-5 of the perfect-CSI bits)."""
    S = harness.setup("default", schemes=("fbmc_aux",))
    poly = harness.engine(S, batch=1024, options={"pic_poly": 1})
    band = harness.engine(S, batch=1024, options={"pic_poly": 0})
    cp = poly.run(SEED, 0, 2048)
    cb = band.run(SEED, 0, 2048)
    assert "pic_poly" in poly.path_info(0)
    bits = poly.bits_per_rep(0)[0] * 2048
    assert np.abs(cp - cb).sum() <= 1e-5 * bits * cp[0, 1].size, np.abs(cp - cb).sum()
    # the MMSE branch does not depend on the perfect-CSI passes at all
    np.testing.assert_array_equal(cp[0, 0], cb[0, 0])
    poly.close()
    band.close()
