"""Results I/O and figures (dsce/results.py, row f3 of SURVEY §8): BER from
counters equals the reference's nanmean of per-realisation BERs, JSON/NPZ
round trip, and Figures 2-5 render (CPU only, synthetic counters)."""
import os

import numpy as np

import harness  # noqa: F401  (sys.path)
from dsce import results
from dsce.configs import build_setup


def _fake(S, names, n_rep, rng):
    shape = (len(names), 2, 2, len(S.snr_db), S.n_iter + 1)
    bits = np.array([[2560, 2000], [2752, 2100], [2560, 2300]])[:len(names)]
    per_rep = rng.integers(0, 200, size=(n_rep,) + shape)
    per_rep[:, :, :, 1] = np.minimum(per_rep[:, :, :, 1], per_rep[:, :, :, 0])
    return per_rep, bits


def test_ber_equals_mean_of_per_realisation_ber(tmp_path):
    S = build_setup("default")
    names = tuple(S.schemes)
    rng = np.random.default_rng(1)
    per_rep, bits = _fake(S, names, 5, rng)
    counts = per_rep.sum(axis=0)
    b = results.ber(counts, bits, 5)
    # script:577-631: nanmean over realisations of mean(bits ~= detected) per realisation
    ref = (per_rep / bits.reshape(1, len(names), 1, 2, 1, 1)).mean(axis=0)
    np.testing.assert_allclose(b, ref, rtol=1e-14)
    res = results.make(S, names, counts, bits, 5, 7)
    p = str(tmp_path / "run.json")
    results.save(p, res, npz=True)
    back = results.load(p)
    np.testing.assert_array_equal(back["counts"], counts)
    assert back["schemes"] == list(names) and back["n_repetitions"] == 5
    z = np.load(str(tmp_path / "run.npz"))
    np.testing.assert_array_equal(z["counts"], counts)
    np.testing.assert_allclose(results.curve(back, "ofdm", "mmse", "all"), b[names.index("ofdm"), 0, 0, :, -1])


def test_figures_render(tmp_path):
    S = build_setup("default")
    names = tuple(S.schemes)
    per_rep, bits = _fake(S, names, 3, np.random.default_rng(2))
    res = results.make(S, names, per_rep.sum(axis=0), bits, 3, 0)
    files = results.figures(res, str(tmp_path))
    assert sorted(os.path.basename(f) for f in files) == ["Figure2.png", "Figure3.png", "Figure4.png", "Figure5.png"]
    assert all(os.path.getsize(f) > 1000 for f in files)
