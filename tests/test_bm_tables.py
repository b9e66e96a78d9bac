"""The device Box-Muller transform (kernels_mc.hip `normal_pair` / `noise_add`,
r05) restated step by step with exactly rounded FMAs (fractions), checked
against the random-stream spec as the oracle evaluates it (oracle/philox.py:
np.log / np.sqrt / np.cos / np.sin) and against 60-digit mpmath.  Also: the
committed tables (csrc/bm_tables.h) are the generator's output.

The spec is unchanged (Philox4x32-10, 53-bit uniforms, sqrt(-2 log(1 - u1))
cis(2 pi u2)); only the evaluation is table-driven, so the device pair may
differ from NumPy's by a few units in the last place — far inside every GPU
parity tolerance (traces 1e-10, IR 1e-12)."""
import os
import subprocess
import sys
from fractions import Fraction

import mpmath as mp
import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_bm_tables  # noqa: E402
from oracle import philox  # noqa: E402

LOGT = gen_bm_tables.log_table()
CIST = gen_bm_tables.cis_table()
TWO_PI = 6.283185307179586


def fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def hi_word(x):
    return int(np.array([x], dtype=np.float64).view(np.uint64)[0] >> np.uint64(32))


def with_hi(x, hi):
    bits = int(np.array([x], dtype=np.float64).view(np.uint64)[0])
    bits = (hi << 32) | (bits & 0xFFFFFFFF)
    return float(np.array([bits], dtype=np.uint64).view(np.float64)[0])


def one_minus_u53(a, b):
    return fma(-float(a >> 5), 2.0 ** -27, fma(-float(b >> 6), 2.0 ** -53, 1.0))


def m2log_unit(x):
    hi = hi_word(x)
    m = with_hi(x, (hi & 0x000FFFFF) | 0x3FE00000)
    invc, t = LOGT[(hi >> 13) & 127]
    ed = float((hi >> 20) - 1022)
    r = fma(m, invc, -1.0)
    p = -2.0 / 7.0
    for c in (1.0 / 3.0, -2.0 / 5.0, 0.5, -2.0 / 3.0, 1.0):
        p = fma(p, r, c)
    s1 = fma(ed, -1.3862943611198906, t)
    return s1 + fma(r, -2.0, (r * r) * p)


def sqrt_bm(a):
    a = max(a, 1e-300)
    y = float(1.0 / np.sqrt(a)) * (1.0 + 3e-8)   # v_rsq_f64 is approximate; the Newton steps fix it
    g, h = a * y, 0.5 * y
    e = fma(-h, g, 0.5)
    g, h = fma(g, e, g), fma(h, e, h)
    d = fma(-g, g, a)
    g = fma(d, h, g)
    d = fma(-g, g, a)
    return fma(d, h, g)


def cis_u53(a, b):
    tx, ty = CIST[a >> 24]
    th = fma(float((a >> 5) & 0x7FFFF), 2.0 ** -27 * TWO_PI, fma(float(b >> 6), 2.0 ** -53 * TWO_PI, -0.01227184630308513))
    t2 = th * th
    s = fma(th * t2, fma(t2, 1.0 / 120.0, -1.0 / 6.0), th)
    cm1 = t2 * fma(fma(t2, -1.0 / 720.0, 1.0 / 24.0), t2, -0.5)
    return fma(tx, cm1, fma(-ty, s, tx)), fma(ty, cm1, fma(tx, s, ty))


def device_pair(w0, w1, w2, w3):
    rad = sqrt_bm(m2log_unit(one_minus_u53(w0, w1)))
    c, s = cis_u53(w2, w3)
    return rad * c, rad * s


def test_tables_are_generated():
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_bm_tables.py"), "--check"], check=True)


def test_one_minus_u53_is_exact():
    for a, b in ((0, 0), (0xFFFFFFFF, 0xFFFFFFFF), (0x80000000, 0x40), (12345, 678910), (0xFFFFFFE0, 0)):
        assert one_minus_u53(a, b) == 1.0 - float(philox.u53(np.uint32(a), np.uint32(b)))


def test_log_accuracy_and_edges():
    mp.mp.dps = 40
    xs = [1.0, 1.0 - 2.0 ** -53, 0.5, 0.5 + 2.0 ** -53, 2.0 ** -53, 0.75, 0.999, 1.0 - 1e-9, 0.501, 0.25]
    xs += list(np.random.default_rng(3).uniform(0, 1, 400))
    for x in xs:
        got = m2log_unit(float(x))
        ref = float(-2 * mp.log(mp.mpf(float(x))))
        assert abs(got - ref) <= 2.5 * np.spacing(abs(ref)) + 1e-300, (x, got, ref)
    assert m2log_unit(1.0) == 0.0


def test_sqrt_is_correctly_rounded_on_samples():
    for a in list(np.random.default_rng(4).uniform(0, 74, 300)) + [0.5, 2.0, 73.6, 1e-12]:
        assert sqrt_bm(float(a)) == float(np.sqrt(a))


def test_cis_accuracy_at_interval_edges():
    mp.mp.dps = 40
    words = [(j << 24, 0) for j in range(0, 256, 17)] + [((j << 24) | 0xFFFFFF, 0xFFFFFFFF) for j in range(0, 256, 23)]
    for a, b in words:
        c, s = cis_u53(a, b)
        u2 = mp.mpf(int(a >> 5) * 2 ** 26 + int(b >> 6)) / 2 ** 53
        assert abs(c - float(mp.cos(2 * mp.pi * u2))) < 3e-16
        assert abs(s - float(mp.sin(2 * mp.pi * u2))) < 3e-16


def test_pairs_match_the_oracle_spec():
    """2000 noise pairs of the oracle's own stream: the device evaluation is
    within a few ulp of NumPy's (the oracle's cis(2 pi u2) itself rounds the
    angle: ~4e-16 absolute)."""
    e = np.arange(2000, dtype=np.uint32)
    w = philox._block(0x5EED, 7, philox.STREAM_NOISE, 3, e)
    re, im = philox.complex_normals(0x5EED, 7, 3, 2000)
    worst = 0.0
    for i in range(2000):
        dr, di = device_pair(*(int(x[i]) for x in w))
        worst = max(worst, abs(dr - re[i]), abs(di - im[i]))
    assert worst < 8e-15, worst


@pytest.mark.parametrize("u1_words", [(0, 0), (0xFFFFFFFF, 0xFFFFFFFF)])
def test_pair_extremes(u1_words):
    """u1 = 0 (radius 0: the device gives ~1e-150) and the largest u1 (radius
    sqrt(2 * 53 ln 2) = 8.57)."""
    dr, di = device_pair(u1_words[0], u1_words[1], 0x12345678, 0x9ABCDEF0)
    u1 = float(philox.u53(np.uint32(u1_words[0]), np.uint32(u1_words[1])))
    rad = np.sqrt(-2.0 * np.log(1.0 - u1))
    assert abs(np.hypot(dr, di) - rad) <= 4 * np.spacing(max(rad, 1e-300)) + 1e-149
