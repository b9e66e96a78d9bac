"""CPU: the MMSE one-tap's batch inversion (kernels_mc.hip mic_detect, r05)
restated in NumPy.  Six rows' scI / |hd|^2 from ONE reciprocal (prefix
products, one reciprocal, two products per row back) agree with the per-row
quotients to a few ulp over the dynamic range a channel estimate spans, and
the fallback bound [2^-160, 2^160] on every factor (r06, ADVICE r05: r05
bounded only the full product) catches the lanes whose product or any prefix
would over- or underflow (a zero or vanishing estimate)."""
import numpy as np

LO, HI = 2.0 ** -160, 2.0 ** 160


def factor_ok(nn):
    """mic_detect's test: max over the rows of hi(nn) - (863 << 20) as unsigned
    < 320 << 20, i.e. every exponent field in [1023 - 160, 1023 + 160)."""
    hi = (np.asarray(nn, dtype=np.float64).view(np.uint64) >> np.uint64(32)).astype(np.int64)
    ex = ((hi - ((1023 - 160) << 20)) & 0xFFFFFFFF).max()
    return bool(ex < (320 << 20))


def batch_inverse(nn, sc):
    """mic_detect's sequence for one lane: nn = |hd|^2 of its six rows (the
    degenerate lanes produce inf / NaN here as on the GPU, where the fallback
    then replaces them)."""
    with np.errstate(all="ignore"):
        return _batch_inverse(nn, sc)


def _batch_inverse(nn, sc):
    pp = np.cumprod(nn)
    inv = (1.0 / pp[5]) * sc
    out = np.empty(6)
    for a in range(5, 0, -1):
        out[a] = inv * pp[a - 1]
        inv *= nn[a]
    out[0] = inv
    ok = factor_ok(nn)
    assert ok == bool(np.all((nn >= LO) & (nn < HI)))        # the integer test is the interval
    return out, ok


def test_batch_inverse_matches_per_row_quotients():
    rng = np.random.default_rng(5)
    worst = 0.0
    for _ in range(20000):
        # |h|^2 of a Rayleigh tap spans decades: exponential power, deep fades included
        nn = rng.exponential(1.0, 6) * 10.0 ** rng.uniform(-6, 3, 6)
        sc = rng.uniform(0.5, 4.0)
        got, ok = batch_inverse(nn, sc)
        assert ok
        ref = sc / nn
        worst = max(worst, float(np.max(np.abs(got / ref - 1.0))))
    # 6 products + 1 reciprocal + 2 products back: a few ulp (the slicer's
    # borderline bar is 1e-9)
    assert worst < 16 * np.finfo(float).eps, worst


def test_fallback_bound_catches_vanishing_and_huge_products():
    sc = 1.0
    assert not batch_inverse(np.array([1.0, 1.0, 0.0, 1.0, 1.0, 1.0]), sc)[1]
    assert not batch_inverse(np.full(6, 1e-60), sc)[1]      # product 1e-360 underflows
    assert not batch_inverse(np.full(6, 1e60), sc)[1]       # 1e360 overflows
    assert batch_inverse(np.full(6, 1e-40), sc)[1]          # 1e-240 is representable
    assert not batch_inverse(np.array([1.0, np.inf, 1.0, 1.0, 1.0, 1.0]), sc)[1]
    assert not batch_inverse(np.array([1.0, np.nan, 1.0, 1.0, 1.0, 1.0]), sc)[1]
    # a prefix in the denormals while the full product is back in range: r05's
    # bound on pp[5] alone accepted this lane (and lost precision)
    nn = np.array([1e-160, 1e-160, 1e200, 1e100, 1.0, 1.0])
    assert 2.0 ** -1000 < np.prod(nn) < 2.0 ** 1000 and not batch_inverse(nn, sc)[1]
