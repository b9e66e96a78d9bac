"""CPU: the DFT-24 factorisation the chain kernels use (k_pic_fft, k_mic_data,
DESIGN.md §2.0 / §2.0b), restated in NumPy and checked against numpy.fft.

Lane r (time quarter / frequency residue) of a unit holds the rows 4a + r.
Inverse: DFT-6 (sign +) per lane over a, then the 4-point step across the
quarters with the lane twiddle folded into A_m[i][k] = w^(6 i k + k m), so the
time sample 6 i + m lands on quarter i.  Forward: A_m[i][k] = s w^-(6 i k + i m)
across the time quarters k, then DFT-6 (sign -) per residue i: row 4 a + i.
These are the tables k_pic_fft / mic2_tables build (`amt`) and the products
mfma4_cmul forms per sample m on v_mfma_f64_4x4x4f64."""
import numpy as np

W = np.exp(2j * np.pi / 24)


def amt(direction, scale=1.0):
    a = np.zeros((6, 4, 4), complex)
    for m in range(6):
        for i in range(4):
            for k in range(4):
                e = (6 * i * k + (i if direction else k) * m) % 24
                v = W ** e
                a[m, i, k] = scale * np.conj(v) if direction else v
    return a


def test_inverse_network_is_idft24():
    rng = np.random.default_rng(1)
    u = rng.standard_normal(24) + 1j * rng.standard_normal(24)
    lanes = u.reshape(6, 4).T                              # lane r: rows 4a + r
    x = np.array([[np.sum(lanes[r] * np.exp(2j * np.pi * np.arange(6) * m / 6)) for m in range(6)]
                  for r in range(4)])                      # DFT-6, sign +
    A = amt(0)
    t = np.array([[A[m, i] @ x[:, m] for m in range(6)] for i in range(4)])   # quarter i, sample m
    np.testing.assert_allclose(t.reshape(24), np.fft.ifft(u) * 24, atol=1e-12)


def test_forward_network_is_dft24_with_the_output_scale():
    rng = np.random.default_rng(2)
    xt = rng.standard_normal(24) + 1j * rng.standard_normal(24)
    s = 0.3 - 0.7j                                         # the folded qs gs
    q = xt.reshape(4, 6)                                   # quarter k, sample m
    A = amt(1, s)
    p = np.array([[A[m, i] @ q[:, m] for m in range(6)] for i in range(4)])    # residue i, sample m
    X = np.array([[np.sum(p[i] * np.exp(-2j * np.pi * np.arange(6) * a / 6)) for a in range(6)]
                  for i in range(4)])                      # DFT-6, sign -
    got = np.zeros(24, complex)
    for i in range(4):
        got[4 * np.arange(6) + i] = X[i]
    np.testing.assert_allclose(got, s * np.fft.fft(xt), atol=1e-12)


def dft6_pfa(x, sign):
    """kernels_mc.hip dft6 (r05): Good-Thomas 6 = 2 x 3 with the DFT-3 rotation
    fused into FMAs; natural-order input, X[k] returned at position p6(k) =
    -k mod 6 (the order the kernels read it in)."""
    H = np.sqrt(3.0) / 2.0
    x = list(x)

    def dft3(a, b, c):
        t, d = b + c, b - c
        m = a - 0.5 * t
        return a + t, m + sign * 1j * H * d, m - sign * 1j * H * d

    x[0], x[2], x[4] = dft3(x[0], x[2], x[4])
    x[3], x[5], x[1] = dft3(x[3], x[5], x[1])
    for k2 in range(3):
        i0, i1 = 2 * k2, (2 * k2 + 3) % 6
        x[i0], x[i1] = x[i0] + x[i1], x[i0] - x[i1]
    return x


def test_prime_factor_dft6_and_its_output_order():
    rng = np.random.default_rng(3)
    for sign in (1, -1):
        u = rng.standard_normal(6) + 1j * rng.standard_normal(6)
        got = dft6_pfa(u, sign)
        ref = np.fft.ifft(u) * 6 if sign > 0 else np.fft.fft(u)
        np.testing.assert_allclose([got[(6 - k) % 6] for k in range(6)], ref, atol=1e-13)
