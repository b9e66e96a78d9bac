"""ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never by the product path).

Counter-based random streams shared by the CPU oracle and the HIP engine
(spec: include/dsce.h "Random streams").  The reference draws from MATLAB's
global mt19937ar/Ziggurat state (FastFading.m:227,:233; script:355-357,
:365-367, :399), which cannot be reproduced offline (SURVEY.md §7 hard part 1),
so "identical RNG seeds" means identical Philox4x32-10 streams here and on
the GPU, in the reference's draw order and shapes.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

STREAM_THETA = 1
STREAM_PHI = 2
STREAM_BITS = 3
STREAM_PILOTS = 4
STREAM_NOISE = 5


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11).  All inputs uint32 arrays
    (broadcastable); returns four uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    for r in range(10):
        p0 = M0 * c0.astype(np.uint64)
        p1 = M1 * c2.astype(np.uint64)
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & MASK32).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & MASK32).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        if r < 9:
            k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def _block(seed, rep, stream, sub, idx):
    seed = int(seed)
    rep = int(rep)
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    c1 = np.uint32(rep & 0xFFFFFFFF)
    c2 = np.uint32((rep >> 32) & 0xFFFFFFFF)
    c3 = np.uint32(((stream & 0xFFFF) << 16) | (sub & 0xFFFF))
    return philox4x32_10(np.asarray(idx, dtype=np.uint32), c1, c2, c3, k0, k1)


def u53(a, b):
    """53-bit uniform double in [0, 1) from two 32-bit words."""
    return ((a >> np.uint32(5)).astype(np.float64) * 67108864.0 + (b >> np.uint32(6)).astype(np.float64)) \
        * (1.0 / 9007199254740992.0)


def uniforms(seed, rep, stream, sub, n):
    """n uniforms; element e comes from counter e//2, words (0,1) if e even else (2,3)."""
    j = np.arange((n + 1) // 2, dtype=np.uint32)
    w0, w1, w2, w3 = _block(seed, rep, stream, sub, j)
    u = np.empty(2 * j.size)
    u[0::2] = u53(w0, w1)
    u[1::2] = u53(w2, w3)
    return u[:n]


def bits(seed, rep, sub, n):
    """n fair bits; bit i is bit (i & 31) of word (i >> 5) & 3 of counter i >> 7."""
    j = np.arange((n + 127) // 128, dtype=np.uint32)
    w = np.stack(_block(seed, rep, STREAM_BITS, sub, j), axis=1).reshape(-1)   # words in order
    i = np.arange(n)
    return ((w[i >> 5] >> (i & 31).astype(np.uint32)) & np.uint32(1)).astype(np.uint8)


def indices(seed, rep, sub, n, m):
    """n integers uniform on [0, m) (m a power of two): word j & (m-1); MATLAB randi(m) - 1."""
    if m & (m - 1):
        raise ValueError("modulation order must be a power of two")
    j = np.arange((n + 3) // 4, dtype=np.uint32)
    w = np.stack(_block(seed, rep, STREAM_PILOTS, sub, j), axis=1).reshape(-1)
    return (w[:n] & np.uint32(m - 1)).astype(np.int64)


def complex_normals(seed, rep, snr_index, n):
    """n complex samples (re, im) ~ N(0,1) each, Box-Muller from counter e:
    u1 = u53(w0,w1), u2 = u53(w2,w3); rad = sqrt(-2 log(1-u1));
    re = rad*cos(2*pi*u2), im = rad*sin(2*pi*u2)."""
    e = np.arange(n, dtype=np.uint32)
    w0, w1, w2, w3 = _block(seed, rep, STREAM_NOISE, snr_index, e)
    u1 = u53(w0, w1)
    u2 = u53(w2, w3)
    rad = np.sqrt(-2.0 * np.log(1.0 - u1))
    ang = (2.0 * np.pi) * u2
    return rad * np.cos(ang), rad * np.sin(ang)


def normal_pairs(seed, rep, stream, sub, counters):
    """Normal pairs (re, im) of the given counters, same Box-Muller as
    :func:`complex_normals` (time-invariant and discrete-Doppler channels)."""
    e = np.asarray(counters, dtype=np.uint32)
    w0, w1, w2, w3 = _block(seed, rep, stream, sub, e)
    u1 = u53(w0, w1)
    u2 = u53(w2, w3)
    rad = np.sqrt(-2.0 * np.log(1.0 - u1))
    ang = (2.0 * np.pi) * u2
    return rad * np.cos(ang), rad * np.sin(ang)
