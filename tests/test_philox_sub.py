"""CPU: the split Philox evaluation of the device (dsce_common.h stream_pre /
stream_sub: round 0 formed once per (seed, rep, idx), nine rounds per
sub-stream, used by k_txrx_fft for the noise of every SNR point) restated in
integer arithmetic and checked against the random-stream spec as the oracle
evaluates it (oracle/philox.py, the full ten rounds per block).  ADVICE r05:
the first round's sub-stream dependence is c2' = hi(M0 idx) ^ c3 ^ k1."""
import numpy as np
import pytest

from oracle import philox

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
U32 = 0xFFFFFFFF


def rounds(c0, c1, c2, c3, k0, k1, r0):
    """Philox rounds r0..9 with the round-r0 keys (dsce_common.h philox_rounds)."""
    for _ in range(r0, 10):
        p0, p1 = M0 * c0, M1 * c2
        c0, c1, c2, c3 = (p1 >> 32) ^ c1 ^ k0, p1 & U32, (p0 >> 32) ^ c3 ^ k1, p0 & U32
        k0, k1 = (k0 + W0) & U32, (k1 + W1) & U32
    return c0, c1, c2, c3


def stream_pre(seed, rep, idx):
    """(n0, lo1, hk, lo0, k0', k1') of dsce_common.h stream_pre."""
    p0, p1 = M0 * idx, M1 * (rep >> 32)
    k0, k1 = seed & U32, seed >> 32
    return ((p1 >> 32) ^ (rep & U32) ^ k0, p1 & U32, (p0 >> 32) ^ k1, p0 & U32, (k0 + W0) & U32, (k1 + W1) & U32)


def stream_sub(pre, stream, sub):
    n0, lo1, hk, lo0, k0, k1 = pre
    return rounds(n0, lo1, hk ^ (((stream & 0xFFFF) << 16) | (sub & 0xFFFF)), lo0, k0, k1, 1)


@pytest.mark.parametrize("seed,rep,idx", [(0x5EED0002, 0, 0), (0x5EED0002, 77, 539), (0x5EED0005, 1 << 33, 1079),
                                           ((1 << 64) - 1, (1 << 64) - 1, U32), (0x123456789ABCDEF0, 12345, 7)])
def test_split_rounds_equal_the_ten_round_block(seed, rep, idx):
    pre = stream_pre(seed, rep, idx)
    for stream, sub in [(philox.STREAM_NOISE, k + 256 * g) for k in (0, 1, 6, 15, 255) for g in (0, 1, 3)] + \
            [(philox.STREAM_THETA, 0), (philox.STREAM_BITS, 2)]:
        got = stream_sub(pre, stream, sub)
        ref = philox._block(seed, rep, stream, sub, np.uint32(idx))
        assert got == tuple(int(x) for x in ref), (seed, rep, idx, stream, sub)
        # and the unsplit device block (stream_block) is the spec itself
        full = rounds(idx, rep & U32, rep >> 32, ((stream & 0xFFFF) << 16) | (sub & 0xFFFF), seed & U32, seed >> 32, 0)
        assert full == got
