"""CPU: k_ic_pair's block -> pass mapping (kernels_mc.hip, Opts::ic_streams 3)
restated.  The launch's grid is cut into 8-block groups; group G belongs to the
pilot pass iff floor((G + 1) P / (C + P)) > floor(G P / (C + P)) (P pilot
groups, C chain groups), and block x of a pass's g-th group gets the pass-local
index 8 g + x.  Every pass-local block must be produced exactly once, keep the
XCD (index mod 8) it has in the pass's own launch, and the pilot groups must be
spread evenly over the grid."""
import numpy as np
import pytest


def ic_pair_map(npic8, npil8):
    ng = npic8 + npil8
    b = np.arange(8 * ng, dtype=np.int64)
    G, x = b >> 3, b & 7
    q0 = G * npil8 // ng
    q1 = (G + 1) * npil8 // ng
    pil = q1 > q0
    local = np.where(pil, q0 * 8 + x, (G - q0) * 8 + x)
    return pil, local


@pytest.mark.parametrize("npic8,npil8", [(12544, 3584), (42, 12), (7, 2), (1, 1), (5, 0), (0, 3), (13, 11)])
def test_every_pass_block_once_on_its_xcd(npic8, npil8):
    pil, local = ic_pair_map(npic8, npil8)
    b = np.arange(pil.size)
    assert np.array_equal(np.sort(local[pil]), np.arange(8 * npil8))
    assert np.array_equal(np.sort(local[~pil]), np.arange(8 * npic8))
    assert np.all(local % 8 == b % 8)


def test_pilot_groups_spread_evenly():
    npic8, npil8 = 12544, 3584                  # C2: 14 symbol blocks x U / 64, U / 16 pilot blocks
    pil, _ = ic_pair_map(npic8, npil8)
    groups = pil[::8]
    idx = np.flatnonzero(groups)
    gaps = np.diff(idx)
    ng = npic8 + npil8
    # Bresenham: consecutive pilot groups are floor or ceil of ng / npil8 apart
    assert gaps.min() >= ng // npil8 and gaps.max() <= -(-ng // npil8)
