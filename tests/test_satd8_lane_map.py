"""CPU: the lane form of HadamardSAD8x8 that the EPZS server's refinement runs
(csrc/jmme_refine_dev.h tile_satd8: one difference row per lane, the row's
8-point Hadamard in the lane, then the column transform across the 8 lanes by
DPP -- the mirror partner 7 - r first, then r ^ 1, then r ^ 2) restated in numpy
and held against JM 18.5's own HadamardSAD8x8 records (tests/golden/tq_jm.npz,
the restatement oracle/tq_oracle.c pinned by test_tq_oracle_golden.py).
Also pins why the order matters: with the mirror stage last the column map is
not a (signed, permuted) Hadamard and the sums differ."""
import os

import numpy as np
import pytest

import oracle_lib as ol

GOLD = os.path.join(os.path.dirname(__file__), "golden", "tq_jm.npz")


def _rows_wht(d):
    d = d.copy()
    h = 1
    while h < 8:
        for i in range(8):
            if not i & h:
                a, b = d[..., i].copy(), d[..., i + h].copy()
                d[..., i], d[..., i + h] = a + b, a - b
        h <<= 1
    return d


# one butterfly across the lanes of a group: partner(r), and whether lane r keeps a + b (else b - a)
MIRROR = (lambda r: 7 - r, lambda r: r < 4)
XOR1 = (lambda r: r ^ 1, lambda r: not r & 1)
XOR2 = (lambda r: r ^ 2, lambda r: not r & 2)


def _lane_satd8(diff, stages):
    """diff: (n, 8, 8) rows; the sum tile_satd8 forms, (s + 2) >> 2"""
    d = _rows_wht(diff.astype(np.int64))
    for part, low in stages:
        n = d.copy()
        for r in range(8):
            p = part(r)
            n[:, r] = d[:, r] + d[:, p] if low(r) else d[:, p] - d[:, r]
        d = n
    return (np.abs(d).sum(axis=(1, 2)) + 2) >> 2


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_lane_map_equals_jm_hadamard_sad8x8(gold):
    diff = gold["satd8x8_in"].reshape(-1, 8, 8)
    want = gold["satd8x8_out"][:, 0]
    np.testing.assert_array_equal(_lane_satd8(diff, (MIRROR, XOR1, XOR2)), want)


def test_lane_map_on_random_extremes():
    rng = np.random.default_rng(5)
    diff = rng.integers(-255, 256, (2000, 8, 8))
    diff[:100] = rng.choice([-255, 255], (100, 8, 8))   # the largest sums
    want = ol.tq_satd(diff.reshape(len(diff), 64), 8)
    np.testing.assert_array_equal(_lane_satd8(diff, (MIRROR, XOR1, XOR2)), want)


def test_mirror_last_is_not_a_hadamard():
    rng = np.random.default_rng(6)
    diff = rng.integers(-255, 256, (200, 8, 8))
    want = ol.tq_satd(diff.reshape(len(diff), 64), 8)
    assert not np.array_equal(_lane_satd8(diff, (XOR1, XOR2, MIRROR)), want)
