"""CPU: known-answer tests of the fractal restatement (oracle/fractal_oracle.c).

Parity of this path is UNPINNED (the thesis sources need a windows.h stand-in
to build, and no reproducible reference fixture exists -- DESIGN.md §4).  These
tests plant affine domain->range maps whose answer is known in closed form."""
import numpy as np
import pytest

import oracle_lib as ol

BLOCKS = [(16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4)]


def _texture(h, w, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 256, (h + 8, w + 8)).astype(np.float64)
    k = np.ones(3) / 3
    x = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, x)
    x = np.apply_along_axis(lambda c: np.convolve(c, k, "same"), 0, x)
    return np.clip(x[4:4 + h, 4:4 + w], 0, 255).astype(np.uint8)


@pytest.mark.parametrize("bsx,bsy", BLOCKS)
def test_planted_shift_and_scale(bsx, bsy):
    """range = 0.5 * domain(shifted by (3, -2)) + 40 exactly -> that shift wins with rms 0."""
    h, w = 96, 128
    ref = _texture(h, w, 1)
    dom = ref.astype(np.int32)
    org = np.zeros((h, w), np.uint8)
    # 0.5*d + 40 is exact when d is even: make the domain even
    ref = (dom & ~1).astype(np.uint8)
    shifted = np.roll(np.roll(ref.astype(np.int32), 2, axis=0), -3, axis=1)   # org(y,x) uses ref(y-2? see below)
    org = (shifted // 2 + 40).astype(np.uint8)
    # org[y, x] = ref[y - 2, x + 3] / 2 + 40  -> domain offset (+3, -2)
    bx, by = 48, 40
    out, xy = ol.fractal_search_batch(org, ref, 7, np.array([[bx, by, bsx, bsy]]))
    assert tuple(xy[0]) == (3, -2)
    assert out[0, 1] == 0.5
    # the fit is exact up to the offset: beta is the range mean quantised by
    # QUAN_A, so rms = n * (beta - mean)^2
    blk = org[by:by + bsy, bx:bx + bsx].astype(np.int64)
    n, mean = blk.size, blk.sum() / blk.size
    assert out[0, 2] == _quan(int(mean))
    assert out[0, 0] == pytest.approx(n * (out[0, 2] - mean) ** 2, rel=1e-9, abs=1e-6)


def _quan(x):
    b, c = int(np.fmod(x, 10)), int(x / 10)
    if 2 < b < 8:
        b = 5
    elif b > 7:
        b, c = 0, c + 1
    else:
        b = 0
    return c * 10 + b


def test_compute_rms_flat_domain_and_rejection():
    org = np.full((32, 32), 100, np.uint8)
    ref = np.full((32, 32), 7, np.uint8)
    lib = ol.load_fractal()
    import ctypes
    a, b = ctypes.c_double(), ctypes.c_double()
    rms = lib.fro_compute_rms(org.ctypes.data, ref.ctypes.data, 32, 0, 0, 4, 4, 4, 4, ctypes.byref(a), ctypes.byref(b))
    assert a.value == 0.0 and b.value == 100.0 and rms == 0.0       # det == 0 -> alpha = 0, beta = mean
    # anti-correlated steep map: alpha < MIN_ALPHA -> rejected (1e30)
    ref2 = np.tile(np.array([0, 100, 0, 100], np.uint8), (32, 8))
    org2 = np.tile(np.array([255, 0, 255, 0], np.uint8), (32, 8))
    rms = lib.fro_compute_rms(org2.ctypes.data, ref2.ctypes.data, 32, 0, 0, 0, 0, 4, 4, ctypes.byref(a), ctypes.byref(b))
    assert rms == 1e30 and a.value == -2.5   # a = -255: QUAN_A zeroes negative units digits -> -250


def test_quan_a_rounding_through_beta():
    """beta = QUAN_A(mean): units digit 0-2 -> 0, 3-7 -> 5, 8-9 -> next ten."""
    lib = ol.load_fractal()
    import ctypes
    ref = np.full((4, 4), 9, np.uint8)
    a, b = ctypes.c_double(), ctypes.c_double()
    for mean, want in [(120, 120), (122, 120), (123, 125), (127, 125), (128, 130), (249, 250), (255, 255)]:
        org = np.full((4, 4), mean, np.uint8)
        lib.fro_compute_rms(org.ctypes.data, ref.ctypes.data, 4, 0, 0, 0, 0, 4, 4, ctypes.byref(a), ctypes.byref(b))
        assert b.value == want


def test_bound_chk_keeps_domain_inside_picture():
    h, w = 40, 48
    org = _texture(h, w, 3)
    ref = _texture(h, w, 4)
    out, xy = ol.fractal_search_batch(org, ref, 20, np.array([[0, 0, 8, 8], [40, 32, 8, 8], [44, 36, 4, 4]]))
    for (bx, by, bsx, bsy), (dx, dy) in zip([(0, 0, 8, 8), (40, 32, 8, 8), (44, 36, 4, 4)], xy):
        assert 0 <= bx + dx <= w - bsx and 0 <= by + dy <= h - bsy


def test_box_sums_are_exact_integer_sums():
    p = _texture(20, 24, 5)
    s, s2 = ol.fractal_box_sums(p, 4, 4)
    ref = np.lib.stride_tricks.sliding_window_view(p.astype(np.int64), (4, 4))
    np.testing.assert_array_equal(s, ref.sum((2, 3)))
    np.testing.assert_array_equal(s2, (ref ** 2).sum((2, 3)))
