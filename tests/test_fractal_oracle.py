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


# ---- a17: encode_one_macroblock quadtree gate (fro_encode_mbs) ----------------
import math  # noqa: E402

from fractal_scenes import gate_scene  # noqa: E402


def _chun_py(org, ref, bx, by):
    """block_enc.c:760-796 in plain Python floats (IEEE double, same order)"""
    R = [float(org[i, j]) for j in range(bx, bx + 16) for i in range(by, by + 16)]
    D = [float(ref[i, j]) for j in range(bx, bx + 16) for i in range(by, by + 16)]
    r, d = sum(R) / 256, sum(D) / 256
    sR = sD = 0.0
    for a, b in zip(R, D):
        sR += (a - r) * (a - r)
        sD += (b - d) * (b - d)
    mr = 0.0
    for a, b in zip(R, D):
        try:
            mr += ((a - r) / math.sqrt(sR)) * ((b - d) / math.sqrt(sD))
        except ZeroDivisionError:
            mr = math.nan
    return mr * mr


def _search(org, refs, R, bx, by, bsx, bsy, quirk4=False):
    """all views, first strict minimum -> (rms, scale, offset, x, y, reference, partition)"""
    best = None
    part = 0
    for k, ref in enumerate(refs):
        out, xy = ol.fractal_search_batch(org, ref, R, np.array([[bx, by, bsx, bsy]], np.int32))
        cand = (out[0, 0], out[0, 1], out[0, 2], int(xy[0, 0]), int(xy[0, 1]), k)
        if best is None or cand[0] < best[0]:
            best = cand
            if quirk4 and k == 1:
                part = 1
    return best + (part,)


def _tree_py(org, refs, R, tol16, tol8):
    """a second, independent statement of the gate in Python over fro_full_search"""
    h, w = org.shape
    recs = []
    for by in range(0, h, 16):
        for bx in range(0, w, 16):
            rec = {"mb": _search(org, refs, R, bx, by, 16, 16), "b8": {}, "sub": {}}
            chun = _chun_py(org, refs[0], bx, by)
            rec["chun"] = chun
            if 0.9 <= chun <= 1 and rec["mb"][0] > tol16 * tol16 * 256:
                rec["mb"] = rec["mb"][:6] + (3,)
                for q in range(4):
                    x8, y8 = bx + (q & 1) * 8, by + (q >> 1) * 8
                    n8 = _search(org, refs, R, x8, y8, 8, 8)
                    part, kids = 0, []
                    if n8[0] > tol8 * tol8 * 64:
                        pairs = [[(x8, y8, 8, 4), (x8, y8 + 4, 8, 4)], [(x8, y8, 4, 8), (x8 + 4, y8, 4, 8)]]
                        for mode, pair in ((1, pairs[0]), (2, pairs[1])):
                            halves = [_search(org, refs, R, *b) for b in pair]
                            if all(not (hv[0] > tol8 * tol8 * 32) for hv in halves):
                                part, kids = mode, halves
                                break
                        else:
                            part = 3
                            kids = [_search(org, refs, R, x8 + (s & 1) * 4, y8 + (s >> 1) * 4, 4, 4, True)
                                    for s in range(4)]
                    rec["b8"][q] = n8[:6] + (part,)
                    rec["sub"][q] = kids
            recs.append(rec)
    return recs


def _node_eq(node, tup):
    got = (node["rms"], node["scale"], node["offset"], node["x"], node["y"], node["reference"], node["partition"])
    return all(a == b for a, b in zip(got, tup))


@pytest.mark.parametrize("seed,K,tols", [(1, 1, (8.0, 5.0)), (2, 2, (4.0, 5.0)), (5, 4, (2.0, 4.0))])
def test_tree_oracle_matches_python_statement(seed, K, tols):
    org, refs = gate_scene(64, 48, seed, K, scale=6)
    R = 3
    out = ol.fractal_encode_mbs(org, refs, R, *tols)
    exp = _tree_py(org, refs, R, *tols)
    zero = np.zeros((), ol.FRO_NODE)
    for m, e in zip(out, exp):
        assert _node_eq(m["mb"], e["mb"])
        assert (np.isnan(m["chun"]) and np.isnan(e["chun"])) or m["chun"] == e["chun"]
        for q in range(4):
            if q in e["b8"]:
                assert _node_eq(m["b8"][q], e["b8"][q])
                kids = e["sub"][q]
                for c in range(4):
                    if c < len(kids):
                        assert _node_eq(m["sub"][q][c], kids[c])
                    else:
                        assert m["sub"][q][c].tobytes() == zero.tobytes()
            else:
                assert m["b8"][q].tobytes() == zero.tobytes()


def test_tree_oracle_reaches_every_partition():
    """the scenes used by the GPU parity tests exercise every branch of the gate"""
    seen_mb, seen_b8, nan, q4 = set(), set(), 0, 0
    for seed in range(3):
        org, refs = gate_scene(128, 96, seed, 2, scale=6)
        out = ol.fractal_encode_mbs(org, refs, 4, 4.0, 5.0)
        seen_mb |= set(out["mb"]["partition"].tolist())
        split = out["mb"]["partition"] == 3
        seen_b8 |= set(out["b8"]["partition"][split].ravel().tolist())
        nan += int(np.isnan(out["chun"]).sum())
        q4 += int((out["sub"]["partition"] == 1).sum())
    assert seen_mb == {0, 3} and seen_b8 == {0, 1, 2, 3} and nan > 0 and q4 > 0


def test_tree_planted_steps_pick_the_pairs():
    """an 8x8 carrying a horizontal offset step fails as a whole but its 8x4
    halves match (partition 1); a vertical step picks the 4x8 pair (2)"""
    h = w = 32
    yy, xx = np.mgrid[0:h, 0:w]
    ref = (128 + 100 * np.sin(xx / 3.0) * np.cos(yy / 4.0)).astype(np.float64)
    org = ref.copy()
    step = np.zeros((h, w))
    step[0:4, 0:8] += 15
    step[4:8, 0:8] -= 15          # MB 0, 8x8 #0: horizontal step
    step[0:8, 8:12] += 15
    step[0:8, 12:16] -= 15        # MB 0, 8x8 #1: vertical step
    org = np.clip(np.rint(org + step), 0, 255).astype(np.uint8)
    ref = np.clip(np.rint(ref), 0, 255).astype(np.uint8)
    out = ol.fractal_encode_mbs(org, [ref], 0, 1.0, 5.0)
    m = out[0]
    assert 0.9 <= m["chun"] <= 1 and m["mb"]["partition"] == 3
    assert m["b8"]["partition"][0] == 1 and m["b8"]["partition"][1] == 2
    assert out[1]["mb"]["partition"] == 0 or out[1]["chun"] < 0.9 or out[1]["mb"]["rms"] > 256
