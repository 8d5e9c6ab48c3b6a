"""The thesis's own fractal dumps constrain the fractal oracle.

tests/golden/trans_show/trans_show_{Y,UV}.txt are the reference's
Debug/trans_show_*.txt: one 640x480 P-frame of the thesis codec (Search_Range 7,
Debug/encoder.cfg), written by tran_show (ZL/src/image.c:996-1106).  Its input
YUV is not in the reference, so the trees cannot be recomputed and the values
stay "parity unpinned".  But every record is an output of full_search /
compute_rms / the quadtree gating, and those leave fingerprints that do not
depend on the input.  Each test below checks one of them against every record,
with the rule taken from oracle/fractal_oracle.c (the restatement the HIP path
is tested against), so a record the restatement could not produce is a
faithfulness bug in the restatement:

* scale: compute_rms sets a = (int)(alpha*100), QUAN_A(a), alpha = a/100
  (ZL/src/compute.c:170-178, QUAN_A ZL/inc/defines_enc.h:591-601).  C's
  truncating % and / make QUAN_A map a positive a to a multiple of 5 and a
  negative a to a multiple of 10, so scale*20 is an integer, even when
  negative, within [MIN_ALPHA, MAX_ALPHA] = [-2.35, 4.0] (defines_enc.h:19-20);
* offset: beta = rsum1/no, QUAN_A((int)beta): rsum1 >= 0, so offset is a
  multiple of 5 in [0, 255] (tighter than [MIN_BETA, MAX_BETA]);
* (x, y): full_search only takes candidates bound_chk accepts
  (ZL/src/block_enc.c:1933-1977, 2894-2919): |x|, |y| <= Search_Range and the
  domain block inside the 640x480 luma / 320x240 chroma plane;
* shape: encode_one_macroblock leaves a macroblock unsplit or split into four
  8x8 (its 16x8 / 8x16 loop never ends early, block_enc.c:798-855), each 8x8
  whole, an 8x4 pair, a 4x8 pair or four 4x4 (block_enc.c:1337-1675);
  chroma is searched at the macroblock level only in this run;
* reference: the C view searches views 0..3; views 1..3 are the zero-filled H,
  M, N planes (ZL/src/memalloc.c:415,595-598), on which every candidate has
  det == 0 -> alpha = 0, so a record with reference > 0 must have scale 0 and
  (x, y) = (0, 0).
"""
import os
import re

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "trans_show")
REC = re.compile(r"\n(luma|2、chroma|3、chroma),mode=([0-9.]+)\n(-?\d+) +(-?\d+) +(-?\d+) +(-?\d+) +(-?[0-9.]+) +(-?[0-9.]+)")
W, H, SEARCH_RANGE = 640, 480, 7          # Debug/encoder.cfg: ImageWidth, ImageHeight, Search_Range
MIN_ALPHA, MAX_ALPHA = -2.35, 4.0         # ZL/inc/defines_enc.h:19-20


def _records(name):
    """[(mb, label, mode, block_type, x, y, reference, offset/5, scale*20)] in file order."""
    text = open(os.path.join(HERE, name), "rb").read().decode("gbk")
    _, *parts = re.split(r"\nCurrentMb=\s*(\d+)", text)
    out = []
    for i in range(0, len(parts), 2):
        mb = int(parts[i])
        for m in REC.finditer(parts[i + 1]):
            out.append((mb, m.group(1), m.group(2), int(m.group(3)), int(m.group(4)), int(m.group(5)),
                        int(m.group(6)), float(m.group(7)), float(m.group(8))))
    return out


def _luma_blocks():
    """(record, block origin x, y, width, height) for trans_show_Y.txt: the
    macroblock node, or per 8x8 quadrant q (raster) its node / pair halves /
    4x4 blocks in the order tran_show prints them (image.c:1012-1040)."""
    recs = _records("trans_show_Y.txt")
    out, i = [], 0
    while i < len(recs):
        mb = recs[i][0]
        bx, by = (mb % (W // 16)) * 16, (mb // (W // 16)) * 16
        if recs[i][2] == "0":
            out.append((recs[i], bx, by, 16, 16))
            i += 1
            continue
        for q in range(4):
            r = recs[i]
            assert r[0] == mb and r[2].startswith("3."), r
            k = int(r[2][2:])
            qx, qy = bx + 8 * (q & 1), by + 8 * (q >> 1)
            if k == 0:
                geo = [(qx, qy, 8, 8)]
            elif k == 1:                              # 8x4 pair: halves stacked (encode_block_rect mode 1)
                geo = [(qx, qy, 8, 4), (qx, qy + 4, 8, 4)]
            elif k == 2:                              # 4x8 pair: side by side (mode 2)
                geo = [(qx, qy, 4, 8), (qx + 4, qy, 4, 8)]
            else:                                     # four 4x4, raster (encode_block_8's i, j loops)
                geo = [(qx + 4 * (j & 1), qy + 4 * (j >> 1), 4, 4) for j in range(4)]
            for g in geo:
                assert recs[i][0] == mb and recs[i][2] == r[2]
                out.append((recs[i],) + g)
                i += 1
    return out


def _chroma_blocks():
    recs = _records("trans_show_UV.txt")
    cw = W // 2
    return [(r, (r[0] % (cw // 16)) * 16, (r[0] // (cw // 16)) * 16, 16, 16) for r in recs]


def _quan_a(x: int) -> int:
    """QUAN_A (defines_enc.h:591-601) with C's truncating / and %."""
    c = int(x / 10)
    b = x - 10 * c
    if 2 < b < 8:
        b = 5
    elif b > 7:
        b, c = 0, c + 1
    else:
        b = 0
    return 10 * c + b


SCALE_LATTICE = {a for a in (_quan_a(v) for v in range(-400, 500)) if MIN_ALPHA <= a / 100 <= MAX_ALPHA}
OFFSET_LATTICE = {_quan_a(v) for v in range(0, 256)}


@pytest.mark.parametrize("which", ["Y", "UV"])
def test_every_record_is_on_the_quantisation_lattice(which):
    blocks = _luma_blocks() if which == "Y" else _chroma_blocks()
    assert len(blocks) == (1211 if which == "Y" else 600)
    for r, *_ in blocks:
        s20, o5 = r[8], r[7]
        a = round(s20 * 5)                       # scale * 100
        assert abs(s20 * 5 - a) < 1e-6 and a in SCALE_LATTICE, r
        off = round(o5 * 5)
        assert abs(o5 * 5 - off) < 1e-6 and off in OFFSET_LATTICE, r


def test_negative_scales_show_truncating_quan_a():
    """The lattice is not vacuous on this data.  Of the 1,787 positive scales
    about half (893) sit on the odd multiples of 0.05 (QUAN_A's "5" branch), yet
    all 23 negative ones are multiples of 0.1: (int)x % 10 is never above 2 for
    a negative x in C, so the restatement's QUAN_A can only produce those (a
    floor-based reading would put about half of them on the 0.05 grid too;
    23 of 23 by chance is ~1e-7)."""
    a = np.array([round(r[8] * 5) for r, *_ in _luma_blocks() + _chroma_blocks()])
    pos, neg = a[a > 0], a[a < 0]
    assert len(neg) == 23 and (neg % 10 == 0).all()
    assert (pos % 10 == 5).sum() > 0.4 * len(pos)


@pytest.mark.parametrize("which", ["Y", "UV"])
def test_every_vector_passes_bound_chk(which):
    blocks = _luma_blocks() if which == "Y" else _chroma_blocks()
    pw, ph = (W, H) if which == "Y" else (W // 2, H // 2)
    for r, bx, by, bw, bh in blocks:
        x, y = r[4], r[5]
        assert max(abs(x), abs(y)) <= SEARCH_RANGE, r
        assert 0 <= bx + x <= pw - bw and 0 <= by + y <= ph - bh, (r, bx, by)


def test_partition_shapes_are_ones_the_gating_emits():
    recs = _records("trans_show_Y.txt")
    mbs = {}
    for r in recs:
        mbs.setdefault(r[0], []).append(r)
    assert sorted(mbs) == list(range((W // 16) * (H // 16)))
    for mb, rs in mbs.items():
        if rs[0][2] == "0":
            assert len(rs) == 1 and rs[0][3] == 0      # macroblock node: block_type 0 (block_enc.c:570)
            continue
        # four 8x8 quadrants, each printing 1, 2, 2 or 4 records for 3.0 .. 3.3
        n = {"3.0": 1, "3.1": 2, "3.2": 2, "3.3": 4}
        i = q = 0
        while i < len(rs):
            i += n[rs[i][2]]
            q += 1
        assert i == len(rs) and q == 4, mb
    uv = _records("trans_show_UV.txt")
    assert all(r[2] == "0" and r[3] == 0 for r in uv)
    assert [r[1] for r in uv] == ["2、chroma", "3、chroma"] * (len(uv) // 2)


@pytest.mark.parametrize("which", ["Y", "UV"])
def test_zero_filled_views_can_only_win_with_scale_zero(which):
    blocks = _luma_blocks() if which == "Y" else _chroma_blocks()
    for r, *_ in blocks:
        assert 0 <= r[6] <= 3
        if r[6] > 0:
            assert r[8] == 0 and (r[4], r[5]) == (0, 0), r


def test_restatement_outputs_lie_on_the_same_lattice():
    """The lattice above is the restatement's: full_search of random blocks
    through oracle/fractal_oracle.c returns only (scale, offset) pairs in it,
    and reaches both parities and both signs."""
    import oracle_lib as ol
    rng = np.random.default_rng(11)
    h, w = 96, 96
    ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
    org = np.clip(ref.astype(int) * rng.choice([-1, 1], (h, w)) // 2 + rng.integers(0, 200, (h, w)), 0, 255)
    org = org.astype(np.uint8)
    req = np.array([[x, y, s, s] for s in (4, 8, 16) for y in range(0, h - s + 1, s) for x in range(0, w - s + 1, s)],
                   np.int32)
    out, xy = ol.fractal_search_batch(org, ref, 7, req)
    scales, offsets = out[:, 1], out[:, 2]
    ok = out[:, 0] < 1e29                         # a candidate passed the alpha/beta bounds
    a = np.round(scales[ok] * 100).astype(int)
    assert np.allclose(scales[ok] * 100, a) and set(a.tolist()) <= SCALE_LATTICE
    assert set(np.round(offsets).astype(int).tolist()) <= OFFSET_LATTICE
    assert (a < 0).any() and (a % 10 == 5).any()
