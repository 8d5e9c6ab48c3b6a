"""GPU: high-bit-depth luma (SourceBitDepthLuma 9..14; JM's imgpel is uint16,
JM/lencod/inc/defines.h:37, JM/lcommon/inc/typedefs.h:30-40).  A context created
with SourceBitDepthLuma > 8 keeps its planes 16-bit on the device and serves
its full / fast full search batches with the v_sad_u16 kernels: small batches
on the small kernel (csrc/jmme_search.hip me_small_kernel<FFS, true>), the rest
on the 64-bit-key instance of the item kernel (me_items_kernel<false, FFS,
true>); `path` forces one or the other.  Checked against the oracle
(oracle/me_oracle.c, which reads uint16 planes as JM does) on random requests,
against the 8-bit path on 8-bit content, at 14-bit extremes, and on the
refusals of the 8-bit-only paths."""
import numpy as np
import pytest

import oracle_lib as ol
from test_gpu_parity import SPIRAL, _ffs_random, _oracle_units, _random_units

pytestmark = pytest.mark.gpu


def _planes(w, h, bits, seed, gmv=(3, -2)):
    """2 frames of structured content at `bits` (the 8-bit texture scaled, plus
    low-order noise that only a 16-bit search sees)"""
    from jmme import synth
    luma = synth.luma_sequence(w, h, 2, seed=seed, gmv=gmv).astype(np.int32)
    rng = np.random.default_rng(seed)
    sh = bits - 8
    out = (luma << sh) + rng.integers(0, 1 << sh, size=luma.shape)
    return np.clip(out, 0, (1 << bits) - 1).astype(np.uint16)


def _cmp(out, keys, mv, cost):
    got = np.array([(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u, s in keys])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(keys[i], got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


def _path(me, path):
    me.set_small_batch_limit(0 if path == "items" else 1 << 20)


@pytest.mark.parametrize("path", ["small", "items"])
@pytest.mark.parametrize("bits,size,R", [(10, (352, 288), 16), (10, (176, 144), 32), (12, (128, 96), 7),
                                         (14, (96, 64), 3), (10, (176, 144), 55), (10, (176, 144), 64)])
def test_hbd_full_search_vs_oracle(bits, size, R, path, gpu):
    """R 55 / 64: staged rows of more than 64 dwords (the item kernel's prefetch
    splits each row over several wave instructions)"""
    from jmme import FULL_SEARCH, MotionEstimator
    w, h = size
    cur, ref = _planes(w, h, bits, seed=bits + R)[::-1]
    rng = np.random.default_rng(bits * 100 + R)
    req = _random_units(rng, w, h, 12, R, lam_max=4000)
    with MotionEstimator({"SearchRange": max(R, 1), "SearchMode": -1, "SourceBitDepthLuma": bits}) as me:
        _path(me, path)
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FULL_SEARCH, req)
    _cmp(out, *_oracle_units(cur, ref, req))


@pytest.mark.parametrize("path", ["small", "items"])
@pytest.mark.parametrize("R,rdopt,far", [(16, 0, 0.0), (8, 1, 0.4)])
def test_hbd_fast_full_search_vs_oracle(R, rdopt, far, path, gpu):
    from jmme import FAST_FULL_SEARCH, MotionEstimator
    w, h = 352, 288
    cur, ref = _planes(w, h, 10, seed=R + rdopt)[::-1]
    rng = np.random.default_rng(7 * R + rdopt)
    req, mbs, blk = _ffs_random(rng, w, h, 12, R, rdopt, far)
    with MotionEstimator({"SearchRange": R, "SearchMode": 0, "RDOptimization": rdopt, "SourceBitDepthLuma": 10}) as me:
        _path(me, path)
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FAST_FULL_SEARCH, req)
        max_mvd = me.max_mvd
    mv, cost = ol.ffs_batch(cur, ref, R, max_mvd, rdopt, mbs, blk)
    keys = [(u, s) for u in range(len(req)) for s in range(41)]
    _cmp(out, keys, mv, cost)
    assert R in SPIRAL


def test_hbd_path_equals_8bit_path_on_8bit_content(gpu):
    """8-bit samples through a 10-bit context (16-bit planes, v_sad_u16) give the
    8-bit context's answers (v_sad_u8 item kernel) on every partition"""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    w, h, R = 352, 288, 24
    luma = synth.luma_sequence(w, h, 2, seed=5, gmv=(2, 1))
    req = _random_units(np.random.default_rng(1), w, h, 40, R)
    res = []
    for bits in (8, 10):
        with MotionEstimator({"SearchRange": R, "SearchMode": -1, "SourceBitDepthLuma": bits}) as me:
            me.upload_cur(luma[1])
            me.upload_ref(0, 0, luma[0])
            res.append(me.search(FULL_SEARCH, req))
    assert np.array_equal(res[0], res[1])


@pytest.mark.parametrize("path,lam_max", [("small", 60000), ("items", 60000), ("items", 2000000)])
def test_hbd_extremes_14bit(path, lam_max, gpu):
    """14-bit planes at both ends of the range (SAD of a 16x16 block near 2^22)
    and a large lambda: the 32-bit costs of the small kernel do not wrap; a
    lambda the small kernel's 32-bit costs cannot hold goes to the item kernel's
    64-bit keys"""
    from jmme import FULL_SEARCH, MotionEstimator
    w, h, R = 64, 64, 4
    rng = np.random.default_rng(3)
    cur = np.where(rng.random((h, w)) < 0.5, 0, 16383).astype(np.uint16)
    ref = (16383 - cur).astype(np.uint16)
    req = _random_units(rng, w, h, 6, R, lam_max=lam_max)
    with MotionEstimator({"SearchRange": R, "SearchMode": -1, "SourceBitDepthLuma": 14}) as me:
        _path(me, path)
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FULL_SEARCH, req)
    _cmp(out, *_oracle_units(cur, ref, req))


@pytest.mark.parametrize("ffs", [0, 1])
def test_hbd_10bit_saturated_keys(ffs, gpu):
    """10-bit planes at both ends of the range: the 32-bit keys of the 10-bit item
    kernel stay exact for 4x4 blocks (SAD < 2^14) while every larger partition's
    key saturates, so those partitions go through the exact 64-bit re-search --
    the results must equal the oracle's everywhere (FS and FFS, RDO off)"""
    from jmme import FAST_FULL_SEARCH, FULL_SEARCH, MotionEstimator
    w, h, R = 96, 64, 8
    rng = np.random.default_rng(11 + ffs)
    cur = np.where(rng.random((h, w)) < 0.5, 0, 1023).astype(np.uint16)
    ref = (1023 - cur).astype(np.uint16)
    ref[::7] = cur[::7]                       # a few rows that match: mixed saturated / exact keys
    with MotionEstimator({"SearchRange": R, "SearchMode": 0 if ffs else -1, "RDOptimization": 0,
                          "SourceBitDepthLuma": 10}) as me:
        _path(me, "items")
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        if ffs:
            req, mbs, blk = _ffs_random(rng, w, h, 12, R, 0, 0.0)
            out = me.search(FAST_FULL_SEARCH, req)
            max_mvd = me.max_mvd
        else:
            req = _random_units(rng, w, h, 12, R, lam_max=4000)
            out = me.search(FULL_SEARCH, req)
    if ffs:
        mv, cost = ol.ffs_batch(cur, ref, R, max_mvd, 0, mbs, blk)
        _cmp(out, [(u, s) for u in range(len(req)) for s in range(41)], mv, cost)
    else:
        _cmp(out, *_oracle_units(cur, ref, req))


def test_hbd_refusals(gpu):
    """samples above the declared depth are refused at upload; SSE sub-pel
    refinement is refused above 11 bits (JM's int sum can wrap there)"""
    from jmme import SUBPEL_REQ, JmmeError, MotionEstimator
    plane = np.full((32, 32), 1023, np.uint16)
    with MotionEstimator({"SourceBitDepthLuma": 10}) as me:
        me.upload_cur(plane)
        me.upload_ref(0, 0, plane)
        with pytest.raises(JmmeError):
            me.upload_cur(np.full((32, 32), 1024, np.uint16))
        q = np.zeros(1, SUBPEL_REQ)
        q["blocktype"] = 1
        q["metric_h"] = q["metric_q"] = 1
        q["search_pos2"] = q["search_pos4"] = 9
        me.subpel_validate(q)                       # SSE at 10 bits: served
    with pytest.raises(JmmeError):
        MotionEstimator({"SourceBitDepthLuma": 15})
    with MotionEstimator({"SourceBitDepthLuma": 12}) as me:
        p12 = np.full((32, 32), 4095, np.uint16)
        me.upload_cur(p12)
        me.upload_ref(0, 0, p12)
        q["metric_q"] = 2
        with pytest.raises(JmmeError):               # SSE half-pel at 12 bits
            me.subpel_refine(q)
        q["metric_h"] = 0
        me.subpel_validate(q)


# ---- sub-pel at high bit depth: 16-bit sub-images (getSubImagesLuma with
# max_imgpel_value = (1 << bits) - 1, img_luma.c:184-329) and the refinement on
# them (me_fullsearch.c:186-289, me_epzs_sub.c:30-222), vs the restatement

@pytest.mark.parametrize("bits,hw", [(10, (144, 176)), (12, (64, 96)), (14, (48, 32))])
def test_hbd_sub_images_vs_oracle(gpu, bits, hw):
    from jmme import MotionEstimator
    h, w = hw
    rng = np.random.default_rng(bits)
    top = (1 << bits) - 1
    # extremes exercise the six-tap clip at 0 and max_imgpel_value
    plane = np.where(rng.random((h, w)) < 0.3, rng.choice(np.array([0, top, 1, top - 1]), size=(h, w)),
                     rng.integers(0, top + 1, size=(h, w))).astype(np.uint16)
    with MotionEstimator({"SourceBitDepthLuma": bits}) as me:
        me.upload_cur(plane)
        me.upload_ref(0, 2, plane)
        got = me.sub_images(0, 2)
    exp = ol.sub_images(plane, bits)
    bad = [k for k in range(16) if not np.array_equal(got[k], exp[k])]
    assert not bad, (bits, bad)
    assert got.max() == top   # the clip bound is reached (not 255)


@pytest.mark.parametrize("bits,seed", [(10, 1), (10, 2), (11, 3), (12, 4), (14, 5)])
def test_hbd_refinement_random_vs_oracle(gpu, bits, seed):
    """both refinement functions, SAD / SSE / SATD 4x4 / 8x8 (SSE up to 11 bits),
    finite bounds, vectors outside the picture"""
    from jmme import MotionEstimator
    from test_subpel_gpu import random_requests, to_oracle
    rng = np.random.default_rng(100 + seed)
    h, w = (144, 176) if seed != 2 else (288, 352)
    cur, ref = _planes(w, h, bits, seed=seed)[::-1]
    q = random_requests(rng, 4000, w, h)
    if bits > 11:   # SSE is refused there
        q["metric_h"] = np.where(q["metric_h"] == 1, 2, q["metric_h"])
        q["metric_q"] = np.where(q["metric_q"] == 1, 0, q["metric_q"])
    # bounds on the scale of these samples (the 8-bit generator's are too small to bind)
    big = rng.random(len(q)) < 0.3
    q["min_mcost"] = np.where(big, rng.integers(0, 60000, len(q)) * 32 << (bits - 8), q["min_mcost"])
    with MotionEstimator({"SourceBitDepthLuma": bits}) as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        got = me.subpel_refine(q)
    sub = ol.sub_images(ref, bits)
    mv = np.zeros((len(q), 2), np.int16)
    cost = np.zeros(len(q), np.int64)
    o = to_oracle(q)
    for v in (0, 1):
        k = q["variant"] == v
        mv[k], cost[k] = ol.sub_pel_batch(cur, sub, o[k], bool(v))
    bad = np.nonzero((got["mv_x"] != mv[:, 0]) | (got["mv_y"] != mv[:, 1]) | (got["cost"] != cost))[0]
    assert len(bad) == 0, (bits, len(bad), q[bad[:3]], got[bad[:3]], mv[bad[:3]], cost[bad[:3]])



# ---- EPZS at high bit depth: the v_sad_u16 instantiation of the EPZS kernel on
# 16-bit planes (integer grid) and 16-bit sub-images (EPZSSubPelGrid = 1), vs
# the 16-bit build of the restatement (oracle/epzs_oracle.c -DEO_PEL16)

@pytest.mark.parametrize("bits,grid,seed", [(10, 0, 0), (10, 1, 1), (12, 0, 2), (14, 1, 3)])
def test_hbd_epzs_random_vs_restatement(gpu, bits, grid, seed):
    from jmme import MotionEstimator
    from test_epzs_gpu import _random_requests, _run_frame
    rng = np.random.default_rng(200 + seed)
    w, h = 96, 64
    cur, r1 = _planes(w, h, bits, seed=seed)[::-1]
    r0 = _planes(w, h, bits, seed=seed + 50, gmv=(-1, 2))[0]
    refs = [r1, r0]
    req, preds, stale = _random_requests(rng, w, h, 1500)
    sc = 1 << (bits - 8)   # thresholds on the scale of these SADs
    for k in ("medthres", "stop_crit"):
        req[k] = req[k] * sc
    if grid:
        req["variant"] += 2
        req["center_x"] += rng.integers(-3, 4, len(req))
        req["center_y"] += rng.integers(-3, 4, len(req))
        req["max_x"] = np.minimum(req["max_x"], 128)
        req["pattern"] = rng.choice([0, 1, 2, 3, 4, 5], len(req))
        exp = ol.epzs_grid_batch(req, preds, stale, cur, refs, bits)
    else:
        exp = ol.epzs_batch(req, preds, stale, cur, refs)
    cfg = {"SourceBitDepthLuma": bits, "SearchMode": 3, "EPZSSubPelGrid": grid, "SearchRange": 32}
    with MotionEstimator(cfg) as me:
        got = _run_frame(me, cur, refs, req, preds, stale)
    for k in ("mv_x", "mv_y", "path", "cost", "prev_sad"):
        bad = np.nonzero(got[k] != exp[k])[0]
        assert len(bad) == 0, (k, len(bad), req[bad[:2]], got[bad[:2]], exp[bad[:2]])
    assert len(set(np.unique(exp["path"]))) >= 4


@pytest.mark.parametrize("grid", [0])   # (sub-images differ: the six-tap clip is max_imgpel_value)
def test_hbd_epzs_equals_8bit_on_8bit_content(gpu, grid):
    from jmme import MotionEstimator, synth
    from test_epzs_gpu import _random_requests, _run_frame
    rng = np.random.default_rng(7 + grid)
    w, h = 96, 64
    luma = synth.luma_sequence(w, h, 3, seed=4, gmv=(2, -1))
    cur, refs = luma[2], [luma[1], luma[0]]
    req, preds, stale = _random_requests(rng, w, h, 1500)
    if grid:
        req["variant"] += 2
        req["max_x"] = np.minimum(req["max_x"], 128)
    res = []
    for bits in (8, 10):
        cfg = {"SourceBitDepthLuma": bits, "SearchMode": 3, "EPZSSubPelGrid": grid, "SearchRange": 32}
        with MotionEstimator(cfg) as me:
            res.append(_run_frame(me, cur, refs, req, preds, stale))
    assert np.array_equal(res[0], res[1])
