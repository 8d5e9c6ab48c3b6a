"""GPU: high-bit-depth luma (SourceBitDepthLuma 9..14; JM's imgpel is uint16,
JM/lencod/inc/defines.h:37, JM/lcommon/inc/typedefs.h:30-40).  A context created
with SourceBitDepthLuma > 8 keeps its planes 16-bit on the device and serves
every full / fast full search batch with the v_sad_u16 small kernel
(csrc/jmme_search.hip me_small_kernel<FFS, true>).  Checked against the oracle
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


@pytest.mark.parametrize("bits,size,R", [(10, (352, 288), 16), (10, (176, 144), 32), (12, (128, 96), 7),
                                         (14, (96, 64), 3)])
def test_hbd_full_search_vs_oracle(bits, size, R, gpu):
    from jmme import FULL_SEARCH, MotionEstimator
    w, h = size
    cur, ref = _planes(w, h, bits, seed=bits + R)[::-1]
    rng = np.random.default_rng(bits * 100 + R)
    req = _random_units(rng, w, h, 12, R, lam_max=4000)
    with MotionEstimator({"SearchRange": max(R, 1), "SearchMode": -1, "SourceBitDepthLuma": bits}) as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FULL_SEARCH, req)
    _cmp(out, *_oracle_units(cur, ref, req))


@pytest.mark.parametrize("R,rdopt,far", [(16, 0, 0.0), (8, 1, 0.4)])
def test_hbd_fast_full_search_vs_oracle(R, rdopt, far, gpu):
    from jmme import FAST_FULL_SEARCH, MotionEstimator
    w, h = 352, 288
    cur, ref = _planes(w, h, 10, seed=R + rdopt)[::-1]
    rng = np.random.default_rng(7 * R + rdopt)
    req, mbs, blk = _ffs_random(rng, w, h, 12, R, rdopt, far)
    with MotionEstimator({"SearchRange": R, "SearchMode": 0, "RDOptimization": rdopt, "SourceBitDepthLuma": 10}) as me:
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


def test_hbd_extremes_14bit(gpu):
    """14-bit planes at both ends of the range (SAD of a 16x16 block near 2^22)
    and a large lambda: the 32-bit costs of the small kernel do not wrap"""
    from jmme import FULL_SEARCH, MotionEstimator
    w, h, R = 64, 64, 4
    rng = np.random.default_rng(3)
    cur = np.where(rng.random((h, w)) < 0.5, 0, 16383).astype(np.uint16)
    ref = (16383 - cur).astype(np.uint16)
    req = _random_units(rng, w, h, 6, R, lam_max=60000)
    with MotionEstimator({"SearchRange": R, "SearchMode": -1, "SourceBitDepthLuma": 14}) as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FULL_SEARCH, req)
    _cmp(out, *_oracle_units(cur, ref, req))


def test_hbd_refusals(gpu):
    """samples above the declared depth are refused at upload; the 8-bit-only
    paths (sub-pel planes / refinement, EPZS) refuse a high-bit-depth context"""
    from jmme import EPZS_REQ, SUBPEL_REQ, JmmeError, MotionEstimator
    plane = np.full((32, 32), 1023, np.uint16)
    with MotionEstimator({"SourceBitDepthLuma": 10}) as me:
        me.upload_cur(plane)
        me.upload_ref(0, 0, plane)
        with pytest.raises(JmmeError):
            me.upload_cur(np.full((32, 32), 1024, np.uint16))
        q = np.zeros(1, SUBPEL_REQ)
        q["blocktype"] = 1
        with pytest.raises(JmmeError):
            me.subpel_refine(q)
        e = np.zeros(1, EPZS_REQ)
        e["bsx"] = e["bsy"] = 16
        e["blocktype"] = 1
        with pytest.raises(JmmeError):
            me.epzs_search(e, np.zeros((0, 2), np.int16))
    with pytest.raises(JmmeError):
        MotionEstimator({"SourceBitDepthLuma": 15})
