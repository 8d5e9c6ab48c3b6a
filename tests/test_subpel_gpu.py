"""GPU: the HIP quarter-pel interpolation and sub-pel refinement
(csrc/jmme_subpel.hip) against JM 18.5 itself -- the sub-images JM built and
every sub-pel refinement of the captured encodes (tests/golden/subpel_*.npz) --
and against the restatement (oracle/subpel_oracle.c) on randomised requests:
both refinement functions, SAD / SSE / SATD 4x4 / SATD 8x8, both
start_me_refinement settings, finite bounds (JM's early-exit return values),
vectors far outside the picture, and the chained integer -> sub-pel path."""
import numpy as np
import pytest

import oracle_lib as ol
from subpel_cases import SubpelCase, cases, subimg_cases

pytestmark = pytest.mark.gpu


def to_req(r, idx):
    """fixture records -> SUBPEL_REQ"""
    from jmme import SP_CHECK0, SP_TEST8x8, SUBPEL_REQ
    q = np.zeros(len(idx), SUBPEL_REQ)
    for f in ("pos_x", "pos_y", "blocktype", "pred_x", "pred_y", "lambda_h", "lambda_q", "subthres", "metric_h",
              "metric_q", "start_hp", "start_qp", "search_pos2", "search_pos4"):
        q[f] = r[f][idx]
    q["ref_slot"] = r["list"][idx] * 32 + r["ref"][idx]
    q["mv_x"], q["mv_y"] = r["mv_in_x"][idx], r["mv_in_y"][idx]
    q["min_mcost"] = r["min_mcost_in"][idx]
    q["variant"] = r["kind"][idx]
    q["flags"] = (np.where(r["test8x8"][idx] != 0, SP_TEST8x8, 0) |
                  np.where((r["rdopt"][idx] == 0) & (r["slice_type"][idx] != 1), SP_CHECK0, 0))
    return q


def to_oracle(q, slice_type=0):
    """SUBPEL_REQ -> SPO_REQ (oracle_lib)"""
    from jmme import SP_CHECK0, SP_TEST8x8
    o = np.zeros(len(q), ol.SPO_REQ)
    bt = q["blocktype"].astype(np.int32)
    o["bsx"] = np.select([bt <= 2, bt <= 5], [16, 8], 4)
    o["bsy"] = np.select([(bt == 1) | (bt == 3), (bt == 2) | (bt == 4) | (bt == 6)], [16, 8], 4)
    for f in ("pos_x", "pos_y", "blocktype", "pred_x", "pred_y", "mv_x", "mv_y", "min_mcost", "lambda_h", "lambda_q",
              "metric_h", "metric_q", "start_hp", "start_qp", "search_pos2", "search_pos4", "subthres"):
        o[f] = q[f]
    o["ref"] = q["ref_slot"] % 32
    o["test8x8"] = (q["flags"] & SP_TEST8x8) != 0
    chk = (q["flags"] & SP_CHECK0) != 0
    o["rdopt"] = np.where(chk, 0, 1)
    o["slice_type"] = slice_type
    return o


def oracle_run(cur, ref, q):
    sub = ol.sub_images(ref)
    mv = np.zeros((len(q), 2), np.int16)
    cost = np.zeros(len(q), np.int64)
    o = to_oracle(q)
    for v in (0, 1):
        k = q["variant"] == v
        if k.any():
            mv[k], cost[k] = ol.sub_pel_batch(cur, sub, o[k], bool(v))
    return mv, cost


@pytest.mark.parametrize("name", subimg_cases())
def test_sub_images_match_jm(gpu, name):
    from jmme import MotionEstimator
    c = SubpelCase(name)
    for src, exp in zip(c.sub_src, c.sub_img):
        with MotionEstimator() as me:
            me.upload_cur(src)
            me.upload_ref(0, 0, src)
            got = me.sub_images(0, 0)
        assert got.shape == exp.shape
        bad = [k for k in range(16) if not np.array_equal(got[k], exp[k])]
        assert not bad, (name, bad)


@pytest.mark.parametrize("hw", [(16, 16), (48, 32), (144, 176), (1088, 1920)])
def test_sub_images_random_vs_oracle(gpu, hw):
    from jmme import MotionEstimator
    h, w = hw
    rng = np.random.default_rng(h * 7 + w)
    # extremes exercise the six-tap clipping at 0 and 255
    plane = rng.choice(np.array([0, 255, 1, 254, 128], np.uint8), size=(h, w)) if h < 200 else \
        rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    with MotionEstimator() as me:
        me.upload_cur(plane)
        me.upload_ref(1, 3, plane)
        got = me.sub_images(1, 3)
    exp = ol.sub_images(plane)
    bad = [k for k in range(16) if not np.array_equal(got[k], exp[k])]
    assert not bad, (hw, bad)


def test_sub_images_device_form(gpu):
    import torch
    from jmme import MotionEstimator
    h, w = 64, 96
    plane = np.random.default_rng(5).integers(0, 256, size=(h, w), dtype=np.uint8)
    pitch, ph = 256, h + 40
    stride = ph * pitch + 64
    src = torch.from_numpy(plane).to(gpu)
    dst = torch.zeros(16 * stride, dtype=torch.uint8, device=gpu)
    with MotionEstimator() as me:
        me.sub_images_async(src.data_ptr(), w, w, h, dst.data_ptr(), pitch, stride, 0)
        torch.cuda.synchronize()
    got = dst.cpu().numpy()[:16 * stride].reshape(16, stride)[:, :ph * pitch].reshape(16, ph, pitch)[:, :, :w + 64]
    assert np.array_equal(got, ol.sub_images(plane).astype(np.uint8))


@pytest.mark.parametrize("name", cases())
def test_refinement_matches_jm(gpu, name):
    from jmme import MotionEstimator
    c = SubpelCase(name)
    n = 0
    with MotionEstimator() as me:
        for f, lst, ref, idx in c.groups():
            me.upload_cur(c.cur[f])
            me.upload_ref(lst, ref, c.ref[(f, lst, ref)])
            got = me.subpel_refine(to_req(c.r, idx))
            emv, ecost = c.expected(idx)
            bad = np.nonzero((got["mv_x"] != emv[:, 0]) | (got["mv_y"] != emv[:, 1]) | (got["cost"] != ecost))[0]
            assert len(bad) == 0, (name, f, ref, len(bad), to_req(c.r, idx)[bad[:3]], got[bad[:3]], emv[bad[:3]],
                                   ecost[bad[:3]])
            n += len(idx)
    assert n == c.meta["n_searches"]


def random_requests(rng, n, w, h, slots=(0,)):
    from jmme import DISTBLK_MAX, SP_CHECK0, SP_TEST8x8, SUBPEL_REQ
    q = np.zeros(n, SUBPEL_REQ)
    bt = rng.integers(1, 8, n)
    q["blocktype"] = bt
    bsx = np.select([bt <= 2, bt <= 5], [16, 8], 4)
    bsy = np.select([(bt == 1) | (bt == 3), (bt == 2) | (bt == 4) | (bt == 6)], [16, 8], 4)
    q["pos_x"] = rng.integers(0, (w - bsx) // 4 + 1) * 4
    q["pos_y"] = rng.integers(0, (h - bsy) // 4 + 1) * 4
    q["ref_slot"] = rng.choice(np.array(slots), n)
    far = rng.random(n) < 0.2   # vectors that leave the picture (UMVLine4X clamps)
    q["mv_x"] = np.where(far, rng.integers(-4 * (w + 80), 4 * (w + 80), n), rng.integers(-40, 41, n) * 4)
    q["mv_y"] = np.where(far, rng.integers(-4 * (h + 60), 4 * (h + 60), n), rng.integers(-40, 41, n) * 4)
    zero = rng.random(n) < 0.1
    q["mv_x"][zero] = 0
    q["mv_y"][zero] = 0
    q["pred_x"] = q["mv_x"] + rng.integers(-9, 10, n)
    q["pred_y"] = q["mv_y"] + rng.integers(-9, 10, n)
    same = rng.random(n) < 0.3
    q["pred_x"][same] = q["mv_x"][same]
    q["pred_y"][same] = q["mv_y"][same]
    q["lambda_h"] = rng.choice(np.array([0, 4, 187, 400, 4000]), n)
    q["lambda_q"] = rng.choice(np.array([0, 4, 187, 400, 4000]), n)
    q["variant"] = rng.integers(0, 2, n)
    q["metric_h"] = rng.integers(0, 3, n)
    q["metric_q"] = rng.integers(0, 3, n)
    q["start_hp"] = rng.integers(0, 2, n)
    q["start_qp"] = rng.integers(0, 2, n)
    q["search_pos2"] = rng.choice(np.array([9, 9, 9, 5, 1, 0]), n)
    q["search_pos4"] = rng.choice(np.array([9, 9, 9, 5, 1, 0]), n)
    # finite bounds as well as DISTBLK_MAX: JM's early-exit return values matter then
    q["min_mcost"] = np.where(rng.random(n) < 0.5, DISTBLK_MAX, rng.integers(0, 60000, n) * 32)
    q["subthres"] = rng.integers(0, 4, n) * 2048 * 32
    t8 = (bsx >= 8) & (bsy >= 8) & (rng.random(n) < 0.5)
    q["flags"] = np.where(t8, SP_TEST8x8, 0) | np.where(rng.random(n) < 0.5, SP_CHECK0, 0)
    return q


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_refinement_random_vs_oracle(gpu, seed):
    from jmme import MotionEstimator
    rng = np.random.default_rng(seed)
    h, w = (144, 176) if seed != 3 else (288, 352)
    cur = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    # reference = shifted, noisy current so refinements find real minima
    ref = np.clip(np.roll(cur, (3, -2), (0, 1)).astype(np.int32) + rng.integers(-6, 7, size=(h, w)), 0, 255)
    ref = ref.astype(np.uint8)
    q = random_requests(rng, 6000, w, h)
    with MotionEstimator() as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        got = me.subpel_refine(q)
    mv, cost = oracle_run(cur, ref, q)
    bad = np.nonzero((got["mv_x"] != mv[:, 0]) | (got["mv_y"] != mv[:, 1]) | (got["cost"] != cost))[0]
    assert len(bad) == 0, (len(bad), q[bad[:3]], got[bad[:3]], mv[bad[:3]], cost[bad[:3]])


def test_chained_integer_then_subpel(gpu):
    """jmme_search_mbs_async -> jmme_subpel_refine_async with d_int: the refinement
    takes the integer results on the device (mv_search.c:960-976)."""
    import torch
    from jmme import (BLOCK_RES, DISTBLK_MAX, FULL_SEARCH, MB_REQ, NSLOT, SP_TEST8x8, SUBPEL_REQ, MotionEstimator,
                      slot_of, synth)
    w, h, R = 176, 144, 16
    luma = synth.luma_sequence(w, h, 2, seed=31, gmv=(3, -2))
    mbs = [(x, y) for y in range(0, h, 16) for x in range(0, w, 16)]
    req = np.zeros(len(mbs), MB_REQ)
    req["mb_x"] = [m[0] for m in mbs]
    req["mb_y"] = [m[1] for m in mbs]
    req["slot_mask"] = (1 << NSLOT) - 1
    req["blk"]["search_range"] = R
    req["blk"]["lambda"] = 187
    req["blk"]["pred_x"] = -12
    req["blk"]["pred_y"] = 8
    req["blk"]["center_x"] = -12
    req["blk"]["center_y"] = 8
    sq = np.zeros(len(mbs) * NSLOT, SUBPEL_REQ)
    for u, (x, y) in enumerate(mbs):
        for bt in range(1, 8):
            bw = 16 if bt <= 2 else 8 if bt <= 5 else 4
            bh = 16 if bt in (1, 3) else 8 if bt in (2, 4, 6) else 4
            for by in range(0, 16, bh):
                for bx in range(0, 16, bw):
                    s = slot_of(bt, bx // 4, by // 4)
                    e = sq[u * NSLOT + s]
                    e["pos_x"], e["pos_y"], e["blocktype"] = x + bx, y + by, bt
                    e["pred_x"], e["pred_y"] = -11, 9
                    e["lambda_h"] = e["lambda_q"] = 187
                    e["metric_h"] = e["metric_q"] = 2
                    e["start_hp"], e["start_qp"] = 0, 1
                    e["search_pos2"] = e["search_pos4"] = 9
                    e["flags"] = SP_TEST8x8 if bt <= 4 else 0
                    sq[u * NSLOT + s] = e
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        ints = me.search(FULL_SEARCH, req).reshape(-1)
        me.subpel_validate(sq)
        d_req = torch.from_numpy(req.view(np.uint8).copy()).to(gpu)
        d_int = torch.zeros(len(mbs) * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=gpu)
        d_sq = torch.from_numpy(sq.view(np.uint8).copy()).to(gpu)
        d_out = torch.zeros_like(d_int)
        stream = torch.cuda.current_stream().cuda_stream
        me.search_async(FULL_SEARCH, d_req.data_ptr(), len(mbs), d_int.data_ptr(), stream)
        me.subpel_refine_async(d_sq.data_ptr(), len(sq), d_int.data_ptr(), d_out.data_ptr(), stream)
        torch.cuda.synchronize()
        got = d_out.cpu().numpy().view(BLOCK_RES)
    q = sq.copy()
    q["mv_x"], q["mv_y"] = ints["mv_x"], ints["mv_y"]
    q["min_mcost"] = DISTBLK_MAX   # start_hp 0: BlockMotionSearch passes max_value (mv_search.c:971)
    mv, cost = oracle_run(luma[1], luma[0], q)
    assert np.array_equal(got["mv_x"], mv[:, 0]) and np.array_equal(got["mv_y"], mv[:, 1])
    assert np.array_equal(got["cost"], cost)


def test_refine_rejects_bad_requests(gpu):
    from jmme import JmmeError, MotionEstimator, SP_TEST8x8, SUBPEL_REQ
    cur = np.zeros((32, 32), np.uint8)
    with MotionEstimator() as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, cur)
        good = np.zeros(1, SUBPEL_REQ)
        good["blocktype"] = 1
        good["search_pos2"] = good["search_pos4"] = 9
        me.subpel_validate(good)
        for field, val in [("blocktype", 8), ("pos_x", 20), ("pos_x", 2), ("ref_slot", 1), ("variant", 2),
                           ("metric_h", 3), ("search_pos2", 10), ("min_mcost", -1)]:
            b = good.copy()
            b[field] = val
            with pytest.raises(JmmeError):
                me.subpel_refine(b)
        b = good.copy()
        b["blocktype"] = 5
        b["flags"] = SP_TEST8x8
        with pytest.raises(JmmeError):
            me.subpel_refine(b)
