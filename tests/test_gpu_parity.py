"""HIP path (libjmme.so on gfx950) against JM 18.5: bit-exact MVs and costs.

Every call goes through the C ABI (include/jmme.h).  The expected values are
the (mv, cost) JM 18.5 itself returned (tests/golden/, captured from the
unmodified encoder), or -- for inputs no JM run produced -- the CPU oracle,
which test_oracle_golden.py pins against those same JM captures.
"""
import numpy as np
import pytest

import golden_io as g
import oracle_lib as ol

pytestmark = pytest.mark.gpu

CASES = g.cases()


def _engine(case, gpu):
    from jmme import MotionEstimator
    ov = g.manifest()[case.name]["cfg_overrides"]
    cfg = {"SearchRange": ov["SearchRange"], "SearchMode": ov["SearchMode"]}
    if case.bits > 8:   # a high-bit-depth capture (JM's uint16 planes hold `bits`-bit samples)
        cfg["SourceBitDepthLuma"] = case.bits
    return MotionEstimator(cfg)


def _run_case(c, me, mode):
    n_ok = n = 0
    for f, lst, rf, idx in c.groups():
        me.upload_cur(c.cur[f])
        me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
        req, unit_of, slots = c.units(idx, mode)
        out = me.search(mode, req)
        res = out[unit_of, slots]
        ok = ((res["mv_x"] == c.r["out_mv_x"][idx]) & (res["mv_y"] == c.r["out_mv_y"][idx]) &
              (res["cost"] == c.r["out_cost"][idx]))
        if not ok.all():
            k = np.nonzero(~ok)[0][:5]
            detail = [(int(idx[i]), int(unit_of[i]), int(slots[i]), (int(res["mv_x"][i]), int(res["mv_y"][i]),
                       int(res["cost"][i])), (int(c.r["out_mv_x"][idx[i]]), int(c.r["out_mv_y"][idx[i]]),
                       int(c.r["out_cost"][idx[i]]))) for i in k]
            raise AssertionError(f"{c.name} frame {f} ref {rf}: {(~ok).sum()}/{len(idx)} differ: {detail}")
        n_ok += int(ok.sum())
        n += len(idx)
    return n_ok, n


@pytest.mark.parametrize("name", CASES)
def test_hip_matches_jm_golden(name, gpu):
    c = g.Case(name)
    mode = g.manifest()[name]["cfg_overrides"]["SearchMode"]
    with _engine(c, gpu) as me:
        n_ok, n = _run_case(c, me, mode)
    assert n_ok == n == c.n


def test_partial_slot_masks_and_shuffled_units(gpu):
    """Units carrying any subset of partitions, in any order, give the same
    per-partition answers (the grouping by window / predictor is exact)."""
    from jmme import FULL_SEARCH
    c = g.Case("syn_cif_adv_fs32")
    rng = np.random.default_rng(3)
    with _engine(c, gpu) as me:
        for f, lst, rf, idx in c.groups():
            me.upload_cur(c.cur[f])
            me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
            req, unit_of, slots = c.units(idx, FULL_SEARCH)
            keep = rng.random(len(idx)) < 0.35
            for u in range(len(req)):
                m = 0
                for k in np.nonzero((unit_of == u) & keep)[0]:
                    m |= 1 << int(slots[k])
                req["slot_mask"][u] = m
            perm = rng.permutation(len(req))
            out = me.search(FULL_SEARCH, req[perm])
            inv = np.argsort(perm)
            res = out[inv[unit_of], slots]
            sel = keep
            assert np.array_equal(res["mv_x"][sel], c.r["out_mv_x"][idx][sel])
            assert np.array_equal(res["mv_y"][sel], c.r["out_mv_y"][idx][sel])
            assert np.array_equal(res["cost"][sel], c.r["out_cost"][idx][sel])


def test_several_references_in_one_launch(gpu):
    """All refs of a frame are uploaded once and their units searched in one call."""
    from jmme import FULL_SEARCH, MB_REQ
    c = g.Case("syn_cif_fs32_rdo0_3ref")
    with _engine(c, gpu) as me:
        frames = sorted({f for f, _, _, _ in c.groups()})
        f = frames[-1]
        groups = [(lst, rf, idx) for ff, lst, rf, idx in c.groups() if ff == f]
        assert len(groups) >= 3
        me.upload_cur(c.cur[f])
        reqs, maps = [], []
        for lst, rf, idx in groups:
            me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
            req, unit_of, slots = c.units(idx, FULL_SEARCH)
            maps.append((idx, unit_of + sum(len(x) for x in reqs), slots))
            reqs.append(req)
        out = me.search(FULL_SEARCH, np.concatenate(reqs).astype(MB_REQ))
        for idx, unit_of, slots in maps:
            res = out[unit_of, slots]
            assert np.array_equal(res["cost"], c.r["out_cost"][idx])
            assert np.array_equal(res["mv_x"], c.r["out_mv_x"][idx])
            assert np.array_equal(res["mv_y"], c.r["out_mv_y"][idx])


def test_intpelme_signature_dropin(gpu):
    """jmme_full_search_block = full_search_motion_estimation's contract."""
    c = g.Case("c1_foreman_qcif_fs16_rdo0")
    r = c.r
    with _engine(c, gpu) as me:
        f, lst, rf, idx = next(iter(c.groups()))
        me.upload_cur(c.cur[f])
        me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
        rng = np.random.default_rng(0)
        for j in rng.choice(idx, 60, replace=False):
            mv, cost = me.full_search_block(lst, rf, r["pos_x"][j], r["pos_y"][j], r["blocktype"][j],
                                            (r["pred_x"][j], r["pred_y"][j]), (r["center_x"][j], r["center_y"][j]),
                                            r["lambda"][j], c.fs_search_range(np.array([j]))[0],
                                            c.fs_check_for_00(np.array([j]))[0])
            assert mv == (r["out_mv_x"][j], r["out_mv_y"][j]) and cost == r["out_cost"][j]


def test_ffs_intpelme_signature_dropin(gpu):
    """jmme_fast_full_search_block = fast_full_search_motion_estimation's contract
    (with setup_fast_full_search's centre / surface range), on JM's own records."""
    for name in ("ffs_foreman_qcif_r16", "ffs_foreman_qcif_r16_rdo0"):
        c = g.Case(name)
        r = c.r
        with _engine(c, gpu) as me:
            f, lst, rf, idx = next(iter(c.groups()))
            me.upload_cur(c.cur[f])
            me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
            rng = np.random.default_rng(1)
            for j in rng.choice(idx, 40, replace=False):
                mv, cost = me.fast_full_search_block(
                    lst, rf, r["pos_x"][j], r["pos_y"][j], r["blocktype"][j], (r["pred_x"][j], r["pred_y"][j]),
                    (r["ffs_center_x"][j], r["ffs_center_y"][j]), r["ffs_max_range"][j],
                    c.ffs_block_range(np.array([j]))[0], r["rdopt"][j], r["lambda"][j])
                assert mv == (r["out_mv_x"][j], r["out_mv_y"][j]) and cost == r["out_cost"][j], (name, j)


def _random_units(rng, w, h, n, R, lam_max=400, mode=-1):
    from jmme import MB_REQ, BLK_CHECK00
    req = np.zeros(n, dtype=MB_REQ)
    req["mb_x"] = rng.integers(0, w // 16, n) * 16
    req["mb_y"] = rng.integers(0, h // 16, n) * 16
    req["slot_mask"] = (1 << 41) - 1
    for u in range(n):
        base = rng.integers(-3 * R, 3 * R + 1, size=2) * 4
        for s in range(41):
            b = req["blk"][u, s]
            cen = base + rng.integers(-2, 3, size=2) * 4 * (rng.random() < 0.3)
            b["center_x"], b["center_y"] = cen
            b["pred_x"], b["pred_y"] = cen + rng.integers(-9, 10, size=2)
            b["search_range"] = R
            b["lambda"] = rng.integers(0, lam_max)
            b["flags"] = BLK_CHECK00 if s == 0 and rng.random() < 0.5 else 0
            req["blk"][u, s] = b
    return req


def _oracle_units(cur, ref, req):
    """Oracle answers for every slot of every unit (FS)."""
    from jmme import slot_of
    rows, keys = [], []
    geo = {}
    for bt, (bw, bh) in {1: (16, 16), 2: (16, 8), 3: (8, 16), 4: (8, 8), 5: (8, 4), 6: (4, 8), 7: (4, 4)}.items():
        for by in range(0, 16, bh):
            for bx in range(0, 16, bw):
                geo[slot_of(bt, bx // 4, by // 4)] = (bx, by, bw, bh)
    for u, q in enumerate(req):
        for s in range(41):
            if not (int(q["slot_mask"]) >> s) & 1:
                continue
            b = q["blk"][s]
            bx, by, bw, bh = geo[s]
            rows.append([q["mb_x"] + bx, q["mb_y"] + by, bw, bh, b["pred_x"], b["pred_y"], b["center_x"],
                         b["center_y"], b["search_range"], b["lambda"], int(b["flags"] & 1)])
            keys.append((u, s))
    mv, cost = ol.full_search_batch(cur, ref, np.array(rows, np.int32))
    return keys, mv, cost


@pytest.mark.parametrize("size,R,n", [((3840, 2160), 32, 24), ((1920, 1088), 16, 24), ((352, 288), 44, 24),
                                      ((176, 144), 0, 24), ((256, 64), 16, 200), ((128, 48), 8, 150)])
def test_random_requests_vs_oracle(size, R, n, gpu):
    """Inputs no JM run produced (4K, unusual ranges, centres far outside the
    picture, mixed windows per MB): HIP == oracle on every partition.  The
    narrow pictures (16 and 8 macroblocks a row) deal items to the XCDs in
    column stripes of 2 and 1 items rotating every 8 rounds, over many rounds
    and a partial last one: every unit must still be served exactly once."""
    from jmme import FULL_SEARCH, MotionEstimator
    from jmme import synth
    w, h = size
    rng = np.random.default_rng(R + w)
    luma = synth.luma_sequence(w, h, 2, seed=w + R, gmv=(3, -2))
    cur, ref = luma[1], luma[0]
    req = _random_units(rng, w, h, n, R)
    with MotionEstimator({"SearchRange": max(R, 1), "SearchMode": -1}) as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FULL_SEARCH, req)
    keys, mv, cost = _oracle_units(cur, ref, req)
    got = np.array([(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u, s in keys])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(keys[i], got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


def _ffs_random(rng, w, h, n, R, rdopt, far_frac):
    """n FFS units (all 41 partitions): surface centre, per-partition ranges at
    or below the surface's, predictors near the window or -- for far_frac of
    the partitions -- beyond JM's GetMaxMVD gate (me_fullfast.c:637,663); with
    RDO off the centre stays within +-R so that (0,0) is in the window, as
    setup_fast_full_search clips it (me_fullfast.c:319-324)."""
    from jmme import MB_REQ, slot_of
    geo = {}
    for bt, (bw, bh) in {1: (16, 16), 2: (16, 8), 3: (8, 16), 4: (8, 8), 5: (8, 4), 6: (4, 8), 7: (4, 4)}.items():
        for by in range(0, 16, bh):
            for bx in range(0, 16, bw):
                geo[slot_of(bt, bx // 4, by // 4)] = (bt, bx // 4, by // 4)
    req = np.zeros(n, dtype=MB_REQ)
    req["mb_x"] = rng.integers(0, w // 16, n) * 16
    req["mb_y"] = rng.integers(0, h // 16, n) * 16
    req["slot_mask"] = (1 << 41) - 1
    span = R if rdopt == 0 else 3 * R
    req["ffs_center_x"] = rng.integers(-span, span + 1, n) * 4
    req["ffs_center_y"] = rng.integers(-span, span + 1, n) * 4
    req["ffs_range"] = R
    req["ffs_pos00_valid"] = 1 if rdopt == 0 else 0
    mbs, blk = [], []
    for u in range(n):
        cx, cy = int(req["ffs_center_x"][u]), int(req["ffs_center_y"][u])
        mbs.append([int(req["mb_x"][u]), int(req["mb_y"][u]), cx, cy])
        # pos_00: the (0,0) vector's index in the surface's spiral (me_fullfast.c:353-365)
        ox, oy = -cx // 4, -cy // 4
        pos00 = int(np.nonzero((SPIRAL[R][:, 0] == ox) & (SPIRAL[R][:, 1] == oy))[0][0]) if max(abs(ox), abs(oy)) <= R else 0
        for sl in range(41):
            b = req["blk"][u, sl]
            far = rng.random() < far_frac
            d = rng.integers(-700, 701, size=2) if far else rng.integers(-9 * R, 9 * R + 1, size=2)
            b["pred_x"], b["pred_y"] = cx + d[0], cy + d[1]
            b["search_range"] = R if rng.random() < 0.6 else rng.integers(0, R + 1)
            b["lambda"] = rng.integers(0, 400)
            req["blk"][u, sl] = b
            bt, bx, by = geo[sl]
            blk.append([u, bt, bx, by, int(b["pred_x"]), int(b["pred_y"]), int(b["search_range"]), int(b["lambda"]),
                        pos00])
    return req, np.array(mbs, np.int32), np.array(blk, np.int32)


SPIRAL = {R: ol.spiral(R) for R in (8, 16, 32)}


@pytest.mark.parametrize("R,rdopt,far", [(16, 0, 0.0), (16, 1, 0.0), (32, 0, 0.3), (8, 1, 0.5)])
def test_ffs_random_requests_vs_oracle(R, rdopt, far, gpu):
    """Fast full search on inputs no JM run produced: surface centres across
    the window, partitions with their own smaller ranges, the (0,0) pre-seed
    on and off, predictors the GetMaxMVD gate cuts (the kernel's exact path):
    HIP == oracle (ora_ffs_batch, pinned to JM's FFS captures) on every partition."""
    from jmme import FAST_FULL_SEARCH, MotionEstimator
    from jmme import synth
    w, h = 352, 288
    rng = np.random.default_rng(100 * R + 10 * rdopt + int(10 * far))
    luma = synth.luma_sequence(w, h, 2, seed=R + rdopt, gmv=(3, -2))
    cur, ref = luma[1], luma[0]
    req, mbs, blk = _ffs_random(rng, w, h, 16, R, rdopt, far)
    with MotionEstimator({"SearchRange": R, "SearchMode": 0, "RDOptimization": rdopt}) as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FAST_FULL_SEARCH, req)
        max_mvd = me.max_mvd
    mv, cost = ol.ffs_batch(cur, ref, R, max_mvd, rdopt, mbs, blk)
    got = np.array([(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u in range(len(req))
                    for s in range(41)])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(divmod(int(i), 41), got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


@pytest.mark.parametrize("path", ["items", "small"])
def test_saturated_32bit_keys_take_the_64bit_path(path, gpu):
    """Huge lambdas push every candidate of the small partitions past the
    32-bit key's cost field; the deferred 64-bit pass must keep results exact.
    `items` forces the throughput kernel (small-batch limit 0), whose 64-bit
    keys and exact re-search this guards; `small` is the latency path."""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    w, h, R = 352, 288, 16
    rng = np.random.default_rng(9)
    luma = synth.luma_sequence(w, h, 2, seed=4)
    req = _random_units(rng, w, h, 6, R)
    req["blk"]["lambda"] = 400000
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.set_small_batch_limit(0 if path == "items" else 1 << 20)
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        out = me.search(FULL_SEARCH, req)
    keys, mv, cost = _oracle_units(luma[1], luma[0], req)
    for i, (u, s) in enumerate(keys):
        assert (out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) == (mv[i, 0], mv[i, 1], cost[i])


@pytest.mark.parametrize("path", ["items", "small"])
@pytest.mark.parametrize("scene", ["flat", "inverted"])
def test_saturated_16x16_keys_are_searched_exactly(scene, path, gpu):
    """Lambdas just inside the 32-bit key range on pictures whose 16x16 SADs
    reach (flat: equal) 65280: every 16x16 key of the sweep saturates, so the
    16x16 result comes from the exact 64-bit re-search; the other partitions
    stay on the 32-bit keys.  HIP == oracle on every partition."""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    w, h, R = 176, 144, 8
    rng = np.random.default_rng(17)
    if scene == "flat":
        cur = np.full((h, w), 255, np.uint8)
        ref = np.zeros((h, w), np.uint8)
    else:
        ref = synth.luma_sequence(w, h, 1, seed=6)[0]
        ref = np.where(ref > 127, 255, 0).astype(np.uint8)
        cur = (255 - ref).astype(np.uint8)
    req = _random_units(rng, w, h, 8, R)
    req["blk"]["lambda"] = rng.integers(13000, 14226, size=req["blk"]["lambda"].shape)
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.set_small_batch_limit(0 if path == "items" else 1 << 20)
        me.upload_cur(cur)
        me.upload_ref(0, 0, ref)
        out = me.search(FULL_SEARCH, req)
    keys, mv, cost = _oracle_units(cur, ref, req)
    got = np.array([(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u, s in keys])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(keys[i], got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


def test_requests_outside_contract_are_rejected(gpu):
    from jmme import FULL_SEARCH, JmmeError, MotionEstimator, MB_REQ, synth
    luma = synth.luma_sequence(176, 144, 2, seed=1)
    with MotionEstimator({"SearchRange": 8, "SearchMode": -1}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        req = np.zeros(1, dtype=MB_REQ)
        req["slot_mask"] = 1
        req["blk"][0, 0]["search_range"] = 9           # > SearchRange
        with pytest.raises(JmmeError):
            me.search(FULL_SEARCH, req)
        req["blk"][0, 0]["search_range"] = 8
        req["blk"][0, 0]["center_x"] = 2                # sub-pel centre (EPZSSubPelGrid)
        with pytest.raises(JmmeError):
            me.search(FULL_SEARCH, req)
        req["blk"][0, 0]["center_x"] = 0
        req["ref_idx"] = 3                              # never uploaded
        with pytest.raises(JmmeError):
            me.search(FULL_SEARCH, req)
        with pytest.raises(JmmeError):
            me.upload_ref(0, 1, np.full((144, 176), 300, np.uint16))  # not 8-bit


@pytest.mark.parametrize("mb,cen", [((0, 0), (0, 0)), ((16, 0), (0, 0)), ((48, 32), (-12, 8)),
                                    ((160, 128), (20, 16)), ((80, 64), (400, -400))])
def test_staged_window_is_the_clamped_reference(mb, cen, gpu):
    """The LDS window the kernel searches equals the reference clamped into the
    picture (UMVLine4X over JM's edge-replicated padding, refbuf.h:22-26)."""
    import ctypes
    from jmme import FULL_SEARCH, MB_REQ, MotionEstimator, synth, _lib
    W, H, R = 176, 144, 16
    luma = synth.luma_sequence(W, H, 2, seed=8)
    req = np.zeros(1, dtype=MB_REQ)
    req["mb_x"], req["mb_y"] = mb
    req["slot_mask"] = 1
    req["blk"][0, 0]["center_x"], req["blk"][0, 0]["center_y"] = cen
    req["blk"][0, 0]["search_range"] = R
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        wp = 2 * R + 13
        out = np.zeros((2 * R + 16) * wp, np.uint32)
        _lib.check(_lib.lib().jmme_debug_window(me._ctx, FULL_SEARCH, _lib.ptr(req), _lib.ptr(out), out.size))
    out = out.reshape(2 * R + 16, wp)
    x0 = mb[0] + cen[0] // 4 - R
    y0 = mb[1] + cen[1] // 4 - R
    ys = np.clip(np.arange(y0, y0 + 2 * R + 16), 0, H - 1)
    exp = np.zeros((2 * R + 16, 2 * R + 13), np.uint32)
    for b in range(4):
        xs = np.clip(np.arange(x0 + b, x0 + b + 2 * R + 13), 0, W - 1)
        exp |= luma[0][np.ix_(ys, xs)].astype(np.uint32) << np.uint32(8 * b)
    bad = np.argwhere(out[:, :2 * R + 13] != exp)
    assert len(bad) == 0, (len(bad), bad[:5].tolist())


def _grouped_units(rng, w, h, n, R, lam):
    """Units whose 41 partitions share one of 3 (centre, predictor, lambda)
    triples at random, so the plan kernel's groups have sparse, non-contiguous
    slot masks (e.g. slots {0, 2, 7, ...} in one group)."""
    from jmme import MB_REQ
    req = np.zeros(n, dtype=MB_REQ)
    req["mb_x"] = rng.integers(0, w // 16, n) * 16
    req["mb_y"] = rng.integers(0, h // 16, n) * 16
    req["slot_mask"] = (1 << 41) - 1
    for u in range(n):
        trip = []
        for _ in range(3):
            cen = rng.integers(-2 * R - 2, 2 * R + 3, size=2) * 4
            trip.append((cen, cen + rng.integers(-9, 10, size=2), lam + int(rng.integers(0, 500))))
        pick = rng.integers(0, 3, 41)
        for s in range(41):
            cen, pred, lm = trip[pick[s]]
            b = req["blk"][u, s]
            b["center_x"], b["center_y"] = cen
            b["pred_x"], b["pred_y"] = pred
            b["search_range"] = R
            b["lambda"] = lm
            req["blk"][u, s] = b
    return req


@pytest.mark.parametrize("path", ["items", "small"])
@pytest.mark.parametrize("R", [1, 7, 23, 44])
def test_64bit_path_with_sparse_group_masks(R, path, gpu):
    """Lambdas beyond the 32-bit keys send every partition through the exact
    64-bit search, one partition after another; groups with non-contiguous slot
    masks make consecutive calls land on slots of equal parity, and the odd
    halves of the exchange buffer sit at the end of the workgroup's LDS.  Every
    SearchRange changes where that end falls.  HIP == oracle on every partition,
    on the item kernel (`items`: small-batch limit 0) and the latency path."""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    w, h = 352, 288
    rng = np.random.default_rng(40 + R)
    luma = synth.luma_sequence(w, h, 2, seed=R, gmv=(2, 1))
    req = _grouped_units(rng, w, h, 8, R, 400000)
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.set_small_batch_limit(0 if path == "items" else 1 << 20)
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        out = me.search(FULL_SEARCH, req)
    keys, mv, cost = _oracle_units(luma[1], luma[0], req)
    got = np.array([(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u, s in keys])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(keys[i], got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


def test_small_batch_with_wrapping_lambda_goes_to_the_item_kernel(gpu):
    """A few units (the small path's size) with lambda ~7e7: the small kernel's
    exact 32-bit cost (SAD << 5) + lambda * mvbits would wrap, so the batch must
    go to the item kernel's 64-bit keys.  HIP == oracle."""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    w, h, R = 176, 144, 8
    rng = np.random.default_rng(77)
    luma = synth.luma_sequence(w, h, 2, seed=12, gmv=(1, 2))
    req = _random_units(rng, w, h, 3, R)
    req["blk"]["lambda"] = rng.integers(67_200_000, 90_000_000, size=req["blk"]["lambda"].shape)
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.set_small_batch_limit(1 << 20)
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        out = me.search(FULL_SEARCH, req)
    keys, mv, cost = _oracle_units(luma[1], luma[0], req)
    got = np.array([(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u, s in keys])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(keys[i], got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


def test_device_requests_outside_contract_are_refused(gpu):
    """The device-request path skips the host validation: the plan kernel must
    refuse an FFS partition whose own range exceeds its surface's (it would
    index past the position tables and the staged window) and report it."""
    import torch
    from jmme import FAST_FULL_SEARCH, FULL_SEARCH, JmmeError, MB_REQ, NSLOT, BLOCK_RES, MotionEstimator, synth
    luma = synth.luma_sequence(176, 144, 2, seed=2)
    req = np.zeros(2, dtype=MB_REQ)
    req["mb_x"] = [16, 64]
    req["mb_y"] = [32, 48]
    req["slot_mask"] = (1 << 41) - 1
    req["ffs_range"] = 8
    req["blk"]["search_range"] = 8
    req["blk"]["lambda"] = 100
    with MotionEstimator({"SearchRange": 16, "SearchMode": 0}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        dev = torch.device("cuda:0")
        d_out = torch.zeros(2 * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=dev)

        def run(r, mode):
            d_req = torch.from_numpy(r.view(np.uint8).copy()).to(dev)
            me.search_async(mode, d_req.data_ptr(), len(r), d_out.data_ptr())
            me.search_status()

        run(req, FAST_FULL_SEARCH)                      # within contract: no error
        bad = req.copy()
        bad["blk"][1, 17]["search_range"] = 12           # block range 12 > surface range 8
        with pytest.raises(JmmeError):
            run(bad, FAST_FULL_SEARCH)
        run(req, FAST_FULL_SEARCH)                      # status is per launch
        fs = req.copy()
        fs["blk"][0, 3]["center_x"] = 6                  # sub-pel centre on the FS path
        with pytest.raises(JmmeError):
            run(fs, FULL_SEARCH)


def test_planes_must_be_dword_aligned(gpu):
    import torch
    from jmme import FULL_SEARCH, JmmeError, MB_REQ, NSLOT, BLOCK_RES, MotionEstimator
    dev = torch.device("cuda:0")
    plane = torch.zeros(144 * 176 + 8, dtype=torch.uint8, device=dev)
    req = np.zeros(1, dtype=MB_REQ)
    req["slot_mask"] = 1
    req["blk"][0, 0]["search_range"] = 4
    d_req = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=dev)
    with MotionEstimator({"SearchRange": 4, "SearchMode": -1}) as me:
        me.search_planes_async(FULL_SEARCH, plane.data_ptr(), plane.data_ptr(), 176, 176, 144,
                               d_req.data_ptr(), 1, d_out.data_ptr())
        me.search_status()
        with pytest.raises(JmmeError):
            me.search_planes_async(FULL_SEARCH, plane.data_ptr() + 1, plane.data_ptr(), 176, 176, 144,
                                   d_req.data_ptr(), 1, d_out.data_ptr())


# ---- the low-latency small-batch path (jmme_set_small_batch_limit) -------------
@pytest.mark.parametrize("name", ["c1_foreman_qcif_fs16", "c1_foreman_qcif_fs16_rdo0", "ffs_foreman_qcif_r16",
                                  "ffs_foreman_qcif_r16_rdo0", "syn_cif_adv_fs32", "syn_cif_ffs32_rdo0_3ref"])
def test_small_batches_match_jm_golden(name, gpu):
    """JM's own searches sent three macroblocks at a time, as the drop-in's
    speculative batches after a failed guess are: every call takes the
    small-batch kernel, every result equals JM's."""
    c = g.Case(name)
    mode = g.manifest()[name]["cfg_overrides"]["SearchMode"]
    with _engine(c, gpu) as me:
        me.set_small_batch_limit(1 << 20)
        n = 0
        for f, lst, rf, idx in c.groups():
            me.upload_cur(c.cur[f])
            me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
            req, unit_of, slots = c.units(idx, mode)
            out = np.zeros((len(req), 41), dtype=me.search(mode, req[:1]).dtype)
            for a in range(0, len(req), 3):
                out[a:a + 3] = me.search(mode, req[a:a + 3])
            res = out[unit_of, slots]
            assert np.array_equal(res["mv_x"], c.r["out_mv_x"][idx]), name
            assert np.array_equal(res["mv_y"], c.r["out_mv_y"][idx]), name
            assert np.array_equal(res["cost"], c.r["out_cost"][idx]), name
            n += len(idx)
    assert n == c.n


@pytest.mark.parametrize("size,R,lam", [((3840, 2160), 32, 400), ((352, 288), 44, 400), ((176, 144), 0, 400),
                                        ((352, 288), 16, 400000), ((1920, 1088), 64, 400)])
def test_small_path_equals_throughput_path_fs(size, R, lam, gpu):
    """Random FS units (centres far outside the picture, mixed windows and
    predictors per MB, check_for_00, huge lambdas, R up to 64): the small-batch
    kernel, the throughput kernels and the oracle agree on every partition."""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    w, h = size
    rng = np.random.default_rng(R + w + lam)
    luma = synth.luma_sequence(w, h, 2, seed=w + R, gmv=(3, -2))
    req = _random_units(rng, w, h, 6, R, lam_max=lam)
    with MotionEstimator({"SearchRange": max(R, 1), "SearchMode": -1}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        me.set_small_batch_limit(1 << 20)
        small = me.search(FULL_SEARCH, req)
        me.set_small_batch_limit(0)
        big = me.search(FULL_SEARCH, req)
    assert small.tobytes() == big.tobytes()
    keys, mv, cost = _oracle_units(luma[1], luma[0], req)
    got = np.array([(small[u, s]["mv_x"], small[u, s]["mv_y"], small[u, s]["cost"]) for u, s in keys])
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost])
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, [(keys[i], got[i].tolist(), exp[i].tolist()) for i in bad[:5]]


@pytest.mark.parametrize("R,rdopt,far", [(16, 0, 0.0), (16, 1, 0.3), (32, 0, 0.3), (8, 1, 0.5)])
def test_small_path_equals_throughput_path_ffs(R, rdopt, far, gpu):
    from jmme import FAST_FULL_SEARCH, MotionEstimator
    from jmme import synth
    w, h = 352, 288
    rng = np.random.default_rng(7 * R + rdopt)
    luma = synth.luma_sequence(w, h, 2, seed=R + 5, gmv=(3, -2))
    req, mbs, blk = _ffs_random(rng, w, h, 4, R, rdopt, far)
    with MotionEstimator({"SearchRange": R, "SearchMode": 0, "RDOptimization": rdopt}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        me.set_small_batch_limit(1 << 20)
        small = me.search(FAST_FULL_SEARCH, req)
        me.set_small_batch_limit(0)
        big = me.search(FAST_FULL_SEARCH, req)
        max_mvd = me.max_mvd
    assert small.tobytes() == big.tobytes()
    mv, cost = ol.ffs_batch(luma[1], luma[0], R, max_mvd, rdopt, mbs, blk)
    got = np.array([(small[u, s]["mv_x"], small[u, s]["mv_y"], small[u, s]["cost"]) for u in range(len(req))
                    for s in range(41)])
    assert np.array_equal(got, np.column_stack([mv[:, 0], mv[:, 1], cost]))
