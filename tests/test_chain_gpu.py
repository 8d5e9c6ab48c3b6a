"""GPU: chained partition searches (jmme_search_mbs_chains).  Each step's
predictor and centre are derived on the device from the chain's neighbours and
the previous steps' answers; here the same derivation is restated in Python
(GetMotionVectorPredictorNormal, JM/lcommon/src/mv_prediction.c:192-300;
BlockMotionSearch's centre, JM/lencod/src/mv_search.c:930-956; CheckSearchRange
:822-848; clip_mv_range, conformance.c:463-469) and every step is searched on
its own through jmme_search_mbs (itself bit-exact vs JM and the oracle).  The
chain must reproduce the derived inputs and the answers step by step."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GEOM = {}   # slot -> (bx, by, w, h) in 4x4 units


def _geom():
    from jmme import slot_of
    if not GEOM:
        for bt, (w, h) in {1: (4, 4), 2: (4, 2), 3: (2, 4), 4: (2, 2), 5: (2, 1), 6: (1, 2), 7: (1, 1)}.items():
            for by in range(0, 4, h):
                for bx in range(0, 4, w):
                    GEOM[slot_of(bt, bx, by)] = (bx, by, w, h)
    return GEOM


def _median(a, b, c):
    return sorted((a, b, c))[1]


def derive(chain, k, prev, max_mvd):
    """(pred, centre, range_min, range_max) of step k; prev[j] = step j's clipped answer"""
    st = chain["steps"][k]
    bx, by, w, h = _geom()[int(st["slot"])]
    r = int(chain["ref_idx"])
    av, rf, mv = [], [], []
    for nb in st["nb"]:
        src = int(nb["src"])
        av.append(src != -1)
        if src >= 0:
            rf.append(r)
            mv.append(prev[src])
        else:
            rf.append(int(nb["ref_idx"]))
            mv.append((int(nb["mv_x"]), int(nb["mv_y"])))
    rL, rU, rUR = (rf[j] if av[j] else -1 for j in range(3))
    t = 0
    if rL == r and rU != r and rUR != r:
        t = 1
    elif rL != r and rU == r and rUR != r:
        t = 2
    elif rL != r and rU != r and rUR == r:
        t = 3
    if (w, h) == (2, 4):
        if bx == 0:
            t = 1 if rL == r else t
        elif rUR == r:
            t = 3
    elif (w, h) == (4, 2):
        if by == 0:
            t = 2 if rU == r else t
        elif rL == r:
            t = 1
    if t == 0:
        if not (av[1] or av[2]):
            p = mv[0] if av[0] else (0, 0)
        else:
            z = [mv[j] if av[j] else (0, 0) for j in range(3)]
            p = (_median(*(q[0] for q in z)), _median(*(q[1] for q in z)))
    else:
        p = mv[t - 1] if av[t - 1] else (0, 0)
    cx, cy = ((p[0] + 2) >> 2) * 4, ((p[1] + 2) >> 2) * 4
    mnx, mxx, mny, mxy = (int(st[f]) for f in ("sr_min_x", "sr_max_x", "sr_min_y", "sr_max_y"))
    if not chain["rdopt"]:
        ccx, ccy = cx, cy
        cx, cy = min(max(cx, mnx), mxx), min(max(cy, mny), mxy)
        if (cx, cy) != (ccx, ccy):
            md = max_mvd - 2
            cl = lambda v, c: min(max(v, c - md), c + md)   # noqa: E731
            left, right = cl(cx + mnx, ccx), cl(cx + mxx, ccx)
            top, down = cl(cy + mny, ccy), cl(cy + mxy, ccy)
            if left < right and top < down:
                cx, cy = (left + right) >> 1, (top + down) >> 1
                mnx, mxx = left - cx, min(cx - left, right - cx)
                mny, mxy = top - cy, min(cy - top, down - cy)
            else:
                cx, cy = ccx, ccy
    cx = min(max(cx, int(chain["mv_lim_x0"])), int(chain["mv_lim_x1"]))
    cy = min(max(cy, int(chain["mv_lim_y0"])), int(chain["mv_lim_y1"]))
    return p, (cx, cy), min(mxx, mxy) >> 2, max(mxx, mxy) >> 2


def _random_chains(rng, w, h, n, R, rdopt, ffs):
    """chains of the shapes the drop-in builds: a 16x8 / 8x16 pair's second
    partition, or one sub-mode of one quadrant, neighbours fixed or in-chain"""
    from jmme._lib import CHAIN
    ch = np.zeros(n, CHAIN)
    groups = [[2], [4], [5], [9, 11], [17, 18], [25, 26, 29, 30], [27, 28, 31, 32], [13, 15], [21, 22],
              [33, 34, 37, 38], [6], [35, 36, 39, 40], [0], [0, 1, 2]]
    for i in range(n):
        c = ch[i]
        c["mb_x"] = rng.integers(0, w // 16) * 16
        c["mb_y"] = rng.integers(0, h // 16) * 16
        c["rdopt"] = rdopt
        c["lambda"] = rng.integers(0, 400)
        c["mv_lim_x0"], c["mv_lim_x1"] = -2048, 2047
        c["mv_lim_y0"], c["mv_lim_y1"] = -512, 511
        if ffs:
            c["ffs_center_x"], c["ffs_center_y"] = rng.integers(-R, R + 1, 2) * 4
            c["ffs_range"] = R
            c["ffs_pos00_valid"] = 1 - rdopt
        g = groups[rng.integers(len(groups))]
        c["n_steps"] = len(g)
        for k, slot in enumerate(g):
            st = c["steps"][k]
            st["slot"] = slot
            if slot == 0 and not ffs and rng.random() < 0.7:
                st["flags"] = 1   # JMME_CHAIN_CHECK00: check_for_00 (me_fullsearch.c:61)
            for j in range(3):
                u = rng.random()
                if k and u < 0.45:
                    st["nb"][j]["src"] = rng.integers(0, k)
                elif u < 0.55:
                    st["nb"][j]["src"] = -1
                else:
                    st["nb"][j]["src"] = -2
                    st["nb"][j]["ref_idx"] = 0 if rng.random() < 0.8 else rng.integers(-1, 3)
                    st["nb"][j]["mv_x"], st["nb"][j]["mv_y"] = rng.integers(-4 * 3 * R, 4 * 3 * R + 1, 2)
            rr = R if rng.random() < 0.7 else rng.integers(1, R + 1)
            st["sr_min_x"], st["sr_max_x"], st["sr_min_y"], st["sr_max_y"] = -4 * rr, 4 * rr, -4 * rr, 4 * rr
            c["steps"][k] = st
        ch[i] = c
    return ch


def _step_req(chain, k, pred, centre, rng_min, rng_max, ffs):
    from jmme import MB_REQ
    q = np.zeros(1, MB_REQ)
    q["mb_x"], q["mb_y"] = chain["mb_x"], chain["mb_y"]
    s = int(chain["steps"][k]["slot"])
    q["slot_mask"] = 1 << s
    b = q["blk"][0, s]
    b["pred_x"], b["pred_y"] = pred
    b["lambda"] = chain["lambda"]
    if chain["steps"][k]["flags"] & 1:
        from jmme import BLK_CHECK00
        b["flags"] = BLK_CHECK00
    if ffs:
        q["ffs_center_x"], q["ffs_center_y"] = chain["ffs_center_x"], chain["ffs_center_y"]
        q["ffs_range"], q["ffs_pos00_valid"] = chain["ffs_range"], chain["ffs_pos00_valid"]
        b["search_range"] = rng_max
    else:
        b["center_x"], b["center_y"] = centre
        b["search_range"] = rng_min
    q["blk"][0, s] = b
    return q, s


@pytest.mark.parametrize("ffs,rdopt,R,bits", [(False, 0, 16, 8), (False, 1, 32, 8), (True, 0, 16, 8), (True, 1, 32, 8),
                                              # 16-bit planes: the v_sad_u16 chain kernel against the
                                              # small kernel's 16-bit searches
                                              (False, 0, 16, 10), (True, 1, 32, 12), (False, 1, 32, 14)])
def test_chains_match_step_by_step_searches(gpu, ffs, rdopt, R, bits):
    from jmme import FAST_FULL_SEARCH, FULL_SEARCH, MB_REQ, MotionEstimator, synth
    w, h = 352, 288
    rng = np.random.default_rng(10 * R + rdopt + 100 * ffs + bits)
    luma = synth.luma_sequence(w, h, 2, seed=R + rdopt, gmv=(3, -2), adversarial=True, adv_range=R)
    if bits > 8:   # the texture scaled, plus low-order noise only a 16-bit search sees
        sh = bits - 8
        luma = ((luma.astype(np.int32) << sh) + rng.integers(0, 1 << sh, size=luma.shape)).astype(np.uint16)
    chains = _random_chains(rng, w, h, 8, R, rdopt, ffs)
    mode = FAST_FULL_SEARCH if ffs else FULL_SEARCH
    n_steps = 0
    cfg = {"SearchRange": R, "SearchMode": 0 if ffs else -1, "RDOptimization": rdopt, "SourceBitDepthLuma": bits}
    with MotionEstimator(cfg) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        _, res = me.search_chains(mode, np.zeros(0, MB_REQ), chains)
        for i, c in enumerate(chains):
            prev = []
            for k in range(int(c["n_steps"])):
                p, cen, rmin, rmax = derive(c, k, prev, me.max_mvd)
                got = res[i, k]
                if not ffs and (cen[0] | cen[1]) & 3:   # a half-way centre (CheckSearchRange): the chain stops
                    assert all(res[i, j]["cost"] == -1 for j in range(k, int(c["n_steps"]))), (i, k, res[i])
                    break
                assert (got["pred_x"], got["pred_y"]) == p, (i, k, got, p)
                assert (got["range_min"], got["range_max"]) == (rmin, rmax), (i, k, got)
                if not ffs:
                    assert (got["center_x"], got["center_y"]) == cen, (i, k, got, cen)
                q, s = _step_req(c, k, p, cen, rmin, rmax, ffs)
                exp = me.search(mode, q)[0, s]
                assert (got["mv_x"], got["mv_y"], got["cost"]) == (exp["mv_x"], exp["mv_y"], exp["cost"]), \
                    (i, k, got, exp)
                prev.append((min(max(int(exp["mv_x"]), -2048), 2047), min(max(int(exp["mv_y"]), -512), 511)))
                n_steps += 1
    assert n_steps >= 8


def test_chains_with_a_batch_in_one_call(gpu):
    """the chains ride with a batch of the same call; both answers are the plain ones"""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    from test_gpu_parity import _random_units
    w, h, R = 352, 288, 16
    rng = np.random.default_rng(7)
    luma = synth.luma_sequence(w, h, 2, seed=3, gmv=(2, 1))
    req = _random_units(rng, w, h, 3, R)
    chains = _random_chains(rng, w, h, 4, R, 0, False)
    with MotionEstimator({"SearchRange": R, "SearchMode": -1}) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        out, res = me.search_chains(FULL_SEARCH, req, chains)
        plain = me.search(FULL_SEARCH, req)
        _, res_alone = me.search_chains(FULL_SEARCH, req[:0], chains)
    assert np.array_equal(out, plain)
    assert np.array_equal(res, res_alone)


def test_chain_requests_outside_contract_are_refused(gpu):
    from jmme import FULL_SEARCH, JmmeError, MB_REQ, MotionEstimator
    from jmme._lib import CHAIN
    plane = np.zeros((64, 64), np.uint8)
    good = np.zeros(1, CHAIN)
    good["n_steps"] = 1
    good["steps"][0, 0]["slot"] = 5
    for j in range(3):
        good["steps"][0, 0]["nb"][j]["src"] = -1
    good["steps"][0, 0]["sr_min_x"] = good["steps"][0, 0]["sr_min_y"] = -16
    good["steps"][0, 0]["sr_max_x"] = good["steps"][0, 0]["sr_max_y"] = 16
    good["mv_lim_x0"], good["mv_lim_x1"], good["mv_lim_y0"], good["mv_lim_y1"] = -2048, 2047, -512, 511
    empty = np.zeros(0, MB_REQ)
    with MotionEstimator({"SearchRange": 4}) as me:
        me.upload_cur(plane)
        me.upload_ref(0, 0, plane)
        me.search_chains(FULL_SEARCH, empty, good)
        for field, val in [("n_steps", 0), ("n_steps", 5), ("mb_x", 8), ("mb_y", 64), ("ref_idx", 3)]:
            bad = good.copy()
            bad[field] = val
            with pytest.raises(JmmeError):
                me.search_chains(FULL_SEARCH, empty, bad)
        bad = good.copy()
        bad["steps"][0, 0]["flags"] = 1              # check_for_00 on a step that is not 16x16
        with pytest.raises(JmmeError):
            me.search_chains(FULL_SEARCH, empty, bad)
        bad = good.copy()
        bad["steps"][0, 0]["nb"][1]["src"] = 0      # a step cannot read itself
        with pytest.raises(JmmeError):
            me.search_chains(FULL_SEARCH, empty, bad)
        with pytest.raises(JmmeError):
            me.search_chains(FULL_SEARCH, empty, np.repeat(good, 9))


def test_prepare_and_reserve_then_search(gpu):
    """jmme_prepare (every kernel variant, chains included, on a dummy plane) and
    jmme_reserve (buffers for the largest batch, plane buffers of the configured
    size) leave the context as fresh: the first searches equal a plain context's"""
    from jmme import FULL_SEARCH, MotionEstimator, synth
    from test_gpu_parity import _random_units
    w, h, R = 352, 288, 16
    luma = synth.luma_sequence(w, h, 2, seed=11, gmv=(1, 2))
    req = _random_units(np.random.default_rng(3), w, h, 40, R)
    chains = _random_chains(np.random.default_rng(4), w, h, 4, R, 0, False)
    res = []
    for warm in (False, True):
        with MotionEstimator({"SearchRange": R, "SearchMode": -1, "SourceWidth": w, "SourceHeight": h}) as me:
            if warm:
                me.prepare(max_units=256)
            me.upload_cur(luma[1])
            me.upload_ref(0, 0, luma[0])
            res.append((me.search(FULL_SEARCH, req), *me.search_chains(FULL_SEARCH, req[:2], chains)))
    for a, b in zip(*res):
        assert np.array_equal(a, b)


def _sp_templates(rng, n, bits):
    from jmme import SUBPEL_REQ
    sp = np.zeros(n, SUBPEL_REQ)
    sp["lambda_h"] = rng.choice([0, 40, 187, 900], n)
    sp["lambda_q"] = rng.choice([0, 40, 187, 900], n)
    sp["metric_h"] = rng.integers(0, 3, n)
    sp["metric_q"] = rng.integers(0, 3, n)
    if bits > 11:   # SSE sub-pel is refused above 11 bits
        sp["metric_h"][sp["metric_h"] == 1] = 2
        sp["metric_q"][sp["metric_q"] == 1] = 0
    sp["start_hp"] = rng.integers(0, 2, n)
    sp["start_qp"] = rng.integers(0, 2, n)
    sp["search_pos2"] = rng.choice([9, 9, 5, 1], n)
    sp["search_pos4"] = rng.choice([9, 9, 5, 0], n)
    sp["flags"] = rng.choice([0, 2], n)   # JMME_SP_CHECK0
    return sp


@pytest.mark.parametrize("ffs,rdopt,R,bits", [(False, 0, 16, 8), (True, 1, 32, 8), (False, 1, 32, 8), (True, 0, 16, 10)])
def test_chains_with_subpel_match_step_by_step(gpu, ffs, rdopt, R, bits):
    """jmme_search_mbs_chains_sp: each step's integer answer equals its own
    search under the predictor derived from the earlier steps' REFINED vectors
    (mv_search.c:960-981), and its refinement equals a jmme_subpel_refine call
    (sub_pel_motion_estimation, variant 0) with that answer as mv and
    min_mcost = start_hp ? cost : DISTBLK_MAX"""
    from jmme import FAST_FULL_SEARCH, FULL_SEARCH, MB_REQ, MotionEstimator, synth
    dmax = (2 ** 31 - 1) << 5
    w, h = 352, 288
    rng = np.random.default_rng(900 + 10 * R + rdopt + 100 * ffs + bits)
    luma = synth.luma_sequence(w, h, 2, seed=R + 7 * rdopt, gmv=(3, -2), adversarial=True, adv_range=R)
    if bits > 8:
        sh = bits - 8
        luma = ((luma.astype(np.int32) << sh) + rng.integers(0, 1 << sh, size=luma.shape)).astype(np.uint16)
    mode = FAST_FULL_SEARCH if ffs else FULL_SEARCH
    cfg = {"SearchRange": R, "SearchMode": 0 if ffs else -1, "RDOptimization": rdopt, "SourceBitDepthLuma": bits}
    n_steps = n_moved = 0
    with MotionEstimator(cfg) as me:
        me.upload_cur(luma[1])
        me.upload_ref(0, 0, luma[0])
        for rnd in range(3):
            chains = _random_chains(rng, w, h, 8, R, rdopt, ffs)
            sp = _sp_templates(rng, 8, bits)
            _, res, spo = me.search_chains_sp(mode, np.zeros(0, MB_REQ), chains, sp)
            for i, c in enumerate(chains):
                prev = []
                for k in range(int(c["n_steps"])):
                    p, cen, rmin, rmax = derive(c, k, prev, me.max_mvd)
                    got = res[i, k]
                    if not ffs and (cen[0] | cen[1]) & 3:
                        assert all(res[i, j]["cost"] == -1 for j in range(k, int(c["n_steps"]))), (i, k, res[i])
                        break
                    assert (got["pred_x"], got["pred_y"]) == p, (rnd, i, k, got, p)
                    q, s = _step_req(c, k, p, cen, rmin, rmax, ffs)
                    exp = me.search(mode, q)[0, s]
                    assert (got["mv_x"], got["mv_y"], got["cost"]) == (exp["mv_x"], exp["mv_y"], exp["cost"]), \
                        (rnd, i, k, got, exp)
                    bx, by, _, _ = _geom()[s]
                    r = sp[i:i + 1].copy()
                    r["pos_x"], r["pos_y"] = int(c["mb_x"]) + 4 * bx, int(c["mb_y"]) + 4 * by
                    r["blocktype"] = {0: 1, 1: 2, 3: 3, 5: 4, 9: 5, 17: 6, 25: 7}[max(v for v in (0, 1, 3, 5, 9, 17, 25)
                                                                                  if v <= s)]
                    r["pred_x"], r["pred_y"] = p
                    r["mv_x"], r["mv_y"] = exp["mv_x"], exp["mv_y"]
                    r["min_mcost"] = exp["cost"] if sp[i]["start_hp"] else dmax
                    ref = me.subpel_refine(r)[0]
                    assert (spo[i, k]["mv_x"], spo[i, k]["mv_y"], spo[i, k]["cost"]) == \
                        (ref["mv_x"], ref["mv_y"], ref["cost"]), (rnd, i, k, spo[i, k], ref)
                    n_moved += (ref["mv_x"], ref["mv_y"]) != (exp["mv_x"], exp["mv_y"])
                    prev.append((min(max(int(ref["mv_x"]), -2048), 2047), min(max(int(ref["mv_y"]), -512), 511)))
                    n_steps += 1
    assert n_steps >= 24 and n_moved >= 8, (n_steps, n_moved)


def test_chain_subpel_templates_outside_contract_are_refused(gpu):
    from jmme import FULL_SEARCH, JmmeError, MB_REQ, SUBPEL_REQ, SP_TEST8x8, MotionEstimator
    rng = np.random.default_rng(5)
    plane = (rng.integers(0, 256, (64, 64))).astype(np.uint8)
    chains = _random_chains(rng, 64, 64, 1, 4, 0, False)
    good = np.zeros(1, SUBPEL_REQ)
    good["search_pos2"] = good["search_pos4"] = 9
    empty = np.zeros(0, MB_REQ)
    with MotionEstimator({"SearchRange": 4}) as me:
        me.upload_cur(plane)
        me.upload_ref(0, 0, plane)
        me.search_chains_sp(FULL_SEARCH, empty, chains, good)
        for field, val in [("variant", 1), ("flags", SP_TEST8x8), ("metric_q", 3), ("search_pos2", 10),
                           ("start_hp", 2), ("lambda_h", -1)]:
            bad = good.copy()
            bad[field] = val
            with pytest.raises(JmmeError):
                me.search_chains_sp(FULL_SEARCH, empty, chains, bad)
