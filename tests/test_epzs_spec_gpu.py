"""GPU: the speculative form of the EPZS kernel (jmme_epzs_speculate) against
the restatement's (oracle/epzs_oracle.c eo_epzs_ex / eo_epzs_grid_ex):
the same (mv, cost, path, prevSad), the same validity intervals of the stop
criterion and prevSad, the same prevSad write and the same stamped EPZSMap
cells, on both grids with the drop-in's predictor conditions; and the sub-pel
refinements chained on the device equal separate jmme_subpel_refine calls
with the searches' results as their inputs (mv_search.c:960-976)."""
import numpy as np
import pytest

import oracle_lib as ol
from epzs_cases import EpzsCase
from test_epzs_gpu import _random_requests

pytestmark = pytest.mark.gpu

DMAX = (2 ** 31 - 1) << 5


def _req_for_engine(req):
    from jmme import EPZS_REQ
    q = np.zeros(len(req), EPZS_REQ)
    for f in EPZS_REQ.names:
        if f in req.dtype.names:
            q[f] = req[f]
    q["ref_slot"] = req["plane"]
    return q


def _scene(seed, grid, n):
    from jmme import synth
    rng = np.random.default_rng(500 + seed + 10 * grid)
    w, h = 96, 64
    luma = synth.luma_sequence(w, h, 3, seed=seed, gmv=(2, -1))
    cur, refs = luma[2].astype(np.uint8), [luma[1].astype(np.uint8), luma[0].astype(np.uint8)]
    req, preds, stale = _random_requests(rng, w, h, n)
    if grid:
        req["variant"] += 2
        req["center_x"] += rng.integers(-3, 4, len(req))
        req["center_y"] += rng.integers(-3, 4, len(req))
        req["max_x"] = np.minimum(req["max_x"], 128)
        req["pattern"] = rng.choice([0, 1, 2, 3, 4, 5], len(req))
        req["dual"] = rng.choice([0, 1, 2, 3, 4, 5, 6], len(req))
    req["stop_crit"] = rng.integers(0, 60000, len(req))
    req["prev_sad"] = rng.integers(0, 60000, len(req))
    cond = rng.choice([0, 0, 0, 1, 2, 3], len(preds)).astype(np.uint8)
    return rng, cur, refs, req, preds, stale, cond


def _compare(got, gb, gv, exp, eb, ev):
    for k in ("mv_x", "mv_y", "path", "cost", "prev_sad"):
        bad = np.nonzero(got[k] != exp[k])[0]
        assert len(bad) == 0, (k, len(bad), got[bad[:3]], exp[bad[:3]])
    for k in ("stop_lo", "stop_hi", "prev_lo", "prev_hi", "prev_written", "n_visited"):
        bad = np.nonzero(gb[k] != eb[k])[0]
        assert len(bad) == 0, (k, len(bad), gb[bad[:3]], eb[bad[:3]])
    assert np.array_equal(got["n_visited"], gb["n_visited"])
    for i in range(len(got)):
        n = min(int(eb["n_visited"][i]), gv.shape[1])
        assert np.array_equal(gv[i, :n], ev[i, :n]), i


@pytest.mark.parametrize("grid", [False, True])
@pytest.mark.parametrize("seed", [0, 1])
def test_speculative_kernel_equals_restatement(grid, seed, gpu):
    from jmme import MotionEstimator
    rng, cur, refs, req, preds, stale, cond = _scene(seed, grid, 2000)
    mv = 512
    exp, eb, ev = ol.epzs_spec_batch(req, preds, cond, stale, cur, refs, grid, max_vis=mv)
    cfg = {"EPZSSubPelGrid": 1, "SearchRange": 32, "SearchMode": 3} if grid else {}
    with MotionEstimator(cfg) as me:
        me.upload_cur(cur)
        for k, r in enumerate(refs):
            me.upload_ref(0, k, r)
        got, gb, gv, _ = me.epzs_speculate(_req_for_engine(req), preds, cond, stale, max_visited=mv)
    _compare(got, gb, gv, exp, eb, ev)
    assert len(set(exp["path"].tolist())) >= 5
    assert (eb["stop_hi"] < np.iinfo(np.int64).max).mean() > 0.2


def test_speculative_kernel_on_jm_captures(gpu):
    """JM's own searches of a 1080p EPZSSubPelGrid P-frame and a QCIF run: JM's
    answers, and the restatement's intervals and cells"""
    from jmme import MotionEstimator
    from test_epzs_gpu import _cfg_for
    for name, take in (("epzs_foreman_qcif", None), ("epzs_grid_syn_1080p_r32", 40000)):
        c = EpzsCase(name)
        with MotionEstimator(_cfg_for(c)) as me:
            for f, cur, refs, req, exp in c.frames():
                if take is not None:
                    sel = np.sort(np.random.default_rng(1).choice(len(req), take, replace=False))
                    req, exp = req[sel], exp[sel]
                grid = bool((req["variant"] >= 2).any())
                me.upload_cur(cur)
                for k, r in enumerate(refs):
                    me.upload_ref(0, k, r)
                got, gb, gv, _ = me.epzs_speculate(_req_for_engine(req), c.preds, None, c.stale, max_visited=256)
                o, ob, ov = ol.epzs_spec_batch(req, c.preds, None, c.stale, cur, refs, grid, max_vis=256)
                for k in ("mv_x", "mv_y", "cost", "prev_sad"):
                    assert np.array_equal(got[k], exp[k]), (name, f, k)
                _compare(got, gb, gv, o, ob, ov)


@pytest.mark.parametrize("grid", [False, True])
def test_chained_subpel_equals_separate_calls(grid, gpu):
    from jmme import BLOCK_RES, SP_TEST8x8, SUBPEL_REQ, MotionEstimator
    rng, cur, refs, req, preds, stale, cond = _scene(7, grid, 1200)
    n = len(req)
    sp = np.zeros(n, SUBPEL_REQ)
    sp["pos_x"], sp["pos_y"], sp["blocktype"] = req["pos_x"], req["pos_y"], req["blocktype"]
    sp["ref_slot"] = req["plane"]
    sp["pred_x"], sp["pred_y"] = req["pred_x"], req["pred_y"]
    sp["lambda_h"] = rng.choice([0, 40, 187], n)
    sp["lambda_q"] = rng.choice([0, 40, 187], n)
    sp["subthres"] = rng.choice([0, 2048, 16384, DMAX], n)
    sp["variant"] = 1
    sp["metric_h"] = rng.integers(0, 3, n)
    sp["metric_q"] = rng.integers(0, 3, n)
    sp["start_hp"] = rng.integers(0, 2, n)
    sp["start_qp"] = rng.integers(0, 2, n)
    sp["search_pos2"] = sp["search_pos4"] = 9
    big = (req["bsx"] >= 8) & (req["bsy"] >= 8)
    sp["flags"] = np.where(big & (rng.random(n) < 0.5), SP_TEST8x8, 0)
    sp["blocktype"][rng.random(n) < 0.1] = 0              # no refinement for these
    cfg = {"EPZSSubPelGrid": 1, "SearchRange": 32, "SearchMode": 3} if grid else {}
    with MotionEstimator(cfg) as me:
        me.upload_cur(cur)
        for k, r in enumerate(refs):
            me.upload_ref(0, k, r)
        got, gb, gv, spo = me.epzs_speculate(_req_for_engine(req), preds, cond, stale, max_visited=64, sp_req=sp)
        want = sp.copy()
        want["mv_x"], want["mv_y"] = got["mv_x"], got["mv_y"]
        want["min_mcost"] = np.where(sp["start_hp"] == 1, got["cost"], DMAX)
        on = sp["blocktype"] != 0
        sep = me.subpel_refine(want[on])
    assert np.array_equal(spo[on], sep)
    assert np.array_equal(spo[~on], np.zeros((~on).sum(), BLOCK_RES))


@pytest.mark.parametrize("grid", [False, True])
def test_fused_refinement_of_small_launches(grid, gpu):
    """a search alone travels in the kernel arguments and refines in the searching wave itself
    (epzs_kernel<..., FUSED>): the same answers and refinements as one big launch
    that chains the refinement kernel"""
    from jmme import SP_TEST8x8, SUBPEL_REQ, MotionEstimator
    rng, cur, refs, req, preds, stale, cond = _scene(11, grid, 240)
    n = len(req)
    sp = np.zeros(n, SUBPEL_REQ)
    sp["pos_x"], sp["pos_y"], sp["blocktype"] = req["pos_x"], req["pos_y"], req["blocktype"]
    sp["ref_slot"] = req["plane"]
    sp["pred_x"], sp["pred_y"] = req["pred_x"], req["pred_y"]
    sp["lambda_h"] = rng.choice([0, 40, 187], n)
    sp["lambda_q"] = rng.choice([0, 40, 187], n)
    sp["subthres"] = rng.choice([0, 2048, 16384, DMAX], n)
    sp["variant"] = 1
    sp["metric_h"] = rng.integers(0, 3, n)
    sp["metric_q"] = rng.integers(0, 3, n)
    sp["start_hp"] = rng.integers(0, 2, n)
    sp["start_qp"] = rng.integers(0, 2, n)
    sp["search_pos2"] = sp["search_pos4"] = 9
    big = (req["bsx"] >= 8) & (req["bsy"] >= 8)
    sp["flags"] = np.where(big & (rng.random(n) < 0.5), SP_TEST8x8, 0)
    sp["blocktype"][rng.random(n) < 0.1] = 0
    cfg = {"EPZSSubPelGrid": 1, "SearchRange": 32, "SearchMode": 3} if grid else {}
    q = _req_for_engine(req)
    with MotionEstimator(cfg) as me:
        me.upload_cur(cur)
        for k, r in enumerate(refs):
            me.upload_ref(0, k, r)
        got, gb, gv, spo = me.epzs_speculate(q, preds, cond, stale, max_visited=64, sp_req=sp)
        for size in (1, 5, 16):
            for a in range(0, 48, size):
                sl = slice(a, a + size)
                g2, b2, v2, s2 = me.epzs_speculate(q[sl], preds, cond, stale, max_visited=64, sp_req=sp[sl])
                for k in ("mv_x", "mv_y", "path", "cost", "prev_sad"):
                    assert np.array_equal(g2[k], got[sl][k]), (size, a, k)
                on = sp[sl]["blocktype"] != 0
                assert np.array_equal(s2[on], spo[sl][on]), (size, a)
