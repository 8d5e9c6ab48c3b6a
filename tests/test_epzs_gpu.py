"""GPU: the HIP EPZS search (csrc/jmme_epzs.hip) against JM 18.5 itself (the
captured EPZS searches of tests/golden/epzs_*.npz: mv, cost and the prevSad
JM leaves) and against the restatement (oracle/epzs_oracle.c) on randomised
requests that reach every branch: both variants, all supported pattern
pairs, pre-marked map cells, picture-edge clamping, ranges 0..64."""
import numpy as np
import pytest

import oracle_lib as ol
from epzs_cases import EpzsCase, cases

pytestmark = pytest.mark.gpu


def _run_frame(me, cur, refs, req, preds, stale):
    from jmme import EPZS_REQ
    me.upload_cur(cur)
    for k, r in enumerate(refs):
        me.upload_ref(0, k, r)
    q = np.zeros(len(req), EPZS_REQ)
    for f in EPZS_REQ.names:
        if f in req.dtype.names:
            q[f] = req[f]
    q["ref_slot"] = req["plane"]
    return me.epzs_search(q, preds, stale)


def _cfg_for(c):
    """EPZSSubPelGrid fixtures need a context in grid mode, its map sized for their ranges"""
    grid = int((c.r["variant"] >= 2).any())
    rng = int(max(c.r["sr_max_x"].max(), c.r["sr_max_y"].max()) + 3) // 4
    return {"EPZSSubPelGrid": grid, "SearchRange": max(rng, 1), "SearchMode": 3}


@pytest.mark.parametrize("name", cases())
def test_epzs_matches_jm(gpu, name):
    from jmme import MotionEstimator
    c = EpzsCase(name)
    n = 0
    with MotionEstimator(_cfg_for(c)) as me:
        for f, cur, refs, req, exp in c.frames():
            got = _run_frame(me, cur, refs, req, c.preds, c.stale)
            for k in ("mv_x", "mv_y", "cost", "prev_sad"):
                bad = np.nonzero(got[k] != exp[k])[0]
                assert len(bad) == 0, (name, f, k, len(bad), req[bad[:2]], got[bad[:2]], exp[bad[:2]])
            n += len(req)
    assert n == c.meta["n_searches"]


def _random_requests(rng, w, h, n):
    req = np.zeros(n, ol.EPZS_REQ)
    sizes = [(16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4)]
    preds, stale = [], []
    po = so = 0
    for i in range(n):
        bt = int(rng.integers(1, 8))
        bsx, bsy = sizes[bt - 1]
        q = req[i]
        q["pos_x"] = rng.integers(0, w // bsx) * bsx
        q["pos_y"] = rng.integers(0, h // bsy) * bsy
        q["bsx"], q["bsy"], q["blocktype"] = bsx, bsy, bt
        q["ref_idx"] = rng.integers(0, 3)
        q["plane"] = rng.integers(0, 2)
        q["pred_x"], q["pred_y"] = rng.integers(-90, 90, 2)
        q["center_x"], q["center_y"] = rng.integers(-30, 30, 2) * 4
        q["max_x"] = rng.choice([0, 4, 32, 64, 128, 256])
        q["max_y"] = rng.choice([0, 4, 32, 64, 128])
        q["lambda"] = rng.choice([0, 4, 50, 187, 900])
        q["variant"] = rng.integers(0, 2)
        q["flags"] = rng.integers(0, 4)
        q["pattern"] = rng.choice([0, 1, 2, 3, 5])
        q["dual"] = rng.choice([0, 1, 2, 3, 4, 6])
        q["medthres"] = rng.choice([0, 512, 4096, 8192])
        q["stop_crit"] = rng.choice([0, 2000, 20000, 80000, 400000])
        q["prev_sad"] = rng.choice([0, 1000, 50000, 10 ** 6, (2 ** 31 - 1) << 5])
        k = int(rng.choice([0, 1, 5, 9, 30, 70, 130]))
        p = np.stack([q["center_x"] + rng.integers(-40, 41, k) * rng.choice([1, 4], k),
                      q["center_y"] + rng.integers(-40, 41, k) * rng.choice([1, 4], k)], 1)
        if k > 3:
            p[k // 2] = p[0]          # duplicates
        preds.append(p)
        q["n_pred"], q["pred_off"] = k, po
        po += k
        m = int(rng.choice([0, 0, 3, 20]))
        sc = rng.integers(-20, 21, (m, 2)) * rng.choice([1, 4], (m, 1))
        stale.append(sc)
        q["n_stale"], q["stale_off"] = m, so
        so += m
    return req, np.concatenate(preds).astype(np.int16), np.concatenate(stale).astype(np.int16)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_epzs_random_vs_restatement(gpu, seed):
    from jmme import MotionEstimator, synth
    rng = np.random.default_rng(seed)
    w, h = 96, 64
    luma = synth.luma_sequence(w, h, 3, seed=seed, gmv=(2, -1))
    cur, refs = luma[2].astype(np.uint8), [luma[1].astype(np.uint8), luma[0].astype(np.uint8)]
    req, preds, stale = _random_requests(rng, w, h, 3000)
    exp = ol.epzs_batch(req, preds, stale, cur, refs)
    with MotionEstimator() as me:
        got = _run_frame(me, cur, refs, req, preds, stale)
    for k in ("mv_x", "mv_y", "path", "cost", "prev_sad"):
        bad = np.nonzero(got[k] != exp[k])[0]
        assert len(bad) == 0, (k, len(bad), req[bad[:2]], got[bad[:2]], exp[bad[:2]])
    assert set(np.unique(exp["path"])) == {1, 2, 3, 4, 5}


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_epzs_grid_random_vs_restatement(gpu, seed):
    """EPZSSubPelGrid = 1: quarter-pel centres / predictors / stale cells, the SBP diamond,
    both variants, ranges up to 4 x SearchRange, picture-edge clamping on the sub-images"""
    from jmme import MotionEstimator, synth
    rng = np.random.default_rng(100 + seed)
    w, h = 96, 64
    luma = synth.luma_sequence(w, h, 3, seed=seed, gmv=(2, -1))
    cur, refs = luma[2].astype(np.uint8), [luma[1].astype(np.uint8), luma[0].astype(np.uint8)]
    req, preds, stale = _random_requests(rng, w, h, 2000)
    req["variant"] += 2
    req["center_x"] += rng.integers(-3, 4, len(req))
    req["center_y"] += rng.integers(-3, 4, len(req))
    req["max_x"] = np.minimum(req["max_x"], 128)
    req["pattern"] = rng.choice([0, 1, 2, 3, 4, 5], len(req))
    req["dual"] = rng.choice([0, 1, 2, 3, 4, 5, 6], len(req))
    exp = ol.epzs_grid_batch(req, preds, stale, cur, refs)
    with MotionEstimator({"EPZSSubPelGrid": 1, "SearchRange": 32, "SearchMode": 3}) as me:
        got = _run_frame(me, cur, refs, req, preds, stale)
    for k in ("mv_x", "mv_y", "path", "cost", "prev_sad"):
        bad = np.nonzero(got[k] != exp[k])[0]
        assert len(bad) == 0, (k, len(bad), req[bad[:2]], got[bad[:2]], exp[bad[:2]])
    assert {1, 2, 3, 4, 5, 6, 7} <= set(np.unique(exp["path"]))


def test_epzs_async_device_arrays(gpu):
    import torch
    from jmme import EPZS_REQ, EPZS_RES, MotionEstimator
    c = EpzsCase("epzs_foreman_qcif")
    f, cur, refs, req, exp = list(c.frames())[-1]
    q = np.zeros(len(req), EPZS_REQ)
    for k in EPZS_REQ.names:
        if k in req.dtype.names:
            q[k] = req[k]
    q["ref_slot"] = req["plane"]
    with MotionEstimator() as me:
        me.upload_cur(cur)
        for k, r in enumerate(refs):
            me.upload_ref(0, k, r)
        d_q = torch.from_numpy(q.view(np.uint8).copy()).to(gpu)
        d_p = torch.from_numpy(np.ascontiguousarray(c.preds)).to(gpu)
        d_s = torch.from_numpy(np.ascontiguousarray(c.stale if len(c.stale) else np.zeros((1, 2), np.int16))).to(gpu)
        d_o = torch.zeros(len(q) * EPZS_RES.itemsize, dtype=torch.uint8, device=gpu)
        me.epzs_search_async(d_q.data_ptr(), len(q), d_p.data_ptr(), d_s.data_ptr(), d_o.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = d_o.cpu().numpy().view(EPZS_RES)
    assert np.array_equal(got["cost"], exp["cost"]) and np.array_equal(got["mv_x"], exp["mv_x"])
    assert np.array_equal(got["mv_y"], exp["mv_y"]) and np.array_equal(got["prev_sad"], exp["prev_sad"])


def test_epzs_rejects_bad_requests(gpu):
    from jmme import EPZS_REQ, JmmeError, MotionEstimator
    cur = np.zeros((32, 32), np.uint8)
    good = np.zeros(1, EPZS_REQ)
    good[0] = (0, 0, 16, 16, 1, 0, 0, 0, 0, 0, 64, 64, 4, 0, 3, 2, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    with MotionEstimator() as me:
        me.upload_cur(cur)
        me.upload_ref(0, 0, cur)
        me.epzs_search(good, np.zeros((0, 2), np.int16))
        for field, val in [("pattern", 4), ("dual", 5), ("center_x", 2), ("bsx", 12), ("pos_x", 24),
                           ("max_x", 1024), ("n_pred", 3), ("ref_slot", 5)]:
            bad = good.copy()
            bad[field] = val
            with pytest.raises(JmmeError):
                me.epzs_search(bad, np.zeros((0, 2), np.int16))
