"""CPU: the validity intervals of the EPZS restatement (oracle/epzs_oracle.c
eo_epzs_ex / eo_epzs_grid_ex), the checker of the kernel's speculative form.

A search reads the stop criterion S (EPZSDetermineStopCriterion) and the
prevSad value P only through comparisons (JM/lencod/src/me_epzs.c:54-407,
me_epzs_int.c:41-782), each monotone in S or P, so the search's whole
execution -- (mv, cost, path, the EPZSMap cells it stamps, whether it writes
*prevSad) -- is the same for every (S, P) inside the intervals it reports.  The
drop-in serves a speculative answer only when JM's real S and P lie inside.
Checked here: the bookkeeping does not change any result (all captured JM
searches), the inputs lie inside their own intervals, and re-running with S and
P drawn from inside the intervals reproduces the execution exactly."""
import numpy as np
import pytest

import oracle_lib as ol
from epzs_cases import EpzsCase, cases
from test_epzs_gpu import _random_requests


def _same(a, b, av, bv, ab, bb):
    if not np.array_equal(a[["mv_x", "mv_y", "path", "cost"]], b[["mv_x", "mv_y", "path", "cost"]]):
        return False
    if not np.array_equal(ab["prev_written"], bb["prev_written"]) or not np.array_equal(ab["n_visited"], bb["n_visited"]):
        return False
    return all(np.array_equal(av[i, :ab["n_visited"][i]], bv[i, :bb["n_visited"][i]]) for i in range(len(a)))


def _draw_inside(rng, lo, hi, guess):
    """values inside [lo, hi] (clipped to a finite range around the guess): both ends and a random point"""
    lo = np.maximum(lo, 0)
    hi = np.minimum(hi, np.maximum(guess, 0) * 4 + 10 ** 6)
    pick = rng.integers(0, 3, len(lo))
    mid = lo + (rng.random(len(lo)) * (hi - lo + 1)).astype(np.int64).clip(0, None)
    return np.where(pick == 0, lo, np.where(pick == 1, hi, np.minimum(mid, hi)))


@pytest.mark.parametrize("name", cases())
def test_bounds_keep_every_captured_result(name):
    """With the bookkeeping on, every captured JM search still gives JM's answer,
    and JM's own S and P lie inside the intervals the search reports."""
    c = EpzsCase(name)
    for f, cur, refs, req, exp in c.frames():
        grid = bool((req["variant"] >= 2).any())
        out, bnd, _ = ol.epzs_spec_batch(req, c.preds, None, c.stale, cur, refs, grid, max_vis=1)
        for k in ("mv_x", "mv_y", "cost", "prev_sad"):
            assert np.array_equal(out[k], exp[k]), (name, f, k)
        s, p = req["stop_crit"], req["prev_sad"]
        assert ((bnd["stop_lo"] <= s) & (s <= bnd["stop_hi"])).all()
        assert ((bnd["prev_lo"] <= p) & (p <= bnd["prev_hi"])).all()
        # prev_written says whether JM's returned slot is the search's cost
        w = bnd["prev_written"] == 1
        assert np.array_equal(out["prev_sad"][w], out["cost"][w])
        assert np.array_equal(out["prev_sad"][~w], req["prev_sad"][~w])


@pytest.mark.parametrize("grid", [False, True])
@pytest.mark.parametrize("seed", [0, 1])
def test_inside_the_bounds_the_search_is_unchanged(grid, seed):
    """Random requests reaching every path; S and P redrawn inside the reported
    intervals (both ends and a random point) reproduce mv, cost, path, the
    stamped cells and the prevSad write exactly."""
    from jmme import synth
    rng = np.random.default_rng(40 + seed + 10 * grid)
    w, h = 96, 64
    luma = synth.luma_sequence(w, h, 3, seed=seed, gmv=(2, -1))
    cur, refs = luma[2].astype(np.uint8), [luma[1].astype(np.uint8), luma[0].astype(np.uint8)]
    req, preds, stale = _random_requests(rng, w, h, 1500)
    if grid:
        req["variant"] += 2
        req["center_x"] += rng.integers(-3, 4, len(req))
        req["center_y"] += rng.integers(-3, 4, len(req))
        req["max_x"] = np.minimum(req["max_x"], 128)
        req["pattern"] = rng.choice([0, 1, 2, 3, 4, 5], len(req))
        req["dual"] = rng.choice([0, 1, 2, 3, 4, 5, 6], len(req))
    # stop criteria near the centre costs, so the intervals are narrow and every branch is taken
    req["stop_crit"] = rng.integers(0, 60000, len(req))
    req["prev_sad"] = rng.integers(0, 60000, len(req))
    cond = rng.choice([0, 0, 0, 1, 2, 3], len(preds)).astype(np.uint8)
    subs = [np.ascontiguousarray(ol.sub_images(r).astype(np.uint8)) for r in refs] if grid else None
    mv = 4096
    out, bnd, vis = ol.epzs_spec_batch(req, preds, cond, stale, cur, refs, grid, max_vis=mv, subs=subs)
    assert (bnd["n_visited"] <= mv).all()
    assert len(set(out["path"].tolist())) >= 5
    narrow = (bnd["stop_lo"] > 0) & (bnd["stop_hi"] < np.iinfo(np.int64).max)
    assert narrow.mean() > 0.2, narrow.mean()
    for trial in range(3):
        r2 = req.copy()
        r2["stop_crit"] = _draw_inside(rng, bnd["stop_lo"], bnd["stop_hi"], req["stop_crit"])
        r2["prev_sad"] = _draw_inside(rng, bnd["prev_lo"], bnd["prev_hi"], req["prev_sad"])
        o2, b2, v2 = ol.epzs_spec_batch(r2, preds, cond, stale, cur, refs, grid, max_vis=mv, subs=subs)
        assert _same(out, o2, vis, v2, bnd, b2), trial
        # a written prevSad is the cost; an unwritten one is the input, whatever it was
        w = b2["prev_written"] == 1
        assert np.array_equal(o2["prev_sad"][w], o2["cost"][w])
        assert np.array_equal(o2["prev_sad"][~w], r2["prev_sad"][~w])


def test_conditions_equal_the_filtered_list():
    """A list with conditional entries searched under cond equals JM's list (the
    entries whose condition holds for the centre's cost) searched plainly."""
    from jmme import synth
    rng = np.random.default_rng(7)
    w, h = 96, 64
    luma = synth.luma_sequence(w, h, 2, seed=3, gmv=(1, 2))
    cur, refs = luma[1].astype(np.uint8), [luma[0].astype(np.uint8)]
    req, preds, stale = _random_requests(rng, w, h, 800)
    req["plane"] = 0
    req["stop_crit"] = rng.integers(0, 40000, len(req))
    cond = rng.choice([0, 0, 1, 2, 3], len(preds)).astype(np.uint8)
    out, bnd, _ = ol.epzs_spec_batch(req, preds, cond, stale, cur, refs, False, max_vis=1)
    # the centre's cost: the same request with no predictors and no early exit past the median
    probe = req.copy()
    probe["n_pred"] = 0
    probe["ref_idx"] = 0
    probe["medthres"] = -(10 ** 12)
    probe["stop_crit"] = 10 ** 15   # min < stop >> 1: returns the centre cost
    centre = ol.epzs_batch(probe, preds, stale, cur, refs)["cost"]
    filt, offs = [], []
    o = 0
    for i, q in enumerate(req):
        s, g = int(q["stop_crit"]), int(centre[i])
        keep = [j for j in range(q["pred_off"], q["pred_off"] + q["n_pred"])
                if cond[j] == 0 or (cond[j] == 1 and g > s) or (cond[j] == 2 and g > 2 * s) or (cond[j] == 3 and g > 3 * s)]
        filt.append(preds[keep].reshape(-1, 2))
        offs.append(o)
        o += len(keep)
    r2 = req.copy()
    r2["pred_off"] = offs
    r2["n_pred"] = [len(x) for x in filt]
    exp = ol.epzs_batch(r2, np.concatenate(filt), stale, cur, refs)
    for k in ("mv_x", "mv_y", "path", "cost", "prev_sad"):
        assert np.array_equal(out[k], exp[k]), k
