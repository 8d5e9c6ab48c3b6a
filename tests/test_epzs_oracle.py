"""CPU: the EPZS restatement (oracle/epzs_oracle.c) reproduces every EPZS
integer search of the captured JM 18.5 runs (tests/golden/epzs_*.npz):
JM's (mv, cost) and the prevSad slot it leaves, for both search variants
(EPZS_motion_estimation / EPZS_subMB_motion_estimation, me_epzs.c:54, 417),
all refinement / dual patterns except the half-pel SBP diamond, 1-3 reference
frames, and a 1080p frame whose uint16 BlkCount wraps (pre-marked map cells)."""
import numpy as np
import pytest

import oracle_lib as ol
from epzs_cases import EpzsCase, cases


@pytest.mark.parametrize("name", cases())
def test_oracle_matches_jm(name):
    c = EpzsCase(name)
    n = 0
    for f, cur, refs, req, exp in c.frames():
        grid = req["variant"] >= 2
        assert grid.all() or not grid.any()
        out = (ol.epzs_grid_batch if grid.any() else ol.epzs_batch)(req, c.preds, c.stale, cur, refs)
        for k in ("mv_x", "mv_y", "cost", "prev_sad"):
            bad = np.nonzero(out[k] != exp[k])[0]
            assert len(bad) == 0, (name, f, k, len(bad), req[bad[:2]], out[bad[:2]], exp[bad[:2]])
        n += len(req)
    assert n == c.meta["n_searches"]


def test_fixtures_cover_the_search_paths():
    """early exits (ref>0 prevSad, stop/2, subMB predictor stop, post-pattern
    ref>0), full refinement, both variants, every supported pattern pair"""
    paths = np.zeros(6, np.int64)
    pats = set()
    for name in cases():
        c = EpzsCase(name)
        for f, cur, refs, req, exp in c.frames():
            if (req["variant"] >= 2).any():
                continue
            out = ol.epzs_batch(req, c.preds, c.stale, cur, refs)
            paths += np.bincount(out["path"], minlength=6)
            pats |= set(zip(req["pattern"].tolist(), req["dual"].tolist()))
    assert (paths[1:] > 0).all(), paths
    assert {(2, 3), (0, 2), (1, 4), (3, 6), (5, 1)} <= pats


def test_grid_fixtures_cover_the_search_paths():
    """EPZSSubPelGrid = 1: both variants, the SBP diamond (half-pel points), quarter-pel
    predictors, and the early exits of me_epzs_int.c (paths 1-3, 6, 7; 4 is not reached by these encodes)"""
    paths = np.zeros(8, np.int64)
    pats, variants, frac = set(), set(), 0
    for name in cases():
        c = EpzsCase(name)
        for f, cur, refs, req, exp in c.frames():
            if not (req["variant"] >= 2).any():
                continue
            out = ol.epzs_grid_batch(req, c.preds, c.stale, cur, refs)
            paths += np.bincount(out["path"], minlength=8)
            pats |= set(zip(req["pattern"].tolist(), req["dual"].tolist()))
            variants |= set(req["variant"].tolist())
            frac += int(((out["mv_x"] & 3) != 0).sum() + ((out["mv_y"] & 3) != 0).sum())
    assert variants == {2, 3}
    assert (4, 5) in pats and frac > 0
    assert (paths[[1, 2, 3, 5, 6, 7]] > 0).all(), paths


def test_16bit_restatement_equals_8bit_on_8bit_content():
    """build/libepzs_oracle16.so (the restatement over JM's 16-bit imgpel, the checker of
    the high-bit-depth EPZS kernel) answers like the 8-bit build on 8-bit samples; with
    the planes scaled to 10 bits it still runs every search path"""
    from test_epzs_gpu import _random_requests
    rng = np.random.default_rng(11)
    w, h = 96, 64
    cur = rng.integers(0, 256, size=(h, w), dtype=np.uint8)
    refs = [np.clip(np.roll(cur, (2, -3), (0, 1)).astype(np.int32) + rng.integers(-5, 6, size=(h, w)), 0, 255)
            .astype(np.uint8), rng.integers(0, 256, size=(h, w), dtype=np.uint8)]
    req, preds, stale = _random_requests(rng, w, h, 600)
    a = ol.epzs_batch(req, preds, stale, cur, refs)
    b = ol.epzs_batch(req, preds, stale, cur.astype(np.uint16), [r.astype(np.uint16) for r in refs])
    assert np.array_equal(a, b)
    c = ol.epzs_batch(req, preds, stale, cur.astype(np.uint16) << 2, [r.astype(np.uint16) << 2 for r in refs])
    assert len(np.unique(c["path"])) >= 4
