"""The CPU oracle (oracle/me_oracle.c) against golden vectors captured from the
real JM 18.5 encoder (tests/golden/, made by tests/golden/make_golden.py).

This pins the oracle: every (mv, cost) JM returned must be reproduced exactly.
"""
import numpy as np
import pytest

import golden_io as g
import oracle_lib as ol

FS_CASES = [c for c in g.cases() if g.manifest()[c]["cfg_overrides"]["SearchMode"] == -1]
FFS_CASES = [c for c in g.cases() if g.manifest()[c]["cfg_overrides"]["SearchMode"] == 0]


def _match(c, idx, mv, cost):
    r = c.r
    return (mv[:, 0] == r["out_mv_x"][idx]) & (mv[:, 1] == r["out_mv_y"][idx]) & (cost == r["out_cost"][idx])


@pytest.mark.parametrize("name", FS_CASES)
def test_oracle_full_search_matches_jm(name):
    c = g.Case(name)
    total = 0
    for f, lst, rf, idx in c.groups():
        if c.n > 100000:   # the 1080p case: a seeded sample keeps the CPU suite fast
            idx = np.sort(np.random.default_rng(5).choice(idx, 6000, replace=False))
        mv, cost = ol.full_search_batch(c.cur[f], c.ref[(f, lst, rf)], c.oracle_fs_req(idx))
        m = _match(c, idx, mv, cost)
        assert m.all(), f"{name}: {(~m).sum()} of {len(idx)} searches differ from JM"
        total += len(idx)
    assert total > 0


@pytest.mark.parametrize("name", FFS_CASES)
def test_oracle_fast_full_search_matches_jm(name):
    c = g.Case(name)
    for f, lst, rf, idx in c.groups():
        surf, mmvd, rdopt, mbs, blk = c.oracle_ffs_args(idx)
        mv, cost = ol.ffs_batch(c.cur[f], c.ref[(f, lst, rf)], surf, mmvd, rdopt, mbs, blk)
        m = _match(c, idx, mv, cost)
        assert m.all(), f"{name}: {(~m).sum()} of {len(idx)} searches differ from JM"


def test_fixture_inputs_are_what_jm_read():
    # golden_io regenerates compact fixtures from the seeded generator and
    # checks the md5 JM's planes had; every case must load.
    for name in g.cases():
        c = g.Case(name)
        assert c.n == g.manifest()[name]["n_searches"]
        for (f, lst, rf), p in c.ref.items():
            # 8-bit captures as uint8; high-bit-depth ones as JM's uint16 imgpel, within the depth
            assert p.dtype == (np.uint8 if c.bits == 8 else np.uint16) and p.shape == c.cur[f].shape
            assert int(p.max()) < (1 << c.bits)


def test_golden_covers_the_edge_cases():
    """The fixtures exercise what the reference's path has: picture borders
    (UMV clamp), check_for_00, several references, per-ref range scaling,
    the FFS (0,0) pre-seed and the GetMaxMVD gate context."""
    seen = set()
    for name in g.cases():
        c = g.Case(name)
        r = c.r
        h, w = next(iter(c.cur.values())).shape
        if np.any(r["pix_x"] == 0) and np.any(r["pix_x"] == w - 16):
            seen.add("border_x")
        if np.any(r["pix_y"] == 0) and np.any(r["pix_y"] == h - 16):
            seen.add("border_y")
        if r["mode"][0] == -1 and np.any(c.fs_check_for_00(np.arange(c.n))):
            seen.add("check_for_00")
        if np.any(r["ref"] > 0):
            seen.add("multi_ref")
        if len(np.unique(c.fs_search_range(np.arange(c.n)))) > 1:
            seen.add("range_scaling")
        if r["mode"][0] == 0 and np.any(r["rdopt"] == 0):
            seen.add("ffs_preseed")
        if c.n > 300000:
            seen.add("1080p")
    assert seen >= {"border_x", "border_y", "check_for_00", "multi_ref", "range_scaling", "ffs_preseed", "1080p"}
