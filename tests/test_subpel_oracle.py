"""CPU: the sub-pel restatement (oracle/subpel_oracle.c) reproduces JM 18.5
itself on the captured encodes (tests/golden/subpel_*.npz):
  * getSubImagesLuma (img_luma.c:611-680): the 16 padded quarter-pel
    sub-images JM built, sample for sample;
  * sub_pel_motion_estimation (me_fullsearch.c:186-289) and
    EPZS_sub_pel_motion_estimation (me_epzs_sub.c:30-222): JM's (mv, cost) for
    every refinement, with SAD / SSE / SATD (4x4 and 8x8) metrics, both
    start_me_refinement settings, 1-3 references."""
import numpy as np
import pytest

import oracle_lib as ol
from subpel_cases import SubpelCase, cases, subimg_cases


@pytest.mark.parametrize("name", subimg_cases())
def test_sub_images_match_jm(name):
    c = SubpelCase(name)
    for src, exp in zip(c.sub_src, c.sub_img):
        got = ol.sub_images(src)
        assert got.shape == exp.shape
        bad = [k for k in range(16) if not np.array_equal(got[k], exp[k])]
        assert not bad, (name, bad)


@pytest.mark.parametrize("name", cases())
def test_refinement_matches_jm(name):
    c = SubpelCase(name)
    n = 0
    for f, lst, ref, idx in c.groups():
        sub = ol.sub_images(c.ref[(f, lst, ref)])
        req = c.oracle_req(idx)
        for epzs in (0, 1):
            k = c.r["kind"][idx] == epzs
            if not k.any():
                continue
            mv, cost = ol.sub_pel_batch(c.cur[f], sub, req[k], bool(epzs))
            emv, ecost = c.expected(idx[k])
            bad = np.nonzero((mv != emv).any(1) | (cost != ecost))[0]
            assert len(bad) == 0, (name, f, ref, len(bad), req[k][bad[:2]], mv[bad[:2]], emv[bad[:2]], cost[bad[:2]],
                                   ecost[bad[:2]])
            n += int(k.sum())
    assert n == c.meta["n_searches"]


def test_fixtures_cover_the_refinement_settings():
    seen = set()
    for name in cases():
        r = SubpelCase(name).r
        seen |= set(zip(r["kind"].tolist(), r["metric_h"].tolist(), r["metric_q"].tolist(), r["start_hp"].tolist(),
                        r["start_qp"].tolist(), r["test8x8"].tolist()))
    kinds = {s[0] for s in seen}
    assert kinds == {0, 1}
    assert {s[1] for s in seen} == {0, 1, 2} and any(s[5] for s in seen)
    assert {(s[3], s[4]) for s in seen} >= {(0, 1), (1, 1), (0, 0)}
