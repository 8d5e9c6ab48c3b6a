"""GPU: BASELINE configs[4], the joint fractal + H.264 frame (jmme/hybrid.py)
at 1080p on one MI355X, and the MB-row band form of the fractal quadtree that
the multi-GPU split uses.

The frame: Y 1920x1088 and U, V 960x544 fractal quadtrees over 4 reference
views at the thesis's R = 7 (encode_one_macroblock, ZL/src/block_enc.c:508),
their reconstruction (decode_one_macroblock, ZL/src/block_dec.c:20), and the
JM 18.5 full search +-32 of the bench frame (334,560 searches JM ran).
Parity: the ME against JM's own results; trees and reconstructions of all
three planes against the restatement (oracle/fractal_oracle.c, parity with the
thesis unpinned)."""
import numpy as np
import pytest

import golden_io as g
import oracle_lib as ol
from fractal_scenes import gate_scene

pytestmark = pytest.mark.gpu


def _tree_bytes(t):
    from jmme import FRACTAL_MB
    t = np.array(t, copy=True).view(FRACTAL_MB)
    t["chun"][np.isnan(t["chun"])] = 0          # 0/0 correlation of flat blocks: NaN payloads may differ
    return t.view(np.uint8).reshape(len(t), -1)


def _scene(W, H, n_views=4):
    return [gate_scene(W, H, 11, n_views, scale=6), gate_scene(W // 2, H // 2, 12, n_views, scale=6),
            gate_scene(W // 2, H // 2, 13, n_views, scale=6)]


def test_hybrid_frame_1080p(gpu):
    from jmme import FULL_SEARCH
    from jmme.hybrid import HybridFrameCoder
    import torch
    c = g.Case("c2_syn_1080p_fs32")
    (f, lst, rf, idx), = list(c.groups())
    req, unit_of, slots = c.units(idx, FULL_SEARCH)
    W, H = 1920, 1088
    scene = _scene(W, H)
    with HybridFrameCoder(W, H, n_views=4, fractal_range=7, tol_16=8.0, tol_8=5.0) as hc:
        hc.load_fractal(scene)
        hc.load_me(c.cur[f], c.ref[(f, lst, rf)], req)
        hc.step()
        torch.cuda.synchronize()
        res = hc.me_results()[unit_of, slots]
        assert np.array_equal(res["mv_x"], c.r["out_mv_x"][idx])
        assert np.array_equal(res["mv_y"], c.r["out_mv_y"][idx])
        assert np.array_equal(res["cost"], c.r["out_cost"][idx])
        for p, (org, views) in zip(hc.planes, scene):
            exp = ol.fractal_encode_mbs(org, views, 7, 8.0, 5.0)
            got = p.trees_host()
            bad = np.nonzero((_tree_bytes(got) != _tree_bytes(exp)).any(1))[0]
            assert len(bad) == 0, (p.component, len(bad), bad[:5].tolist())
            rc, rec = ol.fractal_decode_mbs(exp, views, p.component)
            assert rc == 0 and np.array_equal(p.rec.cpu().numpy(), rec), p.component
        split = [(p.trees_host()["mb"]["partition"] == 3).sum() for p in hc.planes]
        assert all(s > 0 for s in split)               # every gate level is exercised


@pytest.mark.parametrize("ws", [2, 3, 5])
def test_fractal_band_rows_equal_whole_plane(ws, gpu):
    """Each rank's MB-row band (jmme_fractal_encode_mb_rows_async) equals those
    rows of the whole-plane encode: the band's searches still see the whole
    reference and bound_chk's frame limits."""
    import torch
    from jmme import shard
    from jmme.hybrid import FractalPlane
    from jmme import MotionEstimator
    W, H = 352, 288
    org, views = gate_scene(W, H, 21, 4, scale=6)
    dev = torch.device("cuda", 0)
    with MotionEstimator() as me:
        whole = FractalPlane(me, 1, W, H, 4, dev)
        whole.load(org, views)
        whole.encode(7, 8.0, 5.0)
        want = whole.trees_host()
        parts = []
        for r in range(ws):
            band = FractalPlane(me, 1, W, H, 4, dev, mb_rows=shard.band_rows(H // 16, r, ws))
            band.load(org, views)
            band.encode(7, 8.0, 5.0)
            parts.append(band.trees_host())
    got = np.concatenate(parts)
    assert len(got) == len(want)
    assert (_tree_bytes(got) == _tree_bytes(want)).all()
    assert (want["mb"]["partition"] == 3).any()
