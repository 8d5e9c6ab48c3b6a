"""GPU: the HIP fractal domain-range search (csrc/jmme_fractal.hip) returns
bit-identical (rms, scale, offset, x, y) to the restatement of the thesis's
full_search (oracle/fractal_oracle.c) -- parity with the thesis itself is
unpinned."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
BLOCKS = [(16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4)]


@pytest.fixture(scope="module")
def me(gpu):
    from jmme import MotionEstimator
    with MotionEstimator() as m:
        yield m


def _frames(h, w, seed, gmv=(2, -1)):
    from jmme import synth
    luma = synth.luma_sequence(w, h, 2, seed=seed, gmv=gmv)
    return luma[1].astype(np.uint8), luma[0].astype(np.uint8)


def _reqs(w, h, rng, n, sizes=BLOCKS):
    from jmme import FRACTAL_REQ
    req = np.zeros(n, FRACTAL_REQ)
    for k in range(n):
        bsx, bsy = sizes[rng.integers(len(sizes))]
        req[k] = (rng.integers(0, w // bsx) * bsx, rng.integers(0, h // bsy) * bsy, bsx, bsy)
    return req


def _check(got, org, ref, R, req):
    exp, xy = ol.fractal_search_batch(org, ref, R, np.stack([req["block_x"], req["block_y"], req["bsx"],
                                                             req["bsy"]], 1).astype(np.int32))
    bad = np.nonzero((got["rms"] != exp[:, 0]) | (got["scale"] != exp[:, 1]) | (got["offset"] != exp[:, 2]) |
                     (got["x"] != xy[:, 0]) | (got["y"] != xy[:, 1]))[0]
    assert len(bad) == 0, [(req[i].tolist(), got[i].tolist(), exp[i].tolist(), xy[i].tolist()) for i in bad[:4]]


@pytest.mark.parametrize("R", [0, 1, 7, 16])
def test_random_blocks_vs_oracle(me, R):
    h, w = 144, 176
    org, ref = _frames(h, w, 10 + R)
    rng = np.random.default_rng(R)
    req = _reqs(w, h, rng, 300)
    _check(me.fractal_search(org, ref, R, req), org, ref, R, req)


def test_every_4x4_range_block_cif_r7(me):
    """the thesis setting: 4x4 range blocks, search range 7, all of a CIF frame"""
    from jmme import FRACTAL_REQ
    h, w = 288, 352
    org, ref = _frames(h, w, 3, gmv=(3, 2))
    ys, xs = np.mgrid[0:h:4, 0:w:4]
    req = np.zeros(xs.size, FRACTAL_REQ)
    req["block_x"], req["block_y"], req["bsx"], req["bsy"] = xs.ravel(), ys.ravel(), 4, 4
    _check(me.fractal_search(org, ref, 7, req), org, ref, 7, req)


def test_flat_and_edge_content(me):
    """flat areas (det == 0), saturated pels, windows clipped at every border"""
    h, w = 64, 80
    org, ref = _frames(h, w, 7)
    org[:16, :] = 255
    ref[:, :24] = 0
    ref[40:, 40:] = 128
    rng = np.random.default_rng(1)
    req = _reqs(w, h, rng, 400)
    _check(me.fractal_search(org, ref, 9, req), org, ref, 9, req)


def test_planted_affine_map_recovered(me):
    from jmme import FRACTAL_REQ
    h, w = 96, 128
    _, ref = _frames(h, w, 5)
    ref = (ref & np.uint8(0xFE)).astype(np.uint8)
    org = (np.roll(np.roll(ref.astype(np.int32), 2, axis=0), -3, axis=1) // 2 + 40).astype(np.uint8)
    req = np.array([(48, 40, 8, 8), (64, 32, 16, 16), (20, 20, 4, 4)], FRACTAL_REQ)
    got = me.fractal_search(org, ref, 7, req)
    assert list(zip(got["x"], got["y"])) == [(3, -2)] * 3 and np.all(got["scale"] == 0.5)


def test_box_sums_exact(me):
    p, _ = _frames(40, 48, 2)
    for bsx, bsy in BLOCKS:
        s, s2 = me.fractal_box_sums(p, bsx, bsy)
        es, es2 = ol.fractal_box_sums(p, bsx, bsy)
        np.testing.assert_array_equal(s, es)
        np.testing.assert_array_equal(s2, es2)


def test_rejects_bad_requests(me):
    from jmme import FRACTAL_REQ, JmmeError
    org, ref = _frames(32, 32, 1)
    for bad in [(0, 0, 4, 16), (2, 0, 4, 4), (28, 0, 8, 8)]:
        with pytest.raises(JmmeError):
            me.fractal_search(org, ref, 4, np.array([bad], FRACTAL_REQ))


# ---- a17: the macroblock quadtree (jmme_fractal_encode_mbs) vs fro_encode_mbs --
def _tree_check(got, exp):
    """bit-identical records; the chun of a flat block is NaN on both sides
    (its payload differs between x86 and the GPU, so NaNs compare as NaNs)"""
    assert got.dtype.itemsize == exp.dtype.itemsize == 848
    g, e = got.copy(), exp.copy()
    gn, en = np.isnan(g["chun"]), np.isnan(e["chun"])
    assert np.array_equal(gn, en), np.nonzero(gn != en)
    g["chun"][gn] = 0
    e["chun"][en] = 0
    gb = g.view(np.uint8).reshape(len(g), -1)
    eb = e.view(np.uint8).reshape(len(e), -1)
    bad = np.nonzero((gb != eb).any(1))[0]
    assert len(bad) == 0, (len(bad), [(int(i), np.nonzero(gb[i] != eb[i])[0][:8].tolist(), got[i]["mb"].tolist(),
                                       exp[i]["mb"].tolist(), got[i]["chun"], exp[i]["chun"]) for i in bad[:3]])


@pytest.mark.parametrize("seed,K,R,tols", [(0, 1, 7, (8.0, 5.0)), (1, 2, 4, (4.0, 5.0)), (2, 4, 3, (2.0, 4.0)),
                                           (7, 3, 7, (4.0, 3.0)), (2, 1, 0, (3.0, 5.0))])
def test_tree_vs_oracle(me, seed, K, R, tols):
    from fractal_scenes import gate_scene
    org, refs = gate_scene(176, 144, seed, K, scale=6)
    got = me.fractal_encode_mbs(org, refs, R, *tols)
    exp = ol.fractal_encode_mbs(org, refs, R, *tols)
    assert (exp["mb"]["partition"] == 3).any()
    _tree_check(got, exp)


def test_tree_cif_chroma_and_luma(me):
    """the thesis's frame loop: CIF luma (396 MBs) and a chroma plane (99 MBs)"""
    from fractal_scenes import gate_scene
    for w, h, seed in [(352, 288, 11), (176, 144, 12)]:
        org, refs = gate_scene(w, h, seed, 4, scale=6)
        _tree_check(me.fractal_encode_mbs(org, refs, 7, 4.0, 5.0), ol.fractal_encode_mbs(org, refs, 7, 4.0, 5.0))


def test_tree_async_device_form(me, gpu):
    import torch
    from jmme import FRACTAL_MB
    from fractal_scenes import gate_scene
    org, refs = gate_scene(128, 96, 2, 2, scale=6)
    h, w = org.shape
    d_org = torch.from_numpy(org).to(gpu)
    d_refs = [torch.from_numpy(r).to(gpu) for r in refs]
    d_words = [torch.empty(h * w, dtype=torch.int32, device=gpu) for _ in refs]
    d_out = torch.zeros(len(org.ravel()) // 256 * FRACTAL_MB.itemsize, dtype=torch.uint8, device=gpu)
    stream = torch.cuda.current_stream().cuda_stream
    for r, wd in zip(d_refs, d_words):
        me.fractal_words_async(r.data_ptr(), w, w, h, wd.data_ptr(), stream)
    me.fractal_encode_mbs_async(d_org.data_ptr(), d_refs[0].data_ptr(), w, [wd.data_ptr() for wd in d_words], w, h,
                                5, 4.0, 5.0, d_out.data_ptr(), stream)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().view(FRACTAL_MB)
    _tree_check(got, ol.fractal_encode_mbs(org, refs, 5, 4.0, 5.0))


def test_tree_rejects_bad_geometry(me):
    from jmme import JmmeError
    org = np.zeros((40, 48), np.uint8)
    with pytest.raises(JmmeError):
        me.fractal_encode_mbs(org, [org], 4)           # 40 not a multiple of 16
    org = np.zeros((32, 32), np.uint8)
    with pytest.raises(JmmeError):
        me.fractal_encode_mbs(org, [org] * 5, 4)       # more views than the thesis has
