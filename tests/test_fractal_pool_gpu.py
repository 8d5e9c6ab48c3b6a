"""GPU: the pruned domain-pool search (csrc/jmme_fractal_pool.hip) -- the
thesis's full_search (ZL/src/block_enc.c:1933-1977) over large radii up to the
"full domain pool" of BASELINE configs[2] -- returns bit-identical
(rms, scale, offset, x, y) to the restatement (oracle/fractal_oracle.c) and to
the windowed kernel, including exact ties (periodic content), flat domains
(D = 0), saturated pels and rejected scales (rms 1e30).
Parity with the thesis itself is unpinned."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu
BLOCKS = [(16, 16), (16, 8), (8, 16), (8, 8), (8, 4), (4, 8), (4, 4)]
NEVER = 1 << 30


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


def _all_blocks(w, h, bsx, bsy):
    from jmme import FRACTAL_REQ
    ys, xs = np.mgrid[0:h - bsy + 1:bsy, 0:w - bsx + 1:bsx]
    req = np.zeros(xs.size, FRACTAL_REQ)
    req["block_x"], req["block_y"], req["bsx"], req["bsy"] = xs.ravel(), ys.ravel(), bsx, bsy
    return req


def _same(got, exp_out, exp_xy, req):
    bad = np.nonzero((got["rms"] != exp_out[:, 0]) | (got["scale"] != exp_out[:, 1]) |
                     (got["offset"] != exp_out[:, 2]) | (got["x"] != exp_xy[:, 0]) | (got["y"] != exp_xy[:, 1]))[0]
    assert len(bad) == 0, (len(bad), [(req[i].tolist(), got[i].tolist(), exp_out[i].tolist(), exp_xy[i].tolist())
                                      for i in bad[:4]])


def _vs_oracle(me, org, ref, R, req, pool_min=0):
    me.fractal_set_pool_min_range(pool_min)
    try:
        got = me.fractal_search(org, ref, R, req)
    finally:
        me.fractal_set_pool_min_range(80)
    exp, xy = ol.fractal_search_batch(org, ref, R, np.stack([req["block_x"], req["block_y"], req["bsx"],
                                                             req["bsy"]], 1).astype(np.int32))
    _same(got, exp, xy, req)
    return got


@pytest.mark.parametrize("R", [5, 16, 40, 1000])
def test_pool_random_blocks_vs_oracle(me, R):
    """every block size, scattered requests (wide union windows), windowed and full pool"""
    h, w = 96, 112
    org, ref = _frames(h, w, 30 + R)
    req = _reqs(w, h, np.random.default_rng(R), 300)
    _vs_oracle(me, org, ref, R, req)


def test_pool_full_qcif_every_4x4(me):
    """BASELINE configs[2] in miniature: every 4x4 range block of QCIF, full domain pool"""
    h, w = 144, 176
    org, ref = _frames(h, w, 4, gmv=(3, 2))
    _vs_oracle(me, org, ref, max(w, h), _all_blocks(w, h, 4, 4))


@pytest.mark.parametrize("bs", BLOCKS)
def test_pool_full_every_block_each_size(me, bs):
    h, w = 64, 96
    org, ref = _frames(h, w, 8)
    _vs_oracle(me, org, ref, 4096, _all_blocks(w, h, *bs))


def test_pool_unrelated_frames(me):
    """no motion to find: the bound prunes least, the most candidates are evaluated exactly"""
    h, w = 80, 96
    rng = np.random.default_rng(5)
    org = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
    _vs_oracle(me, org, ref, 1000, _all_blocks(w, h, 4, 4))


def test_pool_periodic_ties(me):
    """a periodic reference gives many candidates of exactly equal rms: the
    spiral rank must decide, as full_search's strict '<' does"""
    h, w = 64, 80
    base = np.random.default_rng(2).integers(0, 256, (8, 8), dtype=np.uint8)
    ref = np.tile(base, (h // 8, w // 8))
    org = np.roll(ref, (3, 5), axis=(0, 1)).copy()
    org[::7, ::5] = 17                      # perturb some range blocks
    for bs in [(4, 4), (8, 8), (8, 4)]:
        _vs_oracle(me, org, ref, 1000, _all_blocks(w, h, *bs))
    _vs_oracle(me, org, ref, 12, _all_blocks(w, h, 4, 4))


def test_pool_flat_and_saturated(me):
    """flat domains (D = 0 -> alpha = 0), saturated range blocks, whole flat frame"""
    h, w = 64, 80
    org, ref = _frames(h, w, 9)
    org[:16, :] = 255
    org[16:24, :40] = 0
    ref[:, :24] = 0
    ref[40:, 40:] = 128
    _vs_oracle(me, org, ref, 1000, _reqs(w, h, np.random.default_rng(3), 300))
    flat = np.full((h, w), 77, np.uint8)
    _vs_oracle(me, org, flat, 1000, _all_blocks(w, h, 4, 4))
    _vs_oracle(me, flat, ref, 1000, _all_blocks(w, h, 8, 8))


def test_pool_rejected_alpha(me):
    """high-contrast range blocks against a low-contrast reference: most fits
    need |alpha| beyond [-2.35, 4] and are rejected (rms 1e30), so the bound
    passes many candidates the exact path then rejects"""
    h, w = 64, 64
    rng = np.random.default_rng(11)
    org = rng.integers(0, 256, (h, w), dtype=np.uint8)
    ref = (120 + rng.integers(0, 3, (h, w))).astype(np.uint8)
    _vs_oracle(me, org, ref, 1000, _all_blocks(w, h, 4, 4))


def test_pool_matches_windowed_kernel(me):
    """same radius through both kernels (pool forced on / off), CIF, 4x4 and 8x8"""
    h, w = 288, 352
    org, ref = _frames(h, w, 21, gmv=(-4, 3))
    for bs, R in [((4, 4), 20), ((8, 8), 33)]:
        req = _all_blocks(w, h, *bs)
        me.fractal_set_pool_min_range(NEVER)
        win = me.fractal_search(org, ref, R, req)
        me.fractal_set_pool_min_range(0)
        pool = me.fractal_search(org, ref, R, req)
        me.fractal_set_pool_min_range(80)
        assert win.tobytes() == pool.tobytes()


def test_pool_survivor_counter(me):
    h, w = 64, 64
    org, ref = _frames(h, w, 1)
    me.fractal_set_pool_min_range(0)          # a 64x64 picture clamps the radius to 64 < the default 80
    me.fractal_pool_survivors()
    me.fractal_search(org, ref, 1000, _all_blocks(w, h, 4, 4))
    me.fractal_set_pool_min_range(80)
    n = me.fractal_pool_survivors()
    assert 0 < n < 256 * 61 * 61
    assert me.fractal_pool_survivors() == 0


def test_pool_mfma_matches_valu_kernel(me):
    """4x4 full pool: the matrix-core bound test and the VALU one give the same
    bits (both exact; they differ only in which candidates they evaluate)"""
    h, w = 144, 176
    for seed, content in [(31, "motion"), (32, "noise")]:
        if content == "motion":
            org, ref = _frames(h, w, seed, gmv=(-2, 3))
        else:
            rng = np.random.default_rng(seed)
            org = rng.integers(0, 256, (h, w), dtype=np.uint8)
            ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
        req = _all_blocks(w, h, 4, 4)
        me.fractal_set_pool_min_range(0)
        me.fractal_set_pool_mfma(False)
        valu = me.fractal_search(org, ref, 4096, req)
        me.fractal_set_pool_mfma(True)
        mfma = me.fractal_search(org, ref, 4096, req)
        me.fractal_set_pool_min_range(80)
        assert valu.tobytes() == mfma.tobytes()


def test_pool_1080p_every_4x4_full_pool(me):
    """BASELINE configs[2] at full size: every 4x4 range block of a 1080p frame
    (129,600 blocks) against the full domain pool (2,064,609 positions each).
    * the matrix-core and the VALU bound tests give identical results on every block;
    * every winner's rms is <= the windowed R = 4 result (a prefix of the same
      spiral: the pool minimum cannot be worse);
    * a seeded sample of 1,024 blocks equals the restatement's brute force."""
    from jmme import FRACTAL_RES
    W, H = 1920, 1080
    org, ref = _frames(H, W, 77, gmv=(3, 2))
    req = _all_blocks(W, H, 4, 4)
    assert len(req) == 129600
    R = max(W, H)
    me.fractal_set_pool_min_range(0)
    try:
        me.fractal_set_pool_mfma(True)
        mfma = me.fractal_search(org, ref, R, req)
        me.fractal_set_pool_mfma(False)
        valu = me.fractal_search(org, ref, R, req)
        me.fractal_set_pool_mfma(True)
        me.fractal_set_pool_min_range(NEVER)
        seed = me.fractal_search(org, ref, 4, req)
    finally:
        me.fractal_set_pool_min_range(80)
        me.fractal_set_pool_mfma(True)
    assert mfma.dtype == FRACTAL_RES
    diff = np.nonzero((mfma.view(np.uint8).reshape(len(req), -1) != valu.view(np.uint8).reshape(len(req), -1)).any(1))[0]
    assert len(diff) == 0, (len(diff), diff[:5].tolist())
    assert (mfma["rms"] <= seed["rms"]).all()
    assert (mfma["rms"] < seed["rms"]).sum() > 500         # the pool finds better matches than the window (829 here)
    sel = np.sort(np.random.default_rng(2024).choice(len(req), 1024, replace=False))
    rq = np.stack([req["block_x"][sel], req["block_y"][sel], req["bsx"][sel], req["bsy"][sel]], 1).astype(np.int32)
    exp, xy = ol.fractal_search_batch_par(org, ref, R, rq)
    _same(mfma[sel], exp, xy, req[sel])
