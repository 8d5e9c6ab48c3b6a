"""GPU: EPZS (SearchMode = 3) in the drop-in.  lencod_jmme wraps JM's four EPZS
integer searches (JM/lencod/src/me_epzs.c:54,417; me_epzs_int.c:41,431) and
EPZS_sub_pel_motion_estimation (me_epzs_sub.c:30): the predictor lists are
built host-side with JM's own routines and every search runs in
jmme_epzs_search_ex, JM's never-cleared EPZSMap, BlkCount, prevSad and
spatial-memory vectors kept from the GPU's answers (integration/jm_gpu_me.c).
The stock lencod (oracle/_ref/lencod) is the oracle: bitstream and
reconstruction must be byte-identical, with no EPZS search left on the CPU.

BASELINE_EPZS restates the motion-estimation keys of the reference's
encoder_baseline.cfg (JM/bin/encoder_baseline.cfg: SATD sub-pel, RDO on,
SearchRange 32, the EPZS section) with SearchMode = 3 -- the file itself is not
read at run time."""
import os
import re
import tempfile

import pytest

from test_jm_dropin_gpu import GPU, STOCK, _encode

pytestmark = pytest.mark.gpu

BASELINE_EPZS = {
    "ProfileIDC": 66, "SearchMode": 3, "SearchRange": 32, "DisableSubpelME": 0, "MEDistortionFPel": 0,
    "MEDistortionHPel": 2, "MEDistortionQPel": 2, "MDDistortion": 2, "RestrictSearchRange": 2, "RDOptimization": 1,
    "AdaptiveRounding": 1, "EPZSPattern": 2, "EPZSDualRefinement": 3, "EPZSFixedPredictors": 2, "EPZSTemporal": 1,
    "EPZSSpatialMem": 1, "EPZSBlockType": 1, "EPZSMinThresScale": 0, "EPZSMedThresScale": 1,
    "EPZSMaxThresScale": 2, "EPZSSubPelME": 1, "EPZSSubPelMEBiPred": 1, "EPZSSubPelThresScale": 2,
    "EPZSSubPelGrid": 1,
}

_EPZS_LINE = re.compile(r"(\d+) EPZS searches on the GPU \(libjmme\); (\d+) on the CPU; (\d+) predictors, "
                        r"(\d+) pre-stamped map cells, (\d+) switches to window scans; ([\d.]+) ms in the EPZS wrapper, "
                        r"([\d.]+) ms in the engine")
_SP_LINE = re.compile(r"(\d+) EPZS sub-pel refinements on the GPU \((\d+) chained[^)]*\), (\d+) on the CPU")


_SPEC_LINE = re.compile(r"EPZS speculation: (\d+) searches answered from (\d+) batches \((\d+) guesses\), (\d+) searched "
                        r"alone; (\d+) not speculated; guesses refused: (\d+) inputs, (\d+) bounds, (\d+) map cells; "
                        r"([\d.]+) ms building batches")


def epzs_stats(stderr):
    m = _EPZS_LINE.search(stderr)
    assert m, stderr[-800:]
    k = ("gpu", "cpu", "preds", "stale", "scans", "wrap_ms", "call_ms")
    st = {a: (float(b) if a.endswith("_ms") else int(b)) for a, b in zip(k, m.groups())}
    sp = _SPEC_LINE.search(stderr)
    if sp:
        k = ("hits", "batches", "guesses", "alone", "direct", "refused_inputs", "refused_bounds", "refused_cells",
             "build_ms")
        st.update({a: (float(b) if a.endswith("_ms") else int(b)) for a, b in zip(k, sp.groups())})
        # every GPU search is answered from a batch, starts one, runs alone, or was not speculated
        assert st["hits"] + st["batches"] + st["alone"] + st["direct"] == st["gpu"], stderr[-800:]
    m = _SP_LINE.search(stderr)
    if m:
        st.update(sp_gpu=int(m.group(1)), sp_chained=int(m.group(2)), sp_cpu=int(m.group(3)))
    return st


def _run(w, h, frames, over, seed=5, gmv=(3, -2), adversarial=False, env=None):
    if not (os.path.exists(STOCK) and os.path.exists(GPU)):
        pytest.fail("lencod builds missing: run `make -C oracle ref && make -C integration` in the build container")
    from jmme import synth
    params = dict(BASELINE_EPZS, **over)
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=seed, gmv=gmv, adversarial=adversarial))
        ref264, refrec, _ = _encode(STOCK, d, "cpu", yuv, w, h, frames, params)
        gpu264, gpurec, r = _encode(GPU, d, "gpu", yuv, w, h, frames, params, env)
        st = epzs_stats(r.stderr)
        assert (gpu264, gpurec) == (ref264, refrec), r.stderr[-800:]
        return st, r.stderr


@pytest.mark.parametrize("w,h,frames,over", [
    # encoder_baseline.cfg itself (EPZSSubPelGrid 1: the quarter-pel grid searches, no SubPelME)
    (176, 144, 4, {"NumberReferenceFrames": 1}),
    (176, 144, 4, {"NumberReferenceFrames": 3}),
    # EPZSSubPelGrid 0: integer-grid searches + EPZS_sub_pel_motion_estimation on the GPU
    (176, 144, 4, {"NumberReferenceFrames": 2, "EPZSSubPelGrid": 0}),
    (352, 288, 3, {"NumberReferenceFrames": 3, "EPZSSubPelGrid": 0}),
    (352, 288, 3, {"NumberReferenceFrames": 2}),
    # RDO off; the other refinement patterns (0 small diamond, 1 square, 3 extended diamond,
    # 5 PMVFAST; the SBP large diamond 4 needs the grid) and dual refinements; window
    # predictors on every picture-border macroblock (EPZSFixedPredictors 3)
    (176, 144, 3, {"NumberReferenceFrames": 2, "RDOptimization": 0, "EPZSSubPelGrid": 0, "EPZSPattern": 0,
                   "EPZSDualRefinement": 1, "EPZSFixedPredictors": 3}),
    (176, 144, 3, {"NumberReferenceFrames": 2, "RDOptimization": 0, "EPZSPattern": 4, "EPZSDualRefinement": 5,
                   "EPZSFixedPredictors": 3}),
    (176, 144, 3, {"NumberReferenceFrames": 1, "EPZSSubPelGrid": 0, "EPZSPattern": 3, "EPZSDualRefinement": 6,
                   "EPZSSpatialMem": 0, "EPZSTemporal": 0}),
    (176, 144, 3, {"NumberReferenceFrames": 2, "EPZSPattern": 5, "EPZSDualRefinement": 2, "EPZSBlockType": 0,
                   "Transform8x8Mode": 1, "ProfileIDC": 100}),
    (176, 144, 3, {"NumberReferenceFrames": 1, "EPZSPattern": 1, "EPZSDualRefinement": 0, "SearchRange": 16}),
    # several slices per picture: each slice allocates a fresh EPZS structure (slice.c:1661-1665,
    # BlkCount 1 and a zeroed map), which the adapter must recognise
    (352, 288, 3, {"NumberReferenceFrames": 2, "SliceMode": 1, "SliceArgument": 50}),
    (176, 144, 4, {"NumberReferenceFrames": 2, "EPZSSubPelGrid": 0, "SliceMode": 1, "SliceArgument": 20,
                   "RDOptimization": 0}),
])
def test_lencod_epzs_is_byte_identical(gpu, w, h, frames, over):
    st, err = _run(w, h, frames, over, seed=w + frames + len(over))
    assert st["gpu"] > 0 and st["cpu"] == 0 and st["scans"] == 0, err[-800:]
    if not over.get("EPZSSubPelGrid", 1):
        m = _SP_LINE.search(err)
        assert m and int(m.group(1)) > 0 and int(m.group(3)) == 0, err[-800:]


def test_lencod_epzs_blkcount_wraps(gpu):
    """a 1080p P picture runs 334,560 searches in one slice: BlkCount wraps five times
    (me_epzs.c:92-94) and map cells stamped 65535 searches earlier count as visited.
    JMME_EPZS_CHECK=1 has the adapter check its ring of stamped cells against a scan
    of every search window (integer grid: EPZSSubPelGrid 0, sub-pel on the GPU)"""
    st, err = _run(1920, 1080, 2, {"NumberReferenceFrames": 1, "EPZSSubPelGrid": 0}, seed=77,
                   env={"JMME_EPZS_CHECK": "1"})
    assert st["gpu"] == 8160 * 41 and st["cpu"] == 0 and st["scans"] == 0 and st["stale"] > 0, err[-800:]


def test_lencod_epzs_b_pictures_with_cpu_bipred(gpu):
    """B pictures with bi-predictive ME: JM's own EPZS_bipred_motion_estimation shares
    EPZSMap and BlkCount with the GPU searches, so the adapter falls back to scanning the
    search window for cells holding the next BlkCount -- still byte-identical"""
    st, err = _run(176, 144, 5, {"NumberReferenceFrames": 2, "EPZSSubPelGrid": 0, "ProfileIDC": 77,
                                 "NumberBFrames": 1, "BiPredMotionEstimation": 1}, seed=9)
    assert st["gpu"] > 0 and st["cpu"] == 0 and st["scans"] > 0, err[-800:]


def test_lencod_epzs_1080p_frame(gpu):
    """one 1080p P picture (8160 macroblocks, every partition of the baseline config); the
    speculative batches serve the picture: few batches, most searches answered from them, a
    small share searched alone (round trips), every refinement chained or served on the GPU"""
    st, err = _run(1920, 1080, 2, {"NumberReferenceFrames": 1}, seed=31)
    assert st["gpu"] == 8160 * 41 and st["cpu"] == 0 and st["stale"] > 0, err[-800:]
    print({k: st[k] for k in ("hits", "batches", "alone", "direct", "sp_gpu", "sp_chained", "sp_cpu")})
    # (round 4: 128 batches, 324,555 answered, 9,877 alone)
    assert st["direct"] == 0 and st["batches"] <= 200, err[-800:]
    assert st["hits"] >= 0.95 * st["gpu"] and st["alone"] <= 0.05 * st["gpu"], err[-800:]
    assert st["sp_cpu"] == 0 and st["sp_chained"] >= 0.99 * st["sp_gpu"], err[-800:]


def test_lencod_epzs_4k_frame_matches_stock_golden(gpu):
    """BASELINE configs[3] in the encoder at size: one 3840x2160 P picture (32,400
    macroblocks, level 5.1) with encoder_baseline.cfg's EPZS keys -- quarter-pel
    grid, SATD, RDO on, adaptive rounding -- through lencod_jmme.  The stock
    encoder's md5s were recorded in this container by
    tests/golden/make_golden_encodes.py (the stock 4K encode takes a minute; it is
    not repeated here); the drop-in must reproduce bitstream and reconstruction
    byte for byte with every EPZS search on the GPU."""
    from golden_io import manifest
    from jmme import synth
    from test_jm_dropin_gpu import _md5
    m = manifest()["enc_4k_epzs_baseline"]
    w, h, frames = m["w"], m["h"], m["frames"]
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=m["seed"], gmv=tuple(m["gmv"])))
        assert _md5(yuv) == m["md5_input"], "the seeded clip does not regenerate identically"
        b, r, res = _encode(GPU, d, "gpu", yuv, w, h, frames, m["params"])
        st = epzs_stats(res.stderr)
        assert (b, r) == (m["md5_bitstream"], m["md5_recon"]), res.stderr[-800:]
    assert st["gpu"] == 32400 * 41 and st["cpu"] == 0 and st["stale"] > 0, res.stderr[-800:]
    print({k: st.get(k) for k in ("hits", "batches", "alone", "direct", "wrap_ms", "call_ms")})
    assert st["direct"] == 0 and st["hits"] >= 0.9 * st["gpu"], res.stderr[-800:]


_SRV_LINE = re.compile(r"jmme EPZS server: (\d+) searches over (\d+) launches")


@pytest.mark.parametrize("w,h,frames,over,idle_us", [
    (352, 288, 3, {"NumberReferenceFrames": 2}, 2000),
    # an idle time shorter than the gap between two misses: the server leaves
    # between most requests and the host relaunches it (the exit / relaunch race)
    (352, 288, 3, {"NumberReferenceFrames": 2}, 3),
    (176, 144, 4, {"NumberReferenceFrames": 2, "EPZSSubPelGrid": 0}, 2000),
    (1920, 1080, 2, {"NumberReferenceFrames": 1}, 2000),
])
def test_lencod_epzs_resident_server(gpu, w, h, frames, over, idle_us):
    """JMME_SINGLE_MODE=3: the searches alone go to a resident server kernel that
    polls a mailbox in mapped memory (no launch per search); every other entry
    point stops it first.  Byte-identical, and the server served them."""
    st, err = _run(w, h, frames, over, seed=w + frames,
                   env={"JMME_SINGLE_MODE": "3", "JMME_EPZS_SERVER_IDLE_US": str(idle_us), "JMME_PHASES": "1"})
    assert st["gpu"] > 0 and st["cpu"] == 0, err[-800:]
    m = _SRV_LINE.search(err)
    assert m, err[-800:]
    served, launches = int(m.group(1)), int(m.group(2))
    print({"alone": st.get("alone"), "served": served, "launches": launches, "wrap_ms": st["wrap_ms"]})
    # (the searches alone, plus those searched again when a search stamped more cells than kept)
    assert 0.9 * st["alone"] <= served <= st["alone"] + 64 and 1 <= launches <= served, err[-800:]
    if idle_us >= 2000:   # the server stays up between misses (stopped by the batches and uploads only)
        assert launches <= 0.2 * served, err[-800:]


@pytest.mark.parametrize("mode", ["2", "0"])
def test_lencod_epzs_launch_per_search_modes(gpu, mode):
    """the searches alone as one launch each (JMME_SINGLE_MODE 2: own stream and a
    polled completion word; 0: the null stream and a stream sync) -- the forms the
    resident server replaced as the default -- stay byte-identical"""
    st, err = _run(352, 288, 3, {"NumberReferenceFrames": 2}, seed=11, env={"JMME_SINGLE_MODE": mode, "JMME_PHASES": "1"})
    assert st["gpu"] > 0 and st["cpu"] == 0 and st["alone"] > 0, err[-800:]
    assert not _SRV_LINE.search(err), err[-800:]
