"""GPU: the drop-in at high bit depth.  A 10-bit High 10 encode (ProfileIDC 110,
SourceBitDepthLuma / OutputBitDepthLuma 10: JM keeps 10-bit samples in its
uint16 imgpel planes, JM/lencod/inc/defines.h:37) through lencod_jmme -- the
integer-pel full / fast full searches on the GPU's 16-bit path (v_sad_u16),
sub-pel refinement on the GPU's 16-bit sub-images -- must be byte-identical to
the stock lencod, with no integer-pel search and no sub-pel refinement left on
the CPU.  A 12-bit encode with SATD sub-pel and FFS covers the clip bound above
10 bits."""
import os
import re
import tempfile

import numpy as np
import pytest

from test_jm_dropin_gpu import GPU, STOCK, _encode

pytestmark = pytest.mark.gpu


def write_yuv420_16(path, luma, bits):
    """planar I420, 16-bit little-endian samples (JM reads 2 bytes per sample
    when the source depth is above 8); chroma mid-grey"""
    f, h, w = luma.shape
    grey = np.full((h // 2, w // 2), 1 << (bits - 1), np.uint16)
    with open(path, "wb") as fp:
        for t in range(f):
            fp.write(luma[t].astype("<u2").tobytes())
            fp.write(grey.astype("<u2").tobytes())
            fp.write(grey.astype("<u2").tobytes())


@pytest.mark.parametrize("w,h,frames,params", [
    (176, 144, 3, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 1}),
    (176, 144, 4, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 2}),
    (352, 288, 3, {"SearchMode": -1, "SearchRange": 32, "RDOptimization": 1, "NumberReferenceFrames": 2,
                   "DisableSubpelME": 0, "MEDistortionQPel": 2, "MDDistortion": 2}),
    (176, 144, 3, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 1,
                   "DisableSubpelME": 0, "MEDistortionHPel": 1, "MEDistortionQPel": 0, "MDDistortion": 0,
                   "Transform8x8Mode": 1}),
    (176, 144, 3, {"SearchMode": 0, "SearchRange": 8, "RDOptimization": 1, "NumberReferenceFrames": 1,
                   "DisableSubpelME": 0, "MEDistortionHPel": 2, "MEDistortionQPel": 2, "MDDistortion": 2,
                   "Transform8x8Mode": 1, "_bits": 12}),
])
def test_lencod_10bit_is_byte_identical(gpu, w, h, frames, params):
    if not (os.path.exists(STOCK) and os.path.exists(GPU)):
        pytest.fail("lencod builds missing: run `make -C oracle ref && make -C integration` in the build container")
    from jmme import synth
    params = dict(params)
    bits = params.pop("_bits", 10)
    p = dict(params, ProfileIDC=110 if bits <= 10 else 244, SourceBitDepthLuma=bits, SourceBitDepthChroma=bits, OutputBitDepthLuma=bits,
             OutputBitDepthChroma=bits)
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        luma = synth.luma_sequence(w, h, frames, seed=w + 3 * frames, gmv=(3, -2)).astype(np.int32)
        rng = np.random.default_rng(frames)
        sh = bits - 8
        luma10 = np.clip((luma << sh) + rng.integers(0, 1 << sh, size=luma.shape), 0, (1 << bits) - 1)
        write_yuv420_16(yuv, luma10.astype(np.uint16), bits)
        ref264, refrec, _ = _encode(STOCK, d, "cpu", yuv, w, h, frames, p)
        gpu264, gpurec, r = _encode(GPU, d, "gpu", yuv, w, h, frames, p)
        assert (gpu264, gpurec) == (ref264, refrec), r.stderr[-800:]
        m = re.search(r"(\d+) integer-pel searches on the GPU .*; (\d+) on the CPU", r.stderr)
        assert m and int(m.group(1)) > 0 and int(m.group(2)) == 0, r.stderr[-800:]
        if not p.get("DisableSubpelME", 1):   # sub-pel on: every refinement on the GPU
            m = re.search(r"(\d+) sub-pel refinements: .*, (\d+) on the CPU", r.stderr)
            assert m and int(m.group(1)) > 0 and int(m.group(2)) == 0, r.stderr[-800:]


@pytest.mark.parametrize("bits,over", [
    (10, {"NumberReferenceFrames": 2}),                                # encoder_baseline.cfg's EPZS (quarter-pel grid)
    (10, {"NumberReferenceFrames": 2, "EPZSSubPelGrid": 0}),           # integer grid + EPZS sub-pel on the GPU
    (12, {"NumberReferenceFrames": 1, "EPZSSubPelGrid": 0, "EPZSPattern": 3, "EPZSDualRefinement": 6}),
])
def test_lencod_epzs_high_bit_depth_is_byte_identical(gpu, bits, over):
    """EPZS (SearchMode 3) at 10 and 12 bits: JM's predictor lists and map state around the
    16-bit EPZS kernel, byte-identical, no EPZS search or EPZS refinement on the CPU"""
    if not (os.path.exists(STOCK) and os.path.exists(GPU)):
        pytest.fail("lencod builds missing: run `make -C oracle ref && make -C integration` in the build container")
    from jmme import synth
    from test_jm_dropin_epzs_gpu import BASELINE_EPZS, _SP_LINE, epzs_stats
    w, h, frames = 176, 144, 3
    p = dict(BASELINE_EPZS, **over)
    p.update(ProfileIDC=110 if bits <= 10 else 244, SourceBitDepthLuma=bits, SourceBitDepthChroma=bits,
             OutputBitDepthLuma=bits, OutputBitDepthChroma=bits)
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        luma = synth.luma_sequence(w, h, frames, seed=bits, gmv=(2, -3)).astype(np.int32)
        sh = bits - 8
        rng = np.random.default_rng(bits)
        lum = np.clip((luma << sh) + rng.integers(0, 1 << sh, size=luma.shape), 0, (1 << bits) - 1)
        write_yuv420_16(yuv, lum.astype(np.uint16), bits)
        ref264, refrec, _ = _encode(STOCK, d, "cpu", yuv, w, h, frames, p)
        gpu264, gpurec, r = _encode(GPU, d, "gpu", yuv, w, h, frames, p)
        assert (gpu264, gpurec) == (ref264, refrec), r.stderr[-800:]
        st = epzs_stats(r.stderr)
        assert st["gpu"] > 0 and st["cpu"] == 0 and st["scans"] == 0, r.stderr[-800:]
        if not p.get("EPZSSubPelGrid", 1):
            m = _SP_LINE.search(r.stderr)
            assert m and int(m.group(1)) > 0 and int(m.group(3)) == 0, r.stderr[-800:]
