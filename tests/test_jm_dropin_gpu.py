"""GPU: the drop-in itself.  JM 18.5 lencod with its integer-pel motion search
redirected to libjmme (integration/_build/lencod_jmme: JM's own objects +
integration/jm_gpu_me.c, JM sources untouched) encodes the same input as the
stock lencod (oracle/_ref/lencod, CPU) with the same configuration: the
bitstreams and reconstructions must be byte-identical, for full search and fast
full search, with RDO on and off, several reference frames, and sub-pel
refinement (SubPelME) off and on (SAD/SSE/SATD, 8x8-transform SATD), P and B
pictures.  The stock
encoder is the oracle here; both binaries are built in this container
(`make -C integration`)."""
import hashlib
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STOCK = os.path.join(REPO, "oracle", "_ref", "lencod")
GPU = os.path.join(REPO, "integration", "_build", "lencod_jmme")

CFG = """# minimal JM 18.5 configuration (unlisted keys: JM defaults)
ProfileIDC            = 66
LevelIDC              = 40
IntraPeriod           = 0
QPISlice              = 28
QPPSlice              = 28
DisableSubpelME       = 1
EPZSSubPelGrid        = 0
MDDistortion          = 0
LeakyBucketParamFile  = "leakybucketparam.cfg"
"""


def _md5(p):
    return hashlib.md5(open(p, "rb").read()).hexdigest()


def _encode(binary, d, tag, yuv, w, h, frames, params, env=None):
    cfg = os.path.join(d, "enc.cfg")
    open(cfg, "w").write(CFG)
    out, rec = os.path.join(d, f"{tag}.264"), os.path.join(d, f"{tag}_rec.yuv")
    args = [binary, "-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
            "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}", "-p", f"FramesToBeEncoded={frames}",
            "-p", f"OutputFile={out}", "-p", f"ReconFile={rec}"]
    for k, v in params.items():
        args += ["-p", f"{k}={v}"]
    r = subprocess.run(args, cwd=d, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, (tag, r.stdout[-1500:], r.stderr[-1500:])
    return _md5(out), _md5(rec), r


@pytest.mark.parametrize("speculate", ["1", "0"])
@pytest.mark.parametrize("w,h,frames,params", [
    (176, 144, 3, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 1}),
    (176, 144, 3, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 1}),
    (176, 144, 4, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 2}),
    (176, 144, 3, {"SearchMode": 0, "SearchRange": 32, "RDOptimization": 1, "NumberReferenceFrames": 1}),
    (352, 288, 4, {"SearchMode": -1, "SearchRange": 32, "RDOptimization": 0, "NumberReferenceFrames": 3,
                   "RestrictSearchRange": 0}),
    # sub-pel refinement on (JM's default): SubPelME on the GPU too (JM wants the
    # quarter-pel metric to be the mode-decision one)
    (176, 144, 3, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 1,
                   "DisableSubpelME": 0, "MEDistortionQPel": 0}),
    (176, 144, 4, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 2,
                   "DisableSubpelME": 0, "MEDistortionHPel": 2, "MEDistortionQPel": 1, "MDDistortion": 1}),
    (352, 288, 3, {"SearchMode": -1, "SearchRange": 32, "RDOptimization": 0, "NumberReferenceFrames": 2,
                   "DisableSubpelME": 0, "ProfileIDC": 100, "Transform8x8Mode": 1, "MDDistortion": 2}),
    (352, 288, 3, {"SearchMode": 0, "SearchRange": 32, "RDOptimization": 1, "NumberReferenceFrames": 1,
                   "DisableSubpelME": 0, "ProfileIDC": 100, "Transform8x8Mode": 2, "MDDistortion": 2}),
    # B pictures (Main profile): list-1 searches and the B-slice sub-pel rules (no check_position0)
    (176, 144, 5, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 2,
                   "NumberBFrames": 1, "ProfileIDC": 77, "DisableSubpelME": 0, "MEDistortionQPel": 0}),
    (176, 144, 5, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 2,
                   "NumberBFrames": 1, "ProfileIDC": 77, "DisableSubpelME": 0, "MEDistortionQPel": 0}),
    # slices (neighbours across a slice border are unavailable: other predictors, same pure search)
    (352, 288, 3, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 2,
                   "SliceMode": 1, "SliceArgument": 33, "DisableSubpelME": 0, "MEDistortionQPel": 0}),
])
def test_lencod_with_gpu_me_is_byte_identical(gpu, w, h, frames, params, speculate):
    """speculate=1: full-search calls answered from speculative batches (jm_gpu_me.c);
    speculate=0: every IntPelME call goes to the GPU on its own"""
    if not (os.path.exists(STOCK) and os.path.exists(GPU)):
        pytest.fail("lencod builds missing: run `make -C oracle ref && make -C integration` in the build container")
    from jmme import synth
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=w + frames, gmv=(3, -2)))
        ref264, refrec, _ = _encode(STOCK, d, "cpu", yuv, w, h, frames, params)
        gpu264, gpurec, r = _encode(GPU, d, "gpu", yuv, w, h, frames, params, {"JMME_SPECULATE": speculate})
        assert "searches on the GPU" in r.stderr and " 0 integer-pel" not in r.stderr, r.stderr[-500:]
        assert (gpu264, gpurec) == (ref264, refrec)
        if params.get("DisableSubpelME") == 0 and speculate == "1":
            m = re.search(r"(\d+) sub-pel refinements: (\d+) cached, (\d+) batches, (\d+) on the CPU", r.stderr)
            assert m and int(m.group(1)) > 0 and int(m.group(4)) == 0, r.stderr[-500:]


@pytest.mark.parametrize("w,h,frames,params,cpu_integer", [
    # SATD / SSE integer-pel metrics: JM's own search (fs_on_cpu / ffs_on_cpu), sub-pel still on the GPU
    (176, 144, 3, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 1,
                   "MEDistortionFPel": 2, "DisableSubpelME": 0, "MEDistortionQPel": 2, "MDDistortion": 2}, "all"),
    (176, 144, 3, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 1,
                   "MEDistortionFPel": 1}, "all"),
    # weighted prediction with weighted reference ME: weighted searches on the CPU (JM weights
    # every P picture here); without UseWeightedReferenceME the search is the plain SAD one
    (176, 144, 4, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 2,
                   "ProfileIDC": 77, "WeightedPrediction": 1, "UseWeightedReferenceME": 1,
                   "DisableSubpelME": 0, "MEDistortionQPel": 0}, "some"),
    (176, 144, 4, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 2,
                   "ProfileIDC": 77, "WeightedPrediction": 1, "UseWeightedReferenceME": 1}, "some"),
    (176, 144, 4, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 2,
                   "ProfileIDC": 77, "WeightedPrediction": 1, "UseWeightedReferenceME": 0,
                   "DisableSubpelME": 0, "MEDistortionQPel": 0}, "none"),
    (176, 144, 4, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 2,
                   "ProfileIDC": 77, "WeightedPrediction": 1, "UseWeightedReferenceME": 0}, "none"),
    # RDPictureDecision codes each frame again (rd_pass 1, 2) with other lists / QPs: the planes
    # and cached answers are keyed on the coded picture, not on frame_no
    (176, 144, 4, {"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0, "NumberReferenceFrames": 2,
                   "RDPictureDecision": 1, "DisableSubpelME": 0, "MEDistortionQPel": 0}, "none"),
    (176, 144, 5, {"SearchMode": 0, "SearchRange": 16, "RDOptimization": 1, "NumberReferenceFrames": 2,
                   "NumberBFrames": 1, "ProfileIDC": 77, "RDPictureDecision": 1, "DisableSubpelME": 0,
                   "MEDistortionQPel": 0}, "none"),
])
def test_lencod_metric_and_picture_rules(gpu, w, h, frames, params, cpu_integer):
    """configurations the GPU search cannot serve go to JM's own integer-pel code (and
    are counted); re-coded pictures re-key the uploads.  Bitstreams stay byte-identical."""
    if not (os.path.exists(STOCK) and os.path.exists(GPU)):
        pytest.fail("lencod builds missing: run `make -C oracle ref && make -C integration` in the build container")
    from jmme import synth
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        seq = synth.luma_sequence(w, h, frames, seed=w + 7 * frames, gmv=(2, 1))
        # a brightness step at the last picture, so that weighted prediction is chosen for it
        # and not for the pictures before it
        seq = np.stack([np.clip(f.astype(np.int32) + (12 if i == frames - 1 else 0), 0, 255).astype(np.uint8)
                        for i, f in enumerate(seq)])
        synth.write_yuv420(yuv, seq)
        ref264, refrec, _ = _encode(STOCK, d, "cpu", yuv, w, h, frames, params)
        gpu264, gpurec, r = _encode(GPU, d, "gpu", yuv, w, h, frames, params)
        assert (gpu264, gpurec) == (ref264, refrec)
        m = re.search(r"(\d+) integer-pel searches on the GPU .*; (\d+) on the CPU", r.stderr)
        assert m, r.stderr[-500:]
        on_gpu, on_cpu = int(m.group(1)), int(m.group(2))
        if cpu_integer == "all":
            assert on_gpu == 0 and on_cpu > 0, r.stderr[-500:]
        elif cpu_integer == "none":
            assert on_gpu > 0 and on_cpu == 0, r.stderr[-500:]
        else:
            assert on_cpu > 0, r.stderr[-500:]


def test_lencod_720p_ffs_subpel_speculative(gpu):
    """a 720p P picture (3600 macroblocks): batches grow to their cap and the four-guess
    cache is exercised at scale; fast full search + SATD sub-pel, JM's defaults"""
    if not (os.path.exists(STOCK) and os.path.exists(GPU)):
        pytest.fail("lencod builds missing: run `make -C oracle ref && make -C integration` in the build container")
    from jmme import synth
    w, h, frames = 1280, 720, 2
    params = {"SearchMode": 0, "SearchRange": 32, "RDOptimization": 0, "NumberReferenceFrames": 1,
              "DisableSubpelME": 0, "MEDistortionQPel": 2, "MDDistortion": 2}
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=w + frames, gmv=(3, -2)))
        ref264, refrec, _ = _encode(STOCK, d, "cpu", yuv, w, h, frames, params)
        gpu264, gpurec, r = _encode(GPU, d, "gpu", yuv, w, h, frames, params)
        assert (gpu264, gpurec) == (ref264, refrec)
        m = re.search(r"(\d+) sub-pel refinements: (\d+) cached, (\d+) batches, (\d+) on the CPU", r.stderr)
        assert m and int(m.group(1)) == 3600 * 41 and int(m.group(4)) == 0, r.stderr[-500:]
        # the chains carry sub-pel steps (jmme_search_mbs_chains_sp): some of JM's
        # refinements are answered from them, and none fell back to the CPU
        c = re.search(r"chained sub-pel: (\d+) refinements, (\d+) calls answered", r.stderr)
        assert c and int(c.group(1)) > 0 and int(c.group(2)) > 0, r.stderr[-800:]
