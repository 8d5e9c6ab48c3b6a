#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REAL JM 18.5 encoder.

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py [case ...]

For each case it (1) builds oracle/_ref/lencod_capture from the reference
sources (oracle/Makefile, no JM build system), (2) writes the input YUV
(JM's own foreman_part_qcif.yuv, or our seeded synthetic clip from
jmme.synth), (3) runs the unmodified JM encoder with the case's .cfg
overrides under the --wrap capture shim, and (4) stores the luma planes JM
searched plus every integer-pel search's inputs and JM's (mv, cost) outputs in
tests/golden/<case>.npz, with the run's bitstream/recon md5 in
tests/golden/manifest.json.

The fixtures are data (inputs and JM's outputs), not reference source.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))

from jm_capture import read_capture  # noqa: E402
from jmme import synth  # noqa: E402

JM = "/root/reference/4.对比程序/jm18.5/JM"
BASE_CFG = os.path.join(JM, "bin", "encoder_baseline.cfg")
FOREMAN = os.path.join(JM, "bin", "foreman_part_qcif.yuv")

# integer-pel parity settings used throughout SURVEY.md §8(d)
INT_PEL = {"DisableSubpelME": 1, "EPZSSubPelGrid": 0}

CASES = {
    # config 1 exactly as BASELINE.json configs[0] (all 3 offline frames)
    "c1_foreman_qcif_fs16": dict(src="foreman", w=176, h=144, frames=3,
                                 p={"SearchMode": -1, "SearchRange": 16}),
    # config 1, integer-pel only, RDO off (exercises check_for_00 / CheckSearchRange)
    "c1_foreman_qcif_fs16_rdo0": dict(src="foreman", w=176, h=144, frames=3,
                                      p={"SearchMode": -1, "SearchRange": 16, "RDOptimization": 0,
                                         "MDDistortion": 0, **INT_PEL}),
    # fast full search (JM's default SearchMode=0), RDO on and off
    "ffs_foreman_qcif_r16": dict(src="foreman", w=176, h=144, frames=3,
                                 p={"SearchMode": 0, "SearchRange": 16}),
    "ffs_foreman_qcif_r16_rdo0": dict(src="foreman", w=176, h=144, frames=3,
                                      p={"SearchMode": 0, "SearchRange": 16, "RDOptimization": 0,
                                         "MDDistortion": 0, **INT_PEL}),
    # synthetic CIF at the headline range +-32, 3 refs, RestrictSearchRange=0
    # (per-blocktype / per-ref range scaling, mv_search.c:70-98)
    "syn_cif_fs32_rdo0_3ref": dict(src="synth", w=352, h=288, frames=4, seed=7, gmv=(5, 3),
                                   p={"SearchMode": -1, "SearchRange": 32, "RDOptimization": 0,
                                      "MDDistortion": 0, "NumberReferenceFrames": 3,
                                      "RestrictSearchRange": 0, **INT_PEL}),
    "syn_cif_ffs32_rdo0_3ref": dict(src="synth", w=352, h=288, frames=4, seed=7, gmv=(5, 3),
                                    p={"SearchMode": 0, "SearchRange": 32, "RDOptimization": 0,
                                       "MDDistortion": 0, "NumberReferenceFrames": 3,
                                       "RestrictSearchRange": 1, **INT_PEL}),
    # adversarial per-MB motion (defeats the CPU early exit), RDO on
    "syn_cif_adv_fs32": dict(src="synth", w=352, h=288, frames=2, seed=11, gmv=(0, 0), adversarial=True,
                             p={"SearchMode": -1, "SearchRange": 32, "NumberReferenceFrames": 1, **INT_PEL}),
    # the headline configuration (BASELINE.json configs[1]) at full 1080p: 1 P-frame
    "c2_syn_1080p_fs32": dict(src="synth", w=1920, h=1080, frames=2, seed=2024, gmv=(5, 3),
                              p={"SearchMode": -1, "SearchRange": 32, "NumberReferenceFrames": 1,
                                 "RDOptimization": 0, "MDDistortion": 0, **INT_PEL},
                              keep="compact"),
    # the headline configuration on adversarial content: every 16x16 macroblock of the
    # P-frame moves by its own random vector within +-32 (no global motion for the
    # window centre to ride on; the GPU's exact elimination prunes little)
    "c2_syn_1080p_adv_fs32": dict(src="synth", w=1920, h=1080, frames=2, seed=2025, gmv=(0, 0), adversarial=True,
                                  p={"SearchMode": -1, "SearchRange": 32, "NumberReferenceFrames": 1,
                                     "RDOptimization": 0, "MDDistortion": 0, **INT_PEL},
                                  keep="compact"),
    # the same configuration at 4K (3840x2160, 32,400 MB x ref per P-frame): the bench's UHD block
    # the headline configuration at 10 bits (High 10, SourceBitDepthLuma 10): JM's uint16
    # imgpel planes hold 10-bit samples; the 16-bit search paths' parity fixture
    "c2_syn_1080p_fs32_10bit": dict(src="synth", w=1920, h=1080, frames=2, seed=2024, gmv=(5, 3), bits=10,
                                    p={"ProfileIDC": 110, "SourceBitDepthLuma": 10, "SourceBitDepthChroma": 10,
                                       "OutputBitDepthLuma": 10, "OutputBitDepthChroma": 10,
                                       "SearchMode": -1, "SearchRange": 32, "NumberReferenceFrames": 1,
                                       "RDOptimization": 0, "MDDistortion": 0, **INT_PEL},
                                    keep="compact"),
    "c2_syn_4k_fs32": dict(src="synth", w=3840, h=2160, frames=2, seed=4096, gmv=(5, 3),
                           p={"LevelIDC": 51, "SearchMode": -1, "SearchRange": 32, "NumberReferenceFrames": 1,
                              "RDOptimization": 0, "MDDistortion": 0, **INT_PEL},
                           keep="compact"),
}


def md5(path: str) -> str:
    return hashlib.md5(open(path, "rb").read()).hexdigest()


def build() -> None:
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "-j8", "ref"], check=True)


def run_case(name: str, spec: dict, work: str) -> dict:
    w, h, frames = spec["w"], spec["h"], spec["frames"]
    if spec["src"] == "foreman":
        yuv = FOREMAN
    elif spec.get("bits", 8) > 8:
        yuv = os.path.join(work, f"{name}.yuv")
        synth.write_yuv420_16(yuv, synth.luma_sequence_hbd(w, h, frames, spec["bits"], seed=spec["seed"],
                                                           gmv=spec["gmv"], adversarial=spec.get("adversarial", False)),
                              spec["bits"])
    else:
        yuv = os.path.join(work, f"{name}.yuv")
        luma = synth.luma_sequence(w, h, frames, seed=spec["seed"], gmv=spec["gmv"],
                                   adversarial=spec.get("adversarial", False))
        synth.write_yuv420(yuv, luma)
    cap = os.path.join(work, f"{name}.cap")
    out264 = os.path.join(work, f"{name}.264")
    rec = os.path.join(work, f"{name}_rec.yuv")
    args = [os.path.join(REPO, "oracle", "_ref", "lencod_capture"), "-d", BASE_CFG,
            "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
            "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}",
            "-p", f"FramesToBeEncoded={frames}", "-p", f"OutputFile={out264}", "-p", f"ReconFile={rec}"]
    for k, v in spec["p"].items():
        args += ["-p", f"{k}={v}"]
    env = dict(os.environ, JMME_CAPTURE=cap)
    res = subprocess.run(args, cwd=work, env=env, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(res.stdout[-2000:] + res.stderr[-2000:])
    me_time = [ln for ln in res.stdout.splitlines() if "Total ME time" in ln]
    planes, recs = read_capture(cap)
    return dict(planes=planes, recs=recs, md5_264=md5(out264), md5_rec=md5(rec),
                md5_input=md5(yuv), me_time=me_time[0].strip() if me_time else "",
                cmd=" ".join(a if os.sep not in a else os.path.basename(a) for a in args[1:]))


def coded_synth(spec: dict) -> np.ndarray:
    """The synthetic clip as JM codes it: height padded to a multiple of 16 by
    repeating the last row (JM/lencod/src/lencod.c:463-474 auto-crop)."""
    if spec.get("bits", 8) > 8:
        luma = synth.luma_sequence_hbd(spec["w"], spec["h"], spec["frames"], spec["bits"], seed=spec["seed"],
                                       gmv=spec["gmv"], adversarial=spec.get("adversarial", False))
    else:
        luma = synth.luma_sequence(spec["w"], spec["h"], spec["frames"], seed=spec["seed"], gmv=spec["gmv"],
                                   adversarial=spec.get("adversarial", False))
    hc = (spec["h"] + 15) // 16 * 16
    wc = (spec["w"] + 15) // 16 * 16
    return np.pad(luma, ((0, 0), (0, hc - spec["h"]), (0, wc - spec["w"])), mode="edge")


def save_case(name: str, spec: dict, r: dict) -> dict:
    planes, recs = r["planes"], r["recs"]
    cur_keys = sorted(k for k in planes if k[1] == 0)
    ref_keys = sorted(k for k in planes if k[1] == 1)
    allp = [planes[k] for k in cur_keys + ref_keys]
    bits = spec.get("bits", 8)
    assert max(int(p.max()) for p in allp) < (1 << bits), f"{bits}-bit content expected"
    pel = np.uint8 if bits == 8 else np.uint16
    cur = np.stack([planes[k] for k in cur_keys]).astype(pel)
    ref = np.stack([planes[k] for k in ref_keys]).astype(pel)
    arrays = {
        "cur_frame_no": np.array([k[0] for k in cur_keys], np.int32),
        "ref_key": np.array([[k[0], k[2], k[3]] for k in ref_keys], np.int32),
        "cur_md5": np.array([hashlib.md5(c.tobytes()).hexdigest() for c in cur]),
    }
    if spec.get("keep") == "compact":
        # big case: the current frames are regenerated from the seeded
        # generator (md5-checked by the loader); the reconstructed references
        # are stored as an int8 residual against the generator's original.
        orig = coded_synth(spec)
        assert all(np.array_equal(cur[i], orig[f]) for i, f in enumerate(arrays["cur_frame_no"]))
        res = ref.astype(np.int32) - orig[arrays["ref_key"][:, 0] - 1 - arrays["ref_key"][:, 2]]
        if bits == 8:
            assert res.min() >= -128 and res.max() <= 127
            arrays["ref_residual"] = res.astype(np.int8)
        else:
            assert res.min() >= -32768 and res.max() <= 32767
            arrays["ref_residual"] = res.astype(np.int16)
    else:
        arrays["cur"] = cur
        arrays["ref"] = ref
    for f in recs.dtype.names:
        arrays["r_" + f] = recs[f]
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    return dict(case=name, w=spec["w"], h=spec["h"], frames=spec["frames"], cfg_overrides=spec["p"],
                src=spec["src"], seed=spec.get("seed"), gmv=spec.get("gmv"), bits=spec.get("bits", 8),
                adversarial=spec.get("adversarial", False), n_searches=int(len(recs)),
                md5_bitstream=r["md5_264"], md5_recon=r["md5_rec"], md5_input=r["md5_input"],
                jm_me_time=r["me_time"], jm_cmd=r["cmd"], bytes=os.path.getsize(path))


def main(argv):
    names = argv or list(CASES)
    build()
    mpath = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    with tempfile.TemporaryDirectory() as work:
        for n in names:
            r = run_case(n, CASES[n], work)
            manifest[n] = save_case(n, CASES[n], r)
            print(n, manifest[n]["n_searches"], "searches", manifest[n]["bytes"], "bytes", r["me_time"])
    json.dump(manifest, open(mpath, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
