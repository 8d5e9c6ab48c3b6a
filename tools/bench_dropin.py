#!/usr/bin/env python3
"""End-to-end encode with the drop-in (SURVEY §8(d) "end-to-end frame time in
the drop-in encoder"): JM 18.5 lencod (stock, CPU) and lencod_jmme (the same
JM objects, integer-pel ME through libjmme on the GPU, one IntPelME call per
partition exactly as JM issues them) encode the same synthetic clip with the
same configuration; reports both wall times, JM's own "Total ME time", and
whether the bitstreams / reconstructions are byte-identical.
Usage (GPU box): python3 tools/bench_dropin.py [--size 1920x1080] [--frames 2] [--mode -1] [--subpel]"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "--h.264-by-zhaodongyu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from test_jm_dropin_gpu import CFG, GPU, STOCK  # noqa: E402


def run(binary, d, tag, yuv, w, h, frames, params, env=None):
    cfg = os.path.join(d, "enc.cfg")
    open(cfg, "w").write(CFG)
    out, rec = os.path.join(d, f"{tag}.264"), os.path.join(d, f"{tag}_rec.yuv")
    args = [binary, "-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
            "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}", "-p", f"FramesToBeEncoded={frames}",
            "-p", f"OutputFile={out}", "-p", f"ReconFile={rec}"]
    for k, v in params.items():
        args += ["-p", f"{k}={v}"]
    t0 = time.time()
    r = subprocess.run(args, cwd=d, capture_output=True, text=True, timeout=900, env=dict(os.environ, **(env or {})))
    wall = time.time() - t0
    if r.returncode != 0:
        raise RuntimeError(r.stdout[-1500:] + r.stderr[-1500:])
    me = re.search(r"Total ME time for sequence\s*:\s*([0-9.]+) sec", r.stdout)
    calls = re.search(r"jm_gpu_me: (\d+) integer-pel searches on the GPU \(libjmme\): (\d+) from (\d+) speculative",
                      r.stderr)
    sp = re.search(r"(\d+) sub-pel refinements: (\d+) cached, (\d+) batches, (\d+) on the CPU", r.stderr)
    return dict(wall_s=round(wall, 3), me_s=float(me.group(1)) if me else None,
                subpel=dict(zip(("calls", "cached", "batches", "cpu"), map(int, sp.groups()))) if sp else None,
                gpu_searches=int(calls.group(1)) if calls else None,
                from_speculative_batches=int(calls.group(2)) if calls else None,
                batches=int(calls.group(3)) if calls else None,
                md5=(hashlib.md5(open(out, "rb").read()).hexdigest(), hashlib.md5(open(rec, "rb").read()).hexdigest()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--mode", type=int, default=-1)
    ap.add_argument("--range", type=int, default=32)
    ap.add_argument("--subpel", action="store_true",
                    help="sub-pel refinement on (JM default), SATD quarter-pel = mode-decision metric")
    ap.add_argument("--per-call", action="store_true", help="also time JMME_SPECULATE=0 (one GPU call per search)")
    ap.add_argument("--bits", type=int, default=8,
                    help="SourceBitDepthLuma (9..14: 16-bit planes, High 10 / High 4:4:4 profile)")
    a = ap.parse_args()
    from jmme import synth
    w, h = (int(v) for v in a.size.split("x"))
    params = {"SearchMode": a.mode, "SearchRange": a.range, "RDOptimization": 0, "NumberReferenceFrames": 1}
    if a.subpel:
        params.update(DisableSubpelME=0, MEDistortionQPel=2, MDDistortion=2)
    if a.bits > 8:
        params.update(ProfileIDC=110 if a.bits <= 10 else 244, SourceBitDepthLuma=a.bits, SourceBitDepthChroma=a.bits,
                      OutputBitDepthLuma=a.bits, OutputBitDepthChroma=a.bits)
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        luma = synth.luma_sequence(w, h, a.frames, seed=2024, gmv=(5, 3))
        if a.bits > 8:   # the 8-bit texture scaled, plus low-order noise (tests/test_jm_dropin_hbd_gpu.py)
            import numpy as np
            from test_jm_dropin_hbd_gpu import write_yuv420_16
            sh = a.bits - 8
            l16 = (luma.astype(np.int32) << sh) + np.random.default_rng(a.bits).integers(0, 1 << sh, size=luma.shape)
            write_yuv420_16(yuv, np.clip(l16, 0, (1 << a.bits) - 1).astype(np.uint16), a.bits)
        else:
            synth.write_yuv420(yuv, luma)
        cpu = run(STOCK, d, "cpu", yuv, w, h, a.frames, params)
        gpu = run(GPU, d, "gpu", yuv, w, h, a.frames, params)
        percall = run(GPU, d, "gpu1", yuv, w, h, a.frames, params, {"JMME_SPECULATE": "0"}) if a.per_call else None
    mbs = (w // 16) * ((h + 15) // 16) * (a.frames - 1)
    print(json.dumps({
        "metric": "end-to-end JM 18.5 encode with the drop-in integer-pel ME (lencod_jmme vs stock lencod)",
        "size": a.size, "frames": a.frames, "bits": a.bits, "params": params, "p_frame_macroblocks": mbs,
        "stock_cpu": {k: v for k, v in cpu.items() if k != "md5"},
        "dropin_gpu": {k: v for k, v in gpu.items() if k != "md5"},
        "dropin_gpu_per_call": {k: v for k, v in percall.items() if k != "md5"} if percall else None,
        "byte_identical": cpu["md5"] == gpu["md5"] and (percall is None or percall["md5"] == cpu["md5"]),
        "me_speedup": round(cpu["me_s"] / gpu["me_s"], 3) if cpu["me_s"] and gpu["me_s"] else None}))


if __name__ == "__main__":
    main()
