#!/usr/bin/env python3
"""One drop-in EPZS encode (JM/bin/encoder_baseline.cfg's EPZS keys, 1 ref) of
the seeded 1080p clip with the adapter's speculation trace on; prints JM's ME
time and the adapter's statistics lines.  GPU box.
Usage: python3 tools/epzs_trace.py [--frames 2] [--size 1920x1080] [KEY=VALUE ...] [ENV=VALUE via --env]"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
from test_jm_dropin_epzs_gpu import BASELINE_EPZS  # noqa: E402
from test_jm_dropin_gpu import CFG, GPU  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--raw", action="store_true", help="print the encoder's whole stderr")
    ap.add_argument("params", nargs="*")
    a = ap.parse_args()
    from jmme import synth
    w, h = (int(v) for v in a.size.split("x"))
    params = dict(BASELINE_EPZS, SearchRange=32, NumberReferenceFrames=1)
    for kv in a.params:
        k, v = kv.split("=", 1)
        params[k] = v
    env = dict(os.environ, JMME_EPZS_TRACE="1")
    for kv in a.env:
        k, v = kv.split("=", 1)
        env[k] = v
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, a.frames, seed=2024, gmv=(5, 3)))
        cfg = os.path.join(d, "enc.cfg")
        open(cfg, "w").write(CFG)
        args = [GPU, "-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
                "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}", "-p", f"FramesToBeEncoded={a.frames}",
                "-p", f"OutputFile={os.path.join(d, 'o.264')}", "-p", f"ReconFile={os.path.join(d, 'r.yuv')}"]
        for k, v in params.items():
            args += ["-p", f"{k}={v}"]
        r = subprocess.run(args, cwd=d, capture_output=True, text=True, timeout=900, env=env)
    me = re.search(r"Total ME time for sequence\s*:\s*([0-9.]+) sec", r.stdout)
    enc = re.search(r"Total encoding time for the seq\.\s*:\s*([0-9.]+) sec", r.stdout)
    print("ME time", me.group(1) if me else None, "encoding time", enc.group(1) if enc else None, "rc", r.returncode)
    for line in r.stderr.splitlines():
        if a.raw or line.startswith("jm_gpu_me") or line.startswith("jm_f3_profile"):
            print(line)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
