#!/usr/bin/env python3
"""Diagnostic: one EPZS drop-in encode with the resident server and
JMME_EPZS_SERVER_CHECK=1 (every served search run again by the fused launch);
prints the library's check lines and whether the encode matched the stock one.
Usage (GPU box): python3 tools/dbg_epzs_server.py [--size 1920x1080] [--frames 2] [--seed 1922]"""
import argparse
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--seed", type=int, default=1922)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--mode", default="3", help="JMME_SINGLE_MODE")
    ap.add_argument("--env", action="append", default=[], help="NAME=VALUE for the drop-in encoder")
    ap.add_argument("--param", action="append", default=[], help="JM KEY=VALUE over BASELINE_EPZS (both encoders)")
    a = ap.parse_args()
    from jmme import synth
    from test_jm_dropin_epzs_gpu import BASELINE_EPZS
    from test_jm_dropin_gpu import GPU, STOCK, _encode
    w, h = (int(v) for v in a.size.split("x"))
    params = dict(BASELINE_EPZS, NumberReferenceFrames=1)
    params.update(kv.split("=", 1) for kv in a.param)
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, a.frames, seed=a.seed, gmv=(3, -2)))
        ref = _encode(STOCK, d, "cpu", yuv, w, h, a.frames, params)
        env = {"JMME_SINGLE_MODE": a.mode, "JMME_PHASES": "1"}
        env.update(kv.split("=", 1) for kv in a.env)
        if a.check:
            env["JMME_EPZS_SERVER_CHECK"] = "1"
        got = _encode(GPU, d, "gpu", yuv, w, h, a.frames, params, env)
        for ln in got[2].stderr.splitlines():
            if "server" in ln or "speculation" in ln or "EPZS" in ln or "mismatch" in ln.lower():
                print(ln)
        print("params", params)
        print("byte_identical", got[:2] == ref[:2])


if __name__ == "__main__":
    main()
