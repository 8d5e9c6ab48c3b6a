#!/usr/bin/env python3
"""A/B of the EPZS searches alone in the encoder: JMME_SINGLE_MODE 2 (one fused
launch per search, completion word polled) against 3 (the resident server
kernel, no launch per search) on bench.py's EPZS drop-in row (1080p seeded clip,
encoder_baseline.cfg's EPZS keys, 1 reference).  Runs alternate so that box
drift hits both; each run must be byte-identical with the stock encoder.

Usage (GPU box): python3 tools/ab_epzs_server.py [--reps 3] [--idle-us 2000]"""
import argparse
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--idle-us", type=int, default=2000)
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--b-env", default=None, help="NAME=VALUE: compare the server (mode 3) without and with this "
                                                   "variable instead of mode 2 against mode 3")
    a = ap.parse_args()
    from bench_blocks import _lencod, dropin_modes
    from jmme import synth
    from test_jm_dropin_gpu import CFG
    w, h = (int(v) for v in a.size.split("x"))
    tag, mparams, frames = [m for m in dropin_modes() if m[0] == "EPZS"][0]
    params = dict(mparams, SearchRange=32, NumberReferenceFrames=1)
    stock = os.path.join(REPO, "oracle", "_ref", "lencod")
    gpu = os.path.join(REPO, "integration", "_build", "lencod_jmme")
    res = {"2": [], "3": []}
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=2024, gmv=(5, 3)))
        cpu = _lencod(stock, d, "cpu", yuv, w, h, frames, params, CFG)
        print(json.dumps({"stock_me_ms": round(cpu["me_s"] * 1e3, 1)}), flush=True)
        for r in range(a.reps):
            for mode in ("2", "3"):
                env = {"JMME_SINGLE_MODE": mode, "JMME_EPZS_SERVER_IDLE_US": str(a.idle_us)}
                if a.b_env:   # arm "2" becomes: the server with the extra variable
                    env["JMME_SINGLE_MODE"] = "3"
                    if mode == "2":
                        k, v = a.b_env.split("=", 1)
                        env[k] = v
                g = _lencod(gpu, d, f"gpu_{mode}_{r}", yuv, w, h, frames, params, CFG, env)
                ok = g["md5"] == cpu["md5"]
                res[mode].append(round(g["me_s"] * 1e3, 1))
                print(json.dumps({"mode": mode, "rep": r, "me_ms": res[mode][-1], "byte_identical": ok,
                                  "epzs": g.get("epzs"), "spec": g.get("epzs_speculation"), "lib": g.get("lib_clocks")}), flush=True)
                if not ok:
                    sys.exit(1)
    print(json.dumps({"stock_me_ms": round(cpu["me_s"] * 1e3, 1), "mode2_me_ms": res["2"], "mode3_me_ms": res["3"]}))


if __name__ == "__main__":
    main()
