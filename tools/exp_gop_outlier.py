#!/usr/bin/env python3
"""Why one GOP of a concurrent GOP-encoder run can take many times the others:
the GOP block's launch (integration/jmme_gop.c, `per_gpu` encoders on one GPU)
with JMME_PHASES=1, each encoder's stderr kept (<prefix><gop>.err), then per GOP
JM's ME time and the library's report lines.  GPU box.
Usage: python3 tools/exp_gop_outlier.py OUTDIR [fs|epzs4k] [gops] [gop] [per_gpu]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tools"), os.path.join(REPO, "tests"), os.path.join(REPO, "--h.264-by-zhaodongyu_amd")):
    sys.path.insert(0, p)
import bench_blocks  # noqa: E402
from jmme import synth  # noqa: E402
from test_jm_dropin_gpu import CFG  # noqa: E402

out = os.path.abspath(sys.argv[1])
preset = sys.argv[2] if len(sys.argv) > 2 else "epzs4k"
gops = int(sys.argv[3]) if len(sys.argv) > 3 else 8
gop = int(sys.argv[4]) if len(sys.argv) > 4 else 2
per = int(sys.argv[5]) if len(sys.argv) > 5 else 8
os.makedirs(out, exist_ok=True)
params, (w, h), _ = bench_blocks.encoder_preset(preset)
yuv = os.path.join(out, "in.yuv")
synth.write_yuv420(yuv, synth.luma_sequence(w, h, gops * gop, seed=3000, gmv=(5, 3)))
os.environ["JMME_PHASES"] = "1"
rep, _ = bench_blocks._gop_launch(os.path.join(REPO, "integration", "_build", "jmme_gop"),
                                  os.path.join(REPO, "integration", "_build", "lencod_jmme"), out, "gpu", yuv, w, h,
                                  gops * gop, gop, 1, per, [0], CFG, params)
os.remove(yuv)
print(json.dumps({"preset": preset, "wall_s": rep["python_wall_s"], "hw_queues": rep.get("hw_queues"),
                  "me_s_per_gop": [r["me_s"] for r in rep["runs"]]}))
for k, r in enumerate(rep["runs"]):
    err = os.path.join(out, "gpu", f"g_gop{k:03d}.err")
    lines = open(err).read().splitlines() if os.path.exists(err) else ["(no .err)"]
    keep = [ln for ln in lines if ln.startswith(("jmme", "jm_gpu_me")) and "Warning" not in ln]
    print(f"--- GOP {k}: ME {r['me_s']} s, wall {r.get('wall_s')}")
    for ln in keep:
        print("   ", ln[:400])
