#!/bin/bash
# rocprofv3 kernel + runtime trace of the drop-in encoder itself (1080p, 2 frames,
# sub-pel on unless SUBPEL=0): where a speculative batch's time goes.  GPU box.
set -e
cd "$(dirname "$0")/.."
out=gpurun_out/${OUT:-prof_dropin}
mkdir -p $out
export TMPDIR=/tmp
d=$(mktemp -d)
python3 - "$d" <<'PY'
import os, sys
sys.path.insert(0, "--h.264-by-zhaodongyu_amd"); sys.path.insert(0, "tests")
from jmme import synth
from test_jm_dropin_gpu import CFG
d = sys.argv[1]
adv = os.environ.get("ADV") == "1"   # per-macroblock random motion
synth.write_yuv420(os.path.join(d, "in.yuv"), synth.luma_sequence(1920, 1080, 2, seed=2024, gmv=(0, 0) if adv else (5, 3),
                                                                  adversarial=adv))
open(os.path.join(d, "enc.cfg"), "w").write(CFG)
PY
args="-d $d/enc.cfg -p InputFile=$d/in.yuv -p SourceWidth=1920 -p SourceHeight=1080 -p OutputWidth=1920
 -p OutputHeight=1080 -p FramesToBeEncoded=2 -p OutputFile=$d/o.264 -p ReconFile=$d/r.yuv -p SearchMode=${MODE:--1}
 -p SearchRange=32 -p RDOptimization=0 -p NumberReferenceFrames=1"
if [ "${SUBPEL:-1}" = 1 ]; then args="$args -p DisableSubpelME=0 -p MEDistortionQPel=2 -p MDDistortion=2"; fi
# MODE=3: EPZS with encoder_baseline.cfg's ME keys (tests/test_jm_dropin_epzs_gpu.py BASELINE_EPZS)
if [ "${MODE:--1}" = 3 ]; then
  args="$args $(python3 -c 'import sys; sys.path.insert(0, "tests"); sys.path.insert(0, "--h.264-by-zhaodongyu_amd")
from test_jm_dropin_epzs_gpu import BASELINE_EPZS as b
print(" ".join(f"-p {k}={v}" for k, v in b.items() if k not in ("SearchRange",)))')"
fi
args="$args ${EXTRA:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --runtime-trace --stats --output-format csv -d $out -o run -- \
  "$PWD/integration/_build/lencod_jmme" $args > $out/lencod.log 2>&1
# per-dispatch durations of the latency kernels (chain / small), summarised before the traces go
python3 - $out <<'PY'
import csv, glob, sys, collections
import numpy as np
out = sys.argv[1]
for f in glob.glob(f"{out}/**/*kernel_trace.csv", recursive=True):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = "chain_kernel" if "chain_kernel" in n else "me_small_kernel" if "me_small_kernel" in n else None
        if k:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    with open(f"{out}/latency_kernels.txt", "w") as o:
        for k, v in d.items():
            v = np.array(v)
            o.write(f"{k}: n {len(v)} mean {v.mean():.2f} us p50 {np.median(v):.2f} p90 {np.percentile(v, 90):.2f} "
                    f"max {v.max():.2f}\n")
PY
# keep the summaries (the per-dispatch traces of a 1080p encode run to hundreds of MB)
find $out -name "*.csv" ! -name "*stats.csv" -delete
find $out -name "*stats.csv" | head
