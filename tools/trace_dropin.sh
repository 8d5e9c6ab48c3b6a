#!/bin/bash
# The drop-in encoder (1080p, 2 frames, FS by default: MODE; ADV=1 adversarial motion) with its speculation
# traced: per batch (JMME_TRACE) and per failed guess (JMME_TRACE_MISS), or sampled (SAMPLE=1).  GPU box.
set -e
cd "$(dirname "$0")/.."
out=gpurun_out/${OUT:-trace_dropin}
mkdir -p $out
d=$(mktemp -d)
python3 - "$d" <<'PY'
import os, sys
sys.path.insert(0, "--h.264-by-zhaodongyu_amd"); sys.path.insert(0, "tests")
from jmme import synth
from test_jm_dropin_gpu import CFG
d = sys.argv[1]
adv = os.environ.get("ADV") == "1"   # per-macroblock random motion (SURVEY §8(d) adversarial variant)
synth.write_yuv420(os.path.join(d, "in.yuv"), synth.luma_sequence(1920, 1080, 2, seed=2024, gmv=(0, 0) if adv else (5, 3),
                                                                  adversarial=adv))
open(os.path.join(d, "enc.cfg"), "w").write(CFG)
PY
# SAMPLE=1: a sampling profile of JM's ME region instead of the traces (integration/jm_sample.c)
if [ "${SAMPLE:-0}" = 1 ]; then tr="JMME_SAMPLE=$PWD/$out/samples.txt"
else tr="JMME_TRACE=$PWD/$out/batches.txt JMME_TRACE_MISS=$PWD/$out/misses.txt"; fi
env $tr timeout -k 10 300 \
  "$PWD/integration/_build/lencod_jmme" -d $d/enc.cfg -p InputFile=$d/in.yuv -p SourceWidth=1920 -p SourceHeight=1080 \
  -p OutputWidth=1920 -p OutputHeight=1080 -p FramesToBeEncoded=2 -p OutputFile=$d/o.264 -p ReconFile=$d/r.yuv \
  -p SearchMode=${MODE:--1} -p SearchRange=32 -p RDOptimization=0 -p NumberReferenceFrames=1 ${EXTRA:-} \
  > $out/lencod.log 2>&1
rm -rf "$d"
