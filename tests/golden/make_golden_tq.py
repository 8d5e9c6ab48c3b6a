#!/usr/bin/env python3
"""Golden vectors for SURVEY.md §8 rows a12/a13 (transforms, 4x4 quant, SATD).

Runs oracle/_ref/jm_tq_harness -- JM 18.5's own forward4x4, inverse4x4,
hadamard4x4, ihadamard4x4, hadamard4x2, ihadamard4x2, hadamard2x2,
ihadamard2x2, forward8x8, inverse8x8 (lcommon/src/transform.c),
HadamardSAD4x4/8x8 (lencod/src/me_distortion.c) and quant_4x4_normal
(lencod/src/quant4x4_normal.c), compiled from the reference sources by
oracle/Makefile -- on seeded random blocks and stores inputs + JM outputs in
tests/golden/tq_jm.npz (one (n, in_len) and (n, out_len) int32 array per op).

Usage (this container, needs /root/reference):  python3 tests/golden/make_golden_tq.py
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SEED, N = 20251015, 1000


def parse(path):
    raw = open(path, "rb").read()
    out, off = {}, 0
    while off < len(raw):
        name = raw[off:off + 16].split(b"\0")[0].decode()
        n, lin, lout = np.frombuffer(raw, "<i4", 3, off + 16)
        off += 28
        rec = np.frombuffer(raw, "<i4", int(n) * int(lin + lout), off).reshape(int(n), int(lin + lout))
        off += rec.nbytes
        out[name + "_in"] = rec[:, :lin].copy()
        out[name + "_out"] = rec[:, lin:].copy()
    return out


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    exe = os.path.join(REPO, "oracle", "_ref", "jm_tq_harness")
    with tempfile.TemporaryDirectory() as d:
        b = os.path.join(d, "tq.bin")
        subprocess.run([exe, str(SEED), str(N), b], check=True)
        arrays = parse(b)
    dst = os.path.join(HERE, "tq_jm.npz")
    np.savez_compressed(dst, **arrays)
    man = os.path.join(HERE, "manifest.json")
    m = json.load(open(man))
    m["tq_jm"] = {"case": "tq_jm", "generator": "oracle/_ref/jm_tq_harness (oracle/capture/jm_tq_harness.c)",
                  "seed": SEED, "n_per_op": N, "ops": sorted({k[:-3] for k in arrays if k.endswith("_in")}),
                  "bytes": os.path.getsize(dst)}
    json.dump(m, open(man, "w"), indent=1, sort_keys=True)
    print("wrote", dst, os.path.getsize(dst), "bytes")


if __name__ == "__main__":
    sys.exit(main())
