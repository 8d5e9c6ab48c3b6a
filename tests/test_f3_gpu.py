"""GPU: SURVEY §8(f)3 -- mode decision's inter 4x4 residual coding on the GPU.

jmme_residual4x4 (csrc/jmme_tq.hip residual4x4_kernel) is JM's
residual_transform_quant_luma_4x4 (JM/lencod/src/block.c:660-724) for inter
blocks: check_zero, forward4x4, quant_4x4_normal, inverse4x4 and
sample_reconstruct.  It is checked against the oracle restatement
(oracle/tq_oracle.c, itself pinned to JM's own functions by tq_jm.npz) on
random blocks, and in the encoder: lencod_jmme with JMME_F3=1 serves the inter
calls from GPU batches (integration/jm_f3_gpu.c) and must stay byte-identical to
the stock encoder, with served calls counted."""
import os
import re
import tempfile
import time

import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu


def _params(rng, qp):
    from jmme import QUANT4x4_PARAMS
    p = np.zeros(1, QUANT4x4_PARAMS)
    p["scale"] = rng.integers(1, 13108, 16)
    p["offset"] = rng.integers(0, 1 << (14 + qp // 6), 16)
    p["inv_scale"] = rng.integers(10, 400, 16)
    p["qp_per"] = qp // 6
    p["is_cavlc"] = 1
    p["scan"] = np.array(ol.FRAME_SCAN)
    p["c_cost"] = np.array(ol.C_COST)[0]
    return p


def _expected(p, ores, pred, max_pel):
    """the same call composed from the oracle's forward4x4, quant_4x4_normal and inverse4x4"""
    n = len(ores)
    coef = ol.tq_transform("forward4x4", ores)
    rec = np.zeros((n, 69), np.int32)
    rec[:, :16] = coef
    rec[:, 16:32], rec[:, 32:48], rec[:, 48:64] = p["scale"][0], p["offset"][0], p["inv_scale"][0]
    rec[:, 64], rec[:, 65], rec[:, 66], rec[:, 67] = int(p["qp_per"][0]) * 6, int(p["is_cavlc"][0]), 0, 0
    q = ol.tq_quant_records(rec)
    deq, nz = q[:, 0:16], q[:, 50]
    rres = ol.tq_transform("inverse4x4", deq)
    recon = np.where(nz[:, None] != 0, np.clip(((rres + 32) >> 6) + pred, 0, max_pel), pred)
    zero = ~np.any(ores != 0, axis=1)
    return q, rres, recon, zero


@pytest.mark.parametrize("qp", [4, 28, 45])
def test_residual4x4_matches_oracle(gpu, qp):
    from jmme import MotionEstimator
    rng = np.random.default_rng(qp)
    n = 3000
    pred = rng.integers(0, 256, (n, 16)).astype(np.uint16)
    org = np.clip(pred.astype(np.int32) + rng.integers(-40, 41, (n, 16)) * (rng.random((n, 16)) < 0.8), 0, 255)
    ores = (org - pred).astype(np.int32)
    ores[::7] = 0                                  # check_zero: residual-free blocks
    ores[3::5] = rng.integers(-1, 2, (len(ores[3::5]), 16))   # small residuals (coarse steps quantise them away)
    p = _params(rng, qp)
    with MotionEstimator() as me:
        got = me.residual4x4(p, ores, pred, max_pel=255)
    q, rres, recon, zero = _expected(p, ores, pred, 255)
    np.testing.assert_array_equal(got["zero"] != 0, zero)
    live = ~zero
    np.testing.assert_array_equal(got["nonzero"][live], q[live, 50])
    np.testing.assert_array_equal(got["cost"][live], q[live, 49])
    np.testing.assert_array_equal(got["coef"][live], q[live, 0:16])
    np.testing.assert_array_equal(got["levels"][live][:, 0], q[live, 16])
    for b in np.flatnonzero(live)[:400]:
        k = int(np.argmax(q[b, 16:33] == 0))      # levels up to the terminator, runs beside them
        np.testing.assert_array_equal(got["levels"][b, :k + 1], q[b, 16:17 + k])
        np.testing.assert_array_equal(got["runs"][b, :k], q[b, 33:33 + k])
    nzb = got["nonzero"] != 0
    np.testing.assert_array_equal(got["rres"][nzb], rres[nzb])
    np.testing.assert_array_equal(got["recon"], recon)
    assert nzb.sum() > 100
    if qp >= 28:   # (coarse steps: residuals that quantise to nothing, reconstructed as the prediction)
        assert (~nzb & live).sum() > 10


_F3_LINE = re.compile(r"jm_f3_gpu: (\d+) 4x4 residual calls: (\d+) served from (\d+) GPU batches; on JM's code: "
                      r"(\d+) intra, (\d+) other forms, (\d+) input mismatches")


@pytest.mark.parametrize("symbol_mode", [0, 1])
def test_lencod_inter_residuals_from_gpu_byte_identical(gpu, symbol_mode):
    """lencod_jmme with JMME_F3=1 (FS + sub-pel, RDO on, adaptive rounding off: the
    plain quantiser) vs the stock encoder: identical bitstream and reconstruction,
    inter residual calls served from the GPU; the time delta is printed (the path is
    a round trip per macroblock and mode, off by default)."""
    from jmme import synth
    from test_jm_dropin_gpu import GPU, STOCK, _encode
    params = {"SearchMode": -1, "SearchRange": 16, "NumberReferenceFrames": 2, "RDOptimization": 1,
              "DisableSubpelME": 0, "MEDistortionHPel": 2, "MEDistortionQPel": 2, "MDDistortion": 2,
              "AdaptiveRounding": 0, "SymbolMode": symbol_mode, "ProfileIDC": 77 if symbol_mode else 66}
    w, h, frames = 176, 144, 3
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=17 + symbol_mode, gmv=(2, -1)))
        ref = _encode(STOCK, d, "cpu", yuv, w, h, frames, params)
        t0 = time.time()
        base = _encode(GPU, d, "gpu", yuv, w, h, frames, params)
        t1 = time.time()
        f3 = _encode(GPU, d, "gpuf3", yuv, w, h, frames, params, {"JMME_F3": "1"})
        t2 = time.time()
    assert base[:2] == ref[:2] and f3[:2] == ref[:2], f3[2].stderr[-800:]
    m = _F3_LINE.search(f3[2].stderr)
    assert m, f3[2].stderr[-800:]
    calls, served, batches, intra, other, mism = map(int, m.groups())
    assert served > 0 and batches > 0 and intra > 0 and other == 0, m.group(0)
    assert calls == served + intra + other + mism
    print({"calls": calls, "served": served, "batches": batches, "intra": intra,
           "wall_s_without": round(t1 - t0, 3), "wall_s_with": round(t2 - t1, 3)})
