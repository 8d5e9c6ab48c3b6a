"""GPU: the HIP transform / quant / SATD kernels (csrc/jmme_tq.hip, through the
C ABI) are bit-exact with JM 18.5's own functions (tests/golden/tq_jm.npz) and
with the oracle restatement on large random batches."""
import os

import numpy as np
import pytest

import oracle_lib as ol

GOLD = os.path.join(os.path.dirname(__file__), "golden", "tq_jm.npz")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def me(gpu):
    from jmme import MotionEstimator
    with MotionEstimator() as m:
        yield m


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def _qparams(rec):
    from jmme import QUANT4x4_PARAMS
    p = np.zeros(len(rec), QUANT4x4_PARAMS)
    p["scale"], p["offset"], p["inv_scale"] = rec[:, 16:32], rec[:, 32:48], rec[:, 48:64]
    p["qp_per"] = rec[:, 64] // 6
    p["is_cavlc"] = rec[:, 65]
    p["scan"] = np.where(rec[:, 66, None, None] != 0, np.array(ol.FIELD_SCAN), np.array(ol.FRAME_SCAN))
    p["c_cost"] = np.array(ol.C_COST)[rec[:, 67]]
    return p


@pytest.mark.parametrize("op", sorted(ol.TQ_OPS))
def test_transform_matches_jm(me, gold, op):
    np.testing.assert_array_equal(me.transform(op, gold[op + "_in"]), gold[op + "_out"])


@pytest.mark.parametrize("size", [4, 8])
def test_satd_matches_jm(me, gold, size):
    np.testing.assert_array_equal(me.satd(size, gold[f"satd{size}x{size}_in"]), gold[f"satd{size}x{size}_out"][:, 0])


def test_quant4x4_matches_jm(me, gold):
    rec, exp = gold["quant4x4_in"], gold["quant4x4_out"]
    params = _qparams(rec)
    coef, levels, runs, cost, nz = me.quant4x4(params, rec[:, :16], rec[:, 68], np.arange(len(rec)))
    np.testing.assert_array_equal(coef, exp[:, 0:16])
    np.testing.assert_array_equal(levels, exp[:, 16:33])
    np.testing.assert_array_equal(runs, exp[:, 33:49])
    np.testing.assert_array_equal(cost, exp[:, 49])
    np.testing.assert_array_equal(nz, exp[:, 50])


@pytest.mark.parametrize("op", sorted(ol.TQ_OPS))
def test_transform_random_vs_oracle(me, op):
    from jmme import TRANSFORM_OPS
    rng = np.random.default_rng(hash(op) & 0xffff)
    _, ein, _ = TRANSFORM_OPS[op]
    lim = 255 if op.startswith("forward") else 1 << 14
    x = rng.integers(-lim, lim + 1, (20000, ein), dtype=np.int32)
    got = me.transform(op, x)
    sel = rng.choice(len(x), 2000, replace=False)
    np.testing.assert_array_equal(got[sel], ol.tq_transform(op, x[sel]))


def test_satd_random_vs_oracle_and_identities(me):
    rng = np.random.default_rng(5)
    for size in (4, 8):
        d = rng.integers(-255, 256, (30000, size * size), dtype=np.int16)
        got = me.satd(size, d)
        sel = rng.choice(len(d), 2000, replace=False)
        np.testing.assert_array_equal(got[sel], ol.tq_satd(d[sel], size))
        np.testing.assert_array_equal(me.satd(size, np.zeros((3, size * size), np.int16)), 0)
        np.testing.assert_array_equal(me.satd(size, -d[:500]), got[:500])   # |H(-d)| = |H(d)|


def test_quant4x4_shared_params_and_random(me):
    rng = np.random.default_rng(11)
    n = 5000
    rec = np.zeros((n, 69), np.int32)
    rec[:, :16] = rng.integers(-4000, 4001, (n, 16)) * (rng.random((n, 16)) < 0.7)
    qp = int(rng.integers(0, 52))
    rec[:, 16:32] = rng.integers(0, 13108, 16)
    rec[:, 32:48] = rng.integers(0, 1 << (15 + qp // 6), 16)
    rec[:, 48:64] = rng.integers(0, 400, 16)
    rec[:, 64], rec[:, 65], rec[:, 66], rec[:, 67] = qp, 1, 0, 0
    rec[:, 68] = rng.integers(0, 4, n)
    params = _qparams(rec[:1])           # one parameter set for every block (param_idx NULL)
    coef, levels, runs, cost, nz = me.quant4x4(params, rec[:, :16], rec[:, 68])
    sel = rng.choice(n, 600, replace=False)
    exp = ol.tq_quant_records(rec[sel])
    np.testing.assert_array_equal(coef[sel], exp[:, 0:16])
    np.testing.assert_array_equal(levels[sel], exp[:, 16:33])
    np.testing.assert_array_equal(runs[sel], exp[:, 33:49])
    np.testing.assert_array_equal(cost[sel], exp[:, 49])
    np.testing.assert_array_equal(nz[sel], exp[:, 50])


def test_tq_rejects_bad_input(me):
    from jmme import JmmeError
    with pytest.raises(JmmeError):
        me.satd(5, np.zeros((1, 25), np.int16))
    from jmme import _lib
    with pytest.raises(JmmeError):
        _lib.check(_lib.lib().jmme_transform(me._ctx, 42, None, None, 1))
    assert me.transform("forward4x4", np.zeros((0, 16), np.int32)).shape == (0, 16)
