"""CPU: the transform / quant / SATD restatement (oracle/tq_oracle.c) equals
JM 18.5's own functions on every record of tests/golden/tq_jm.npz."""
import os

import numpy as np
import pytest

import oracle_lib as ol

GOLD = os.path.join(os.path.dirname(__file__), "golden", "tq_jm.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.mark.parametrize("op", sorted(ol.TQ_OPS))
def test_transform_matches_jm(gold, op):
    got = ol.tq_transform(op, gold[op + "_in"])
    np.testing.assert_array_equal(got, gold[op + "_out"])


@pytest.mark.parametrize("size", [4, 8])
def test_satd_matches_jm(gold, size):
    got = ol.tq_satd(gold[f"satd{size}x{size}_in"], size)
    np.testing.assert_array_equal(got, gold[f"satd{size}x{size}_out"][:, 0])


def test_quant4x4_matches_jm(gold):
    got = ol.tq_quant_records(gold["quant4x4_in"])
    np.testing.assert_array_equal(got, gold["quant4x4_out"])
