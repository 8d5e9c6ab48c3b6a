"""ctypes binding to the CPU oracle (oracle/build/libme_oracle.so).

TEST INFRASTRUCTURE: the oracle is the checker.  Only tests/, smoke() and
bench.py's cpu_baseline leg load it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libme_oracle.so")
DISTBLK_MAX = (0x7FFFFFFF) << 5
REQ_FIELDS = 11

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "me_oracle.c")
    if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "port"], check=True)
    lib = ctypes.CDLL(ORACLE_SO)
    P = ctypes.c_void_p
    I = ctypes.c_int
    lib.ora_spiral.argtypes = [I, P]
    lib.ora_spiral.restype = I
    lib.ora_mvbits_table.argtypes = [I, P, I]
    lib.ora_mvbits_table.restype = I
    lib.ora_full_search.argtypes = [P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, ctypes.c_int64, P]
    lib.ora_full_search.restype = ctypes.c_int64
    lib.ora_full_search_batch.argtypes = [P, P, I, I, I, P, P, P]
    lib.ora_full_search_batch.restype = None
    lib.ora_ffs_batch.argtypes = [P, P, I, I, I, I, I, I, P, I, P, P, P]
    lib.ora_ffs_batch.restype = None
    _lib = lib
    return lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def spiral(R: int) -> np.ndarray:
    n = (2 * R + 1) ** 2
    out = np.zeros((n, 2), dtype=np.int16)
    load().ora_spiral(R, _p(out))
    return out


def mvbits_table(R: int):
    buf = np.zeros(1 << 16, dtype=np.int32)
    m = load().ora_mvbits_table(R, _p(buf), buf.size)
    return m, buf[:2 * m + 1].copy()


def full_search_batch(cur: np.ndarray, ref: np.ndarray, req: np.ndarray):
    """req: int32 [n, 11] (see me_oracle.h ORA_REQ_FIELDS). cur/ref uint16 [H, W]."""
    cur = np.ascontiguousarray(cur, dtype=np.uint16)
    ref = np.ascontiguousarray(ref, dtype=np.uint16)
    req = np.ascontiguousarray(req, dtype=np.int32)
    n = req.shape[0]
    mv = np.zeros((n, 2), dtype=np.int16)
    cost = np.zeros(n, dtype=np.int64)
    h, w = cur.shape
    load().ora_full_search_batch(_p(cur), _p(ref), w, h, n, _p(req), _p(mv), _p(cost))
    return mv, cost


def ffs_batch(cur, ref, surf_range, max_mvd, rdopt, mbs, blk):
    """mbs int32 [nmb,4] (mb_x,mb_y,cx,cy qpel); blk int32 [nblk,9] sorted by mb index."""
    cur = np.ascontiguousarray(cur, dtype=np.uint16)
    ref = np.ascontiguousarray(ref, dtype=np.uint16)
    mbs = np.ascontiguousarray(mbs, dtype=np.int32)
    blk = np.ascontiguousarray(blk, dtype=np.int32)
    n = blk.shape[0]
    mv = np.zeros((n, 2), dtype=np.int16)
    cost = np.zeros(n, dtype=np.int64)
    h, w = cur.shape
    load().ora_ffs_batch(_p(cur), _p(ref), w, h, surf_range, max_mvd, rdopt,
                         mbs.shape[0], _p(mbs), n, _p(blk), _p(mv), _p(cost))
    return mv, cost
