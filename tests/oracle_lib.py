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


# ---- transforms / quant / SATD (oracle/tq_oracle.c) --------------------------
TQ_SO = os.path.join(ORACLE_DIR, "build", "libtq_oracle.so")
_tq = None

TQ_OPS = {  # op -> (in elements, out elements)
    "forward4x4": (16, 16), "inverse4x4": (16, 16), "hadamard4x4": (16, 16), "ihadamard4x4": (16, 16),
    "hadamard4x2": (8, 8), "ihadamard4x2": (8, 8), "hadamard2x2": (4, 4), "ihadamard2x2": (4, 4),
    "forward8x8": (64, 64), "inverse8x8": (64, 64),
}


class QuantParams(ctypes.Structure):
    _fields_ = [("scale", ctypes.c_int32 * 16), ("offset", ctypes.c_int32 * 16), ("inv_scale", ctypes.c_int32 * 16),
                ("qp_per", ctypes.c_int32), ("is_cavlc", ctypes.c_int32), ("scan", (ctypes.c_uint8 * 2) * 16),
                ("c_cost", ctypes.c_uint8 * 16)]


def load_tq() -> ctypes.CDLL:
    global _tq
    if _tq is not None:
        return _tq
    src = os.path.join(ORACLE_DIR, "tq_oracle.c")
    if not os.path.exists(TQ_SO) or os.path.getmtime(TQ_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "port"], check=True)
    lib = ctypes.CDLL(TQ_SO)
    for op in TQ_OPS:
        getattr(lib, "tqo_" + op).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.tqo_hadamard_sad4x4.argtypes = [ctypes.c_void_p]
    lib.tqo_hadamard_sad8x8.argtypes = [ctypes.c_void_p]
    lib.tqo_quant_4x4_normal.argtypes = [ctypes.c_void_p, ctypes.POINTER(QuantParams), ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]
    _tq = lib
    return lib


def tq_transform(op, blocks):
    """blocks int32 [n, in] -> [n, out] through the oracle's tqo_<op>."""
    lib = load_tq()
    fn = getattr(lib, "tqo_" + op)
    blocks = np.ascontiguousarray(blocks, np.int32)
    out = np.zeros((blocks.shape[0], TQ_OPS[op][1]), np.int32)
    for i in range(blocks.shape[0]):
        fn(blocks[i].ctypes.data, out[i].ctypes.data)
    return out


def tq_satd(diff, size):
    lib = load_tq()
    fn = lib.tqo_hadamard_sad4x4 if size == 4 else lib.tqo_hadamard_sad8x8
    diff = np.ascontiguousarray(diff, np.int16)
    return np.array([fn(diff[i].ctypes.data) for i in range(diff.shape[0])], np.int32)


FRAME_SCAN = [(0, 0), (1, 0), (0, 1), (0, 2), (1, 1), (2, 0), (3, 0), (2, 1),
              (1, 2), (0, 3), (1, 3), (2, 2), (3, 1), (3, 2), (2, 3), (3, 3)]
FIELD_SCAN = [(0, 0), (0, 1), (1, 0), (0, 2), (0, 3), (1, 1), (1, 2), (1, 3),
              (2, 0), (2, 1), (2, 2), (2, 3), (3, 0), (3, 1), (3, 2), (3, 3)]
C_COST = [[3, 2, 2, 1, 1, 1] + [0] * 10, [9] * 16]


def quant_params(scale, offset, inv, qp, cavlc, scan_sel, cost_sel) -> QuantParams:
    q = QuantParams()
    for k in range(16):
        q.scale[k], q.offset[k], q.inv_scale[k] = int(scale[k]), int(offset[k]), int(inv[k])
        sc = (FIELD_SCAN if scan_sel else FRAME_SCAN)[k]
        q.scan[k][0], q.scan[k][1] = sc
        q.c_cost[k] = C_COST[cost_sel][k]
    q.qp_per = int(qp) // 6
    q.is_cavlc = int(cavlc)
    return q


def tq_quant_records(rec_in):
    """Rows laid out as the harness's quant4x4 records -> rows like its outputs."""
    lib = load_tq()
    rec_in = np.asarray(rec_in, np.int32)
    out = np.zeros((rec_in.shape[0], 51), np.int32)
    for i, r in enumerate(rec_in):
        coef = r[0:16].copy()
        q = quant_params(r[16:32], r[32:48], r[48:64], r[64], r[65], r[66], r[67])
        levels = np.zeros(17, np.int32)
        runs = np.zeros(16, np.int32)
        cost = np.array([r[68]], np.int32)
        nz = lib.tqo_quant_4x4_normal(coef.ctypes.data, ctypes.byref(q), levels.ctypes.data, runs.ctypes.data,
                                      cost.ctypes.data)
        out[i] = np.concatenate([coef, levels, runs, cost, [nz]])
    return out


# ---- thesis fractal domain-range search (oracle/fractal_oracle.c, parity unpinned) --
FR_SO = os.path.join(ORACLE_DIR, "build", "libfractal_oracle.so")
_fr = None


def load_fractal() -> ctypes.CDLL:
    global _fr
    if _fr is not None:
        return _fr
    src = os.path.join(ORACLE_DIR, "fractal_oracle.c")
    if not os.path.exists(FR_SO) or os.path.getmtime(FR_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "port"], check=True)
    lib = ctypes.CDLL(FR_SO)
    P, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    lib.fro_box_sums.argtypes = [P, I, I, I, I, I, P, P]
    lib.fro_compute_rms.argtypes = [P, P, I, I, I, I, I, I, I, P, P]
    lib.fro_compute_rms.restype = D
    lib.fro_full_search.argtypes = [P, P, I, I, I, I, I, I, I, I, P, P, P, P]
    lib.fro_full_search.restype = D
    lib.fro_full_search_batch.argtypes = [P, P, I, I, I, I, I, P, P, P]
    _fr = lib
    return lib


def fractal_search_batch(org, ref, R, req):
    """org/ref uint8 HxW; req int32 [n,4] (bx,by,bsx,bsy) -> (out f64 [n,3] rms/scale/offset, xy int32 [n,2])"""
    lib = load_fractal()
    org = np.ascontiguousarray(org, np.uint8)
    ref = np.ascontiguousarray(ref, np.uint8)
    req = np.ascontiguousarray(req, np.int32)
    h, w = org.shape
    out = np.zeros((len(req), 3), np.float64)
    xy = np.zeros((len(req), 2), np.int32)
    lib.fro_full_search_batch(org.ctypes.data, ref.ctypes.data, w, w, h, int(R), len(req), req.ctypes.data,
                              out.ctypes.data, xy.ctypes.data)
    return out, xy


def host_threads(cap: int = 16) -> int:
    """CPU threads this process may use, capped (the GPU box's share per GPU is 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


def fractal_search_batch_par(org, ref, R, req, threads: int | None = None):
    """fractal_search_batch over `threads` threads (ctypes drops the GIL for the
    call; the restatement is a pure function of its arguments)."""
    from concurrent.futures import ThreadPoolExecutor
    req = np.ascontiguousarray(req, np.int32)
    threads = threads or host_threads()
    parts = np.array_split(np.arange(len(req)), threads)
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(lambda ix: fractal_search_batch(org, ref, R, req[ix]), parts))
    return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])


def fractal_box_sums(plane, bsx, bsy):
    lib = load_fractal()
    plane = np.ascontiguousarray(plane, np.uint8)
    h, w = plane.shape
    s = np.zeros((h - bsy + 1, w - bsx + 1), np.float64)
    s2 = np.zeros_like(s)
    lib.fro_box_sums(plane.ctypes.data, w, w, h, bsx, bsy, s.ctypes.data, s2.ctypes.data)
    return s, s2


FRO_NODE = np.dtype([("rms", "<f8"), ("scale", "<f8"), ("offset", "<f8"), ("x", "<i4"), ("y", "<i4"),
                     ("reference", "<i4"), ("partition", "<i4")])
FRO_MB = np.dtype([("mb", FRO_NODE), ("b8", FRO_NODE, (4,)), ("sub", FRO_NODE, (4, 4)), ("chun", "<f8")])
assert FRO_NODE.itemsize == 40 and FRO_MB.itemsize == 848


def fractal_encode_mbs(org, refs, R, tol_16, tol_8):
    """encode_one_macroblock for every macroblock of org (H x W, multiples of
    16) against the reference views refs (list of H x W uint8) -> FRO_MB [n_mb]"""
    lib = load_fractal()
    org = np.ascontiguousarray(org, np.uint8)
    refs = [np.ascontiguousarray(r, np.uint8) for r in refs]
    h, w = org.shape
    ptrs = (ctypes.c_void_p * len(refs))(*[r.ctypes.data for r in refs])
    out = np.zeros((w // 16) * (h // 16), FRO_MB)
    lib.fro_encode_mbs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
    lib.fro_encode_mbs(org.ctypes.data, ptrs, len(refs), w, w, h, int(R), float(tol_16), float(tol_8),
                       out.ctypes.data)
    return out


# ---- JM EPZS integer search (oracle/epzs_oracle.c, pinned against JM captures) --
EPZS_REQ = np.dtype([("pos_x", "<i2"), ("pos_y", "<i2"), ("bsx", "<i2"), ("bsy", "<i2"),
                     ("blocktype", "<i2"), ("ref_idx", "<i2"), ("pred_x", "<i2"), ("pred_y", "<i2"),
                     ("center_x", "<i2"), ("center_y", "<i2"), ("max_x", "<i2"), ("max_y", "<i2"),
                     ("lambda", "<i4"), ("variant", "u1"), ("flags", "u1"), ("pattern", "u1"), ("dual", "u1"),
                     ("n_pred", "<i4"), ("pred_off", "<i4"), ("n_stale", "<i4"), ("stale_off", "<i4"),
                     ("plane", "<i4"), ("pad", "<i4"),
                     ("prev_sad", "<i8"), ("medthres", "<i8"), ("stop_crit", "<i8")])
EPZS_RES = np.dtype([("mv_x", "<i2"), ("mv_y", "<i2"), ("path", "<i4"), ("cost", "<i8"), ("prev_sad", "<i8")])
assert EPZS_REQ.itemsize == 80 and EPZS_RES.itemsize == 24
EP_SO = os.path.join(ORACLE_DIR, "build", "libepzs_oracle.so")
EP16_SO = os.path.join(ORACLE_DIR, "build", "libepzs_oracle16.so")   # 16-bit samples (-DEO_PEL16)
_ep = {}


def load_epzs(wide: bool = False) -> ctypes.CDLL:
    if wide in _ep:
        return _ep[wide]
    so = EP16_SO if wide else EP_SO
    src = os.path.join(ORACLE_DIR, "epzs_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "port"], check=True)
    lib = ctypes.CDLL(so)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.eo_epzs_batch.argtypes = [P, I, P, P, P, P, I, I, I, P]
    _ep[wide] = lib
    return lib


def epzs_batch(req, preds, stale, cur, refs):
    """req EPZS_REQ[n]; preds/stale int16 [k, 2] pools; cur / refs[plane] HxW -> EPZS_RES[n];
    uint16 planes (SourceBitDepthLuma 9..14) go to the 16-bit build of the restatement"""
    wide = np.asarray(cur).dtype == np.uint16
    pel = np.uint16 if wide else np.uint8
    lib = load_epzs(wide)
    req = np.ascontiguousarray(req, EPZS_REQ)
    preds = np.ascontiguousarray(preds, np.int16).reshape(-1, 2)
    stale = np.ascontiguousarray(stale, np.int16).reshape(-1, 2)
    if len(preds) == 0:
        preds = np.zeros((1, 2), np.int16)
    if len(stale) == 0:
        stale = np.zeros((1, 2), np.int16)
    cur = np.ascontiguousarray(cur, pel)
    refs = [np.ascontiguousarray(r, pel) for r in refs]
    h, w = cur.shape
    ptrs = (ctypes.c_void_p * len(refs))(*[r.ctypes.data for r in refs])
    out = np.zeros(len(req), EPZS_RES)
    lib.eo_epzs_batch(req.ctypes.data, len(req), preds.ctypes.data, stale.ctypes.data, cur.ctypes.data, ptrs, w, w, h,
                      out.ctypes.data)
    return out


# ---- sub-pel interpolation and refinement (oracle/subpel_oracle.c) ----------
SPO_REQ = np.dtype([("pos_x", "<i4"), ("pos_y", "<i4"), ("bsx", "<i4"), ("bsy", "<i4"), ("blocktype", "<i4"),
                    ("ref", "<i4"), ("pred_x", "<i4"), ("pred_y", "<i4"), ("mv_x", "<i4"), ("mv_y", "<i4"),
                    ("min_mcost", "<i8"), ("lambda_h", "<i4"), ("lambda_q", "<i4"), ("rdopt", "<i4"),
                    ("slice_type", "<i4"), ("start_hp", "<i4"), ("start_qp", "<i4"), ("metric_h", "<i4"),
                    ("metric_q", "<i4"), ("test8x8", "<i4"), ("search_pos2", "<i4"), ("search_pos4", "<i4"),
                    ("pad", "<i4"), ("subthres", "<i8")], align=True)
SP_SO = os.path.join(ORACLE_DIR, "build", "libsubpel_oracle.so")
_sp = None


def load_subpel() -> ctypes.CDLL:
    global _sp
    if _sp is not None:
        return _sp
    src = os.path.join(ORACLE_DIR, "subpel_oracle.c")
    if not os.path.exists(SP_SO) or os.path.getmtime(SP_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "port"], check=True)
    lib = ctypes.CDLL(SP_SO)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.spo_sub_images.argtypes = [P, I, I, P]
    lib.spo_set_bitdepth.argtypes = [I]
    lib.spo_sub_pel_batch.argtypes = [P, P, I, I, P, I, I, P, P]
    _sp = lib
    return lib


def sub_images(plane: np.ndarray, bits: int = 8) -> np.ndarray:
    """getSubImagesLuma of an HxW plane -> uint16 [16, H+40, W+64] (JM's padded sub-images);
    bits = SourceBitDepthLuma (the six-tap clip bound)"""
    lib = load_subpel()
    src = np.ascontiguousarray(plane, np.uint16)
    h, w = src.shape
    out = np.zeros((16, h + 40, w + 64), np.uint16)
    lib.spo_set_bitdepth(int(bits))
    try:
        lib.spo_sub_images(src.ctypes.data, w, h, out.ctypes.data)
    finally:
        lib.spo_set_bitdepth(8)
    return out


def sub_pel_batch(cur: np.ndarray, sub: np.ndarray, req: np.ndarray, epzs: bool):
    """req SPO_REQ[n] against one reference's sub-images -> (mv int16 [n,2], cost int64 [n])"""
    lib = load_subpel()
    cur = np.ascontiguousarray(cur, np.uint16)
    sub = np.ascontiguousarray(sub, np.uint16)
    req = np.ascontiguousarray(req, SPO_REQ)
    h, w = cur.shape
    mv = np.zeros((len(req), 2), np.int16)
    cost = np.zeros(len(req), np.int64)
    lib.spo_sub_pel_batch(cur.ctypes.data, sub.ctypes.data, w, h, req.ctypes.data, len(req), int(epzs),
                          mv.ctypes.data, cost.ctypes.data)
    return mv, cost


def epzs_grid_batch(req, preds, stale, cur, refs, bits=8):
    """EPZSSubPelGrid = 1 searches (variants 2 / 3) against the sub-images of refs[plane] -> EPZS_RES[n];
    bits > 8: uint16 planes and 16-bit sub-images clipped to (1 << bits) - 1"""
    wide = bits > 8
    pel = np.uint16 if wide else np.uint8
    lib = load_epzs(wide)
    if not hasattr(lib, "_grid_sig"):
        P, I = ctypes.c_void_p, ctypes.c_int
        lib.eo_epzs_grid_batch.argtypes = [P, I, P, P, P, I, P, I, I, P]
        lib._grid_sig = True
    req = np.ascontiguousarray(req, EPZS_REQ)
    preds = np.ascontiguousarray(preds, np.int16).reshape(-1, 2)
    stale = np.ascontiguousarray(stale, np.int16).reshape(-1, 2)
    if len(preds) == 0:
        preds = np.zeros((1, 2), np.int16)
    if len(stale) == 0:
        stale = np.zeros((1, 2), np.int16)
    cur = np.ascontiguousarray(cur, pel)
    subs = [np.ascontiguousarray(sub_images(r, bits).astype(pel)) for r in refs]
    h, w = cur.shape
    ptrs = (ctypes.c_void_p * len(subs))(*[s.ctypes.data for s in subs])
    out = np.zeros(len(req), EPZS_RES)
    lib.eo_epzs_grid_batch(req.ctypes.data, len(req), preds.ctypes.data, stale.ctypes.data, cur.ctypes.data, w, ptrs,
                           w, h, out.ctypes.data)
    return out


EPZS_BOUNDS = np.dtype([("stop_lo", "<i8"), ("stop_hi", "<i8"), ("prev_lo", "<i8"), ("prev_hi", "<i8"),
                        ("prev_written", "<i4"), ("n_visited", "<i4")])
assert EPZS_BOUNDS.itemsize == 40


def epzs_spec_batch(req, preds, cond, stale, cur, refs, grid: bool, bits=8, max_vis=64, subs=None):
    """eo_epzs_ex / eo_epzs_grid_ex: the searches with predictor conditions (cond
    uint8 parallel to preds, or None) and their validity intervals -> (EPZS_RES[n],
    EPZS_BOUNDS[n], visited int16 [n, max_vis, 2]); subs: prebuilt sub-images per
    ref (grid), else built here"""
    wide = bits > 8
    pel = np.uint16 if wide else np.uint8
    lib = load_epzs(wide)
    if not hasattr(lib, "_ex_sig"):
        P, I = ctypes.c_void_p, ctypes.c_int
        lib.eo_epzs_ex_batch.argtypes = [P, I, P, P, P, P, P, I, I, I, P, P, P, I]
        lib.eo_epzs_grid_ex_batch.argtypes = [P, I, P, P, P, P, I, P, I, I, P, P, P, I]
        lib._ex_sig = True
    req = np.ascontiguousarray(req, EPZS_REQ)
    preds = np.ascontiguousarray(preds, np.int16).reshape(-1, 2)
    stale = np.ascontiguousarray(stale, np.int16).reshape(-1, 2)
    if len(preds) == 0:
        preds = np.zeros((1, 2), np.int16)
    if len(stale) == 0:
        stale = np.zeros((1, 2), np.int16)
    cnd = None if cond is None else np.ascontiguousarray(cond, np.uint8)
    if cnd is not None and len(cnd) == 0:
        cnd = np.zeros(1, np.uint8)
    cur = np.ascontiguousarray(cur, pel)
    h, w = cur.shape
    out = np.zeros(len(req), EPZS_RES)
    bnd = np.zeros(len(req), EPZS_BOUNDS)
    vis = np.zeros((len(req), max_vis, 2), np.int16)
    cptr = None if cnd is None else cnd.ctypes.data
    if grid:
        if subs is None:
            subs = [np.ascontiguousarray(sub_images(r, bits).astype(pel)) for r in refs]
        ptrs = (ctypes.c_void_p * len(subs))(*[x.ctypes.data for x in subs])
        lib.eo_epzs_grid_ex_batch(req.ctypes.data, len(req), preds.ctypes.data, cptr, stale.ctypes.data,
                                  cur.ctypes.data, w, ptrs, w, h, out.ctypes.data, bnd.ctypes.data, vis.ctypes.data,
                                  max_vis)
    else:
        refs = [np.ascontiguousarray(r, pel) for r in refs]
        ptrs = (ctypes.c_void_p * len(refs))(*[r.ctypes.data for r in refs])
        lib.eo_epzs_ex_batch(req.ctypes.data, len(req), preds.ctypes.data, cptr, stale.ctypes.data, cur.ctypes.data,
                             ptrs, w, w, h, out.ctypes.data, bnd.ctypes.data, vis.ctypes.data, max_vis)
    return out, bnd, vis


def fractal_decode_mbs(mbs, views, component=1):
    """fro_decode_mbs: the thesis decoder (block_dec.c) -> (rc, rec H x W uint8)"""
    lib = load_fractal()
    views = [np.ascontiguousarray(v, np.uint8) for v in views]
    h, w = views[0].shape
    mbs = np.ascontiguousarray(mbs, FRO_MB)
    ptrs = (ctypes.c_void_p * len(views))(*[v.ctypes.data for v in views])
    rec = np.zeros((h, w), np.uint8)
    lib.fro_decode_mbs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.fro_decode_mbs.restype = ctypes.c_int
    rc = lib.fro_decode_mbs(mbs.ctypes.data, ptrs, len(views), w, w, h, int(component), rec.ctypes.data)
    return rc, rec
