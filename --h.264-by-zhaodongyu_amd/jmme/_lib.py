"""ctypes binding of libjmme.so (the C ABI declared in include/jmme.h).

The product path: every search call below runs the HIP kernels in libjmme.so.
There is no CPU fallback -- if the library is missing this module raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# JMME_LIB: A/B experiments with an alternative in-tree build (lib/variants/...)
LIB_PATH = os.environ.get("JMME_LIB") or os.path.join(PKG_DIR, "lib", "libjmme.so")

NSLOT = 41
DISTBLK_MAX = 0x7FFFFFFF << 5
FULL_SEARCH = -1
FAST_FULL_SEARCH = 0
BLK_CHECK00 = 1

BLOCK_REQ = np.dtype([("pred_x", "<i2"), ("pred_y", "<i2"), ("center_x", "<i2"), ("center_y", "<i2"),
                      ("search_range", "<i2"), ("flags", "<i2"), ("lambda", "<i4")])
MB_REQ = np.dtype([("mb_x", "<i2"), ("mb_y", "<i2"), ("list", "<i2"), ("ref_idx", "<i2"),
                   ("slot_mask", "<u8"),
                   ("ffs_center_x", "<i2"), ("ffs_center_y", "<i2"), ("ffs_range", "<i2"),
                   ("ffs_pos00_valid", "<i2"), ("reserved", "<i2", (4,)),
                   ("blk", BLOCK_REQ, (NSLOT,))])
BLOCK_RES = np.dtype([("mv_x", "<i2"), ("mv_y", "<i2"), ("reserved", "<i4"), ("cost", "<i8")])
CHAIN_MAX_STEPS, NB_UNAVAILABLE, NB_FIXED = 4, -1, -2
CHAIN_NB = np.dtype([("src", "<i2"), ("ref_idx", "<i2"), ("mv_x", "<i2"), ("mv_y", "<i2")])
CHAIN_STEP = np.dtype([("slot", "<i2"), ("flags", "<i2"), ("nb", CHAIN_NB, (3,)), ("sr_min_x", "<i2"),
                       ("sr_max_x", "<i2"), ("sr_min_y", "<i2"), ("sr_max_y", "<i2")])
CHAIN = np.dtype([("mb_x", "<i2"), ("mb_y", "<i2"), ("list", "<i2"), ("ref_idx", "<i2"), ("n_steps", "<i2"),
                  ("rdopt", "<i2"), ("ffs_center_x", "<i2"), ("ffs_center_y", "<i2"), ("ffs_range", "<i2"),
                  ("ffs_pos00_valid", "<i2"), ("mv_lim_x0", "<i2"), ("mv_lim_x1", "<i2"), ("mv_lim_y0", "<i2"),
                  ("mv_lim_y1", "<i2"), ("lambda", "<i4"), ("steps", CHAIN_STEP, (4,))])
CHAIN_RES = np.dtype([("pred_x", "<i2"), ("pred_y", "<i2"), ("center_x", "<i2"), ("center_y", "<i2"),
                      ("range_min", "<i2"), ("range_max", "<i2"), ("mv_x", "<i2"), ("mv_y", "<i2"), ("cost", "<i8")])
FRACTAL_REQ = np.dtype([("block_x", "<i2"), ("block_y", "<i2"), ("bsx", "<i2"), ("bsy", "<i2")])
FRACTAL_RES = np.dtype([("rms", "<f8"), ("scale", "<f8"), ("offset", "<f8"), ("x", "<i4"), ("y", "<i4")])
FRACTAL_NODE = np.dtype([("rms", "<f8"), ("scale", "<f8"), ("offset", "<f8"), ("x", "<i4"), ("y", "<i4"),
                         ("reference", "<i4"), ("partition", "<i4")])
FRACTAL_MB = np.dtype([("mb", FRACTAL_NODE), ("b8", FRACTAL_NODE, (4,)), ("sub", FRACTAL_NODE, (4, 4)),
                       ("chun", "<f8")])
FRACTAL_MAX_VIEWS = 4
EPZS_REQ = np.dtype([("pos_x", "<i2"), ("pos_y", "<i2"), ("bsx", "<i2"), ("bsy", "<i2"),
                     ("blocktype", "<i2"), ("ref_idx", "<i2"), ("pred_x", "<i2"), ("pred_y", "<i2"),
                     ("center_x", "<i2"), ("center_y", "<i2"), ("max_x", "<i2"), ("max_y", "<i2"),
                     ("lambda", "<i4"), ("variant", "u1"), ("flags", "u1"), ("pattern", "u1"), ("dual", "u1"),
                     ("n_pred", "<i4"), ("pred_off", "<i4"), ("n_stale", "<i4"), ("stale_off", "<i4"),
                     ("ref_slot", "<i4"), ("reserved", "<i4"),
                     ("prev_sad", "<i8"), ("medthres", "<i8"), ("stop_crit", "<i8")])
EPZS_RES = np.dtype([("mv_x", "<i2"), ("mv_y", "<i2"), ("path", "<i4"), ("cost", "<i8"), ("prev_sad", "<i8"),
                     ("motion_x", "<i2"), ("motion_y", "<i2"), ("n_visited", "<i4")])
EPZS_FRAME, EPZS_PSLICE = 1, 2
EPZS_BOUNDS = np.dtype([("stop_lo", "<i8"), ("stop_hi", "<i8"), ("prev_lo", "<i8"), ("prev_hi", "<i8"),
                        ("prev_written", "<i4"), ("n_visited", "<i4")])
SUBPEL_REQ = np.dtype([("pos_x", "<i2"), ("pos_y", "<i2"), ("blocktype", "<i2"), ("ref_slot", "<i2"),
                       ("pred_x", "<i2"), ("pred_y", "<i2"), ("mv_x", "<i2"), ("mv_y", "<i2"),
                       ("lambda_h", "<i4"), ("lambda_q", "<i4"), ("min_mcost", "<i8"), ("subthres", "<i8"),
                       ("variant", "u1"), ("flags", "u1"), ("metric_h", "u1"), ("metric_q", "u1"),
                       ("start_hp", "u1"), ("start_qp", "u1"), ("search_pos2", "u1"), ("search_pos4", "u1")])
SP_TEST8x8, SP_CHECK0 = 1, 2
SUBPEL_PAD_Y, SUBPEL_PAD_X = 20, 32
QUANT4x4_PARAMS = np.dtype([("scale", "<i4", (16,)), ("offset", "<i4", (16,)), ("inv_scale", "<i4", (16,)),
                            ("qp_per", "<i4"), ("is_cavlc", "<i4"), ("scan", "u1", (16, 2)), ("c_cost", "u1", (16,))])
RESID4x4_REQ = np.dtype([("ores", "<i4", (16,)), ("pred", "<u2", (16,)), ("param", "<i4"), ("max_pel", "<i4")])
RESID4x4_RES = np.dtype([("coef", "<i4", (16,)), ("rres", "<i4", (16,)), ("levels", "<i4", (17,)),
                         ("runs", "<i4", (16,)), ("cost", "<i4"), ("nonzero", "<i4"), ("zero", "<i4"),
                         ("recon", "<u2", (16,))])
TRANSFORM_OPS = {"forward4x4": (0, 16, 16), "inverse4x4": (1, 16, 16), "hadamard4x4": (2, 16, 16),
                 "ihadamard4x4": (3, 16, 16), "hadamard4x2": (4, 8, 8), "ihadamard4x2": (5, 8, 8),
                 "hadamard2x2": (6, 4, 4), "ihadamard2x2": (7, 4, 4), "forward8x8": (8, 64, 64),
                 "inverse8x8": (9, 64, 64)}   # name -> (jmme_transform_op, in elems, out elems)
assert BLOCK_REQ.itemsize == 16 and MB_REQ.itemsize == 688 and BLOCK_RES.itemsize == 16
assert RESID4x4_REQ.itemsize == 104 and RESID4x4_RES.itemsize == 304
assert QUANT4x4_PARAMS.itemsize == 248 and FRACTAL_REQ.itemsize == 8 and FRACTAL_RES.itemsize == 32
assert FRACTAL_NODE.itemsize == 40 and FRACTAL_MB.itemsize == 848
assert EPZS_REQ.itemsize == 80 and EPZS_RES.itemsize == 32 and SUBPEL_REQ.itemsize == 48
assert CHAIN_NB.itemsize == 8 and CHAIN_STEP.itemsize == 36 and CHAIN.itemsize == 176 and CHAIN_RES.itemsize == 24

CONFIG_FIELDS = ["SourceWidth", "SourceHeight", "SearchMode", "SearchRange", "NumberReferenceFrames",
                 "DisableSubpelME", "RDOptimization", "MEDistortionFPel", "MDDistortion", "EPZSSubPelGrid",
                 "RestrictSearchRange", "UseMVLimits", "SetMVXLimit", "SetMVYLimit", "ChromaMEEnable",
                 "SourceBitDepthLuma"]


class JmmeConfig(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int) for f in CONFIG_FIELDS]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f in CONFIG_FIELDS}


class JmmeMv(ctypes.Structure):
    _fields_ = [("mv_x", ctypes.c_int16), ("mv_y", ctypes.c_int16)]


class JmmeError(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise JmmeError(f"{LIB_PATH} not built: run __graft_entry__.build() (make -C <pkg>)")
    L = ctypes.CDLL(LIB_PATH)
    P, I, D, V = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, None
    sig = {
        "jmme_config_default": (I, [P]),
        "jmme_config_parse": (I, [P, ctypes.c_char_p, I, P]),
        "jmme_max_mvd": (I, [P]),
        "jmme_create": (P, [P, I]),
        "jmme_destroy": (V, [P]),
        "jmme_last_error": (ctypes.c_char_p, []),
        "jmme_version": (ctypes.c_char_p, []),
        "jmme_upload_cur": (I, [P, P, I, I]),
        "jmme_upload_ref": (I, [P, I, I, P, I, I]),
        "jmme_slot": (I, [I, I, I]),
        "jmme_search_mbs": (I, [P, I, P, I, P]),
        "jmme_search_mbs_chains": (I, [P, I, P, I, P, P, I, P]),
        "jmme_search_mbs_chains_sp": (I, [P, I, P, I, P, P, I, P, P, P]),
        "jmme_search_mbs_async": (I, [P, I, P, I, P, P]),
        "jmme_search_mbs_planes_async": (I, [P, I, P, P, I, I, I, P, I, P, P]),
        "jmme_search_status": (I, [P, P]),
        "jmme_set_small_batch_limit": (I, [P, I]),
        "jmme_prepare": (I, [P]),
        "jmme_reserve": (I, [P, I]),
        "jmme_full_search_block": (ctypes.c_int64, [P, I, I, I, I, I, P, P, ctypes.c_int64, I, I, I]),
        "jmme_fast_full_search_block": (ctypes.c_int64, [P, I, I, I, I, I, P, P, I, I, I, P, ctypes.c_int64, I]),
        "jmme_last_kernel_ms": (ctypes.c_float, [P]),
        "jmme_transform": (I, [P, I, P, P, I]),
        "jmme_transform_async": (I, [P, I, P, P, I, P]),
        "jmme_satd": (I, [P, I, P, P, I]),
        "jmme_satd_async": (I, [P, I, P, P, I, P]),
        "jmme_quant4x4": (I, [P, P, I, P, P, P, P, P, P, I]),
        "jmme_residual4x4": (I, [P, P, I, P, P, I]),
        "jmme_fractal_search": (I, [P, P, P, I, I, I, I, P, I, P]),
        "jmme_fractal_words_async": (I, [P, P, I, I, I, P, P]),
        "jmme_fractal_search_async": (I, [P, P, I, P, I, I, I, P, I, P, P]),
        "jmme_fractal_box_sums": (I, [P, P, I, I, I, I, I, P, P]),
        "jmme_fractal_set_pool_min_range": (I, [P, I]),
        "jmme_fractal_pool_survivors": (I, [P, P]),
        "jmme_fractal_set_pool_mfma": (I, [P, I]),
        "jmme_fractal_encode_mbs": (I, [P, P, P, I, I, I, I, I, D, D, P]),
        "jmme_epzs_search": (I, [P, P, I, P, I, P, I, P]),
        "jmme_epzs_search_async": (I, [P, P, I, P, P, P, P]),
        "jmme_epzs_search_ex": (I, [P, P, I, P, P, I, P, I, P, P, I]),
        "jmme_epzs_speculate": (I, [P, P, I, P, P, I, P, I, P, P, P, I, P, P]),
        "jmme_fractal_encode_mbs_async": (I, [P, P, P, I, P, I, I, I, I, D, D, P, P]),
        "jmme_fractal_encode_mb_rows_async": (I, [P, P, P, I, P, I, I, I, I, I, I, D, D, P, P]),
        "jmme_fractal_decode_mbs": (I, [P, P, P, I, I, I, I, I, P]),
        "jmme_fractal_decode_mbs_async": (I, [P, P, P, I, I, I, I, I, P, P, P]),
        "jmme_quant4x4_async": (I, [P, P, P, P, P, P, P, P, I, P]),
        "jmme_interpolate_ref": (I, [P, I, I, P]),
        "jmme_get_sub_images": (I, [P, I, I, P]),
        "jmme_sub_images_async": (I, [P, P, I, I, I, P, I, ctypes.c_size_t, P]),
        "jmme_subpel_validate": (I, [P, P, I]),
        "jmme_subpel_refine": (I, [P, P, I, P]),
        "jmme_subpel_refine_async": (I, [P, P, I, P, P, P]),
        "jmme_spiral_index": (I, [I, I]),
        "jmme_spiral_offset": (V, [I, P, P]),
        "jmme_mvbits": (I, [I]),
        "jmme_debug_window": (I, [P, I, P, P, I]),
        "jmme_debug_stamps": (I, [P, P, I]),
    }
    optional = {"jmme_debug_stamps"}   # absent from older builds (A/B baselines)
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int) -> None:
    if status != 0:
        raise JmmeError(lib().jmme_last_error().decode())


def ptr(a: np.ndarray) -> ctypes.c_void_p:
    return a.ctypes.data_as(ctypes.c_void_p)
