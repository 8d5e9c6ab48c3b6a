"""Host mirror of JM 18.5's integer-pel ME entry points over libjmme.so.

JM 18.5 (JM = /root/reference/4.对比程序/jm18.5/JM) reference points:
  * config keys / -d file -p k=v   JM/lencod/src/configfile.c:314 (Configure)
  * frame buffers                  get_mem2Dpel JM/lcommon/src/memalloc.c:864
  * IntPelME contract              JM/lencod/inc/global.h:459,
                                   me_fullsearch.c:39 / me_fullfast.c:618
  * per-MB partition searches      PartitionMotionSearch mv_search.c:1564,
                                   SubPartitionMotionSearch mv_search.c:1686
"""
from __future__ import annotations

import ctypes
from typing import Mapping

import numpy as np

from . import _lib
from ._lib import BLOCK_RES, MB_REQ, NSLOT, JmmeConfig, JmmeMv, check, lib, ptr


def config_from_cfg(cfg_path: str | None = None, overrides: Mapping[str, object] | None = None) -> JmmeConfig:
    """JM's `lencod -d cfg_path -p Key=Value ...` for the ME keys."""
    c = JmmeConfig()
    check(lib().jmme_config_default(ctypes.byref(c)))
    args = [f"{k}={v}".encode() for k, v in (overrides or {}).items()]
    argv = (ctypes.c_char_p * max(1, len(args)))(*args)
    check(lib().jmme_config_parse(ctypes.byref(c), cfg_path.encode() if cfg_path else None, len(args),
                                  ctypes.cast(argv, ctypes.c_void_p)))
    return c


def slot_of(blocktype: int, block_x: int, block_y: int) -> int:
    return int(lib().jmme_slot(int(blocktype), int(block_x), int(block_y)))


def spiral(R: int) -> np.ndarray:
    """JM's spiral_search order (integer pels), from the library's own formula."""
    n = (2 * R + 1) ** 2
    out = np.zeros((n, 2), dtype=np.int32)
    ox, oy = ctypes.c_int(), ctypes.c_int()
    for i in range(n):
        lib().jmme_spiral_offset(i, ctypes.byref(ox), ctypes.byref(oy))
        out[i] = (ox.value, oy.value)
    return out


def _rows(plane: np.ndarray):
    """get_mem2Dpel layout: one uint16 allocation + a row-pointer array."""
    p = np.ascontiguousarray(plane, dtype=np.uint16)
    h, w = p.shape
    base = p.ctypes.data
    rows = (ctypes.c_void_p * h)(*[base + 2 * w * y for y in range(h)])
    return p, rows


class MotionEstimator:
    """One libjmme context: a device, the current picture and the DPB references."""

    def __init__(self, cfg: JmmeConfig | Mapping[str, object] | None = None, device: int = -1):
        if cfg is None or isinstance(cfg, Mapping):
            cfg = config_from_cfg(None, cfg or {})
        self.cfg = cfg
        self._ctx = lib().jmme_create(ctypes.byref(cfg), int(device))
        if not self._ctx:
            raise _lib.JmmeError(lib().jmme_last_error().decode())
        self.max_mvd = int(lib().jmme_max_mvd(ctypes.byref(cfg)))

    def close(self) -> None:
        if self._ctx:
            lib().jmme_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- frame buffers -------------------------------------------------
    def upload_cur(self, plane: np.ndarray) -> None:
        keep, rows = _rows(plane)
        self._shape = keep.shape
        check(lib().jmme_upload_cur(self._ctx, ctypes.cast(rows, ctypes.c_void_p), keep.shape[1], keep.shape[0]))

    def upload_ref(self, list_idx: int, ref_idx: int, plane: np.ndarray) -> None:
        keep, rows = _rows(plane)
        self._shape = keep.shape
        check(lib().jmme_upload_ref(self._ctx, int(list_idx), int(ref_idx), ctypes.cast(rows, ctypes.c_void_p),
                                    keep.shape[1], keep.shape[0]))

    # ---- searches ------------------------------------------------------
    def search(self, mode: int, req: np.ndarray) -> np.ndarray:
        """Batched per-MB search; returns BLOCK_RES [n, 41] (unsearched slots zero)."""
        req = np.ascontiguousarray(req, dtype=MB_REQ)
        out = np.zeros((req.shape[0], NSLOT), dtype=BLOCK_RES)
        check(lib().jmme_search_mbs(self._ctx, int(mode), ptr(req), req.shape[0], ptr(out)))
        return out

    def search_chains(self, mode: int, req: np.ndarray, chains: np.ndarray):
        """jmme_search_mbs_chains: the batch (BLOCK_RES [n, 41]) and the chains'
        steps (CHAIN_RES [n_chains, 4]) in one round trip."""
        req = np.ascontiguousarray(req, dtype=MB_REQ)
        chains = np.ascontiguousarray(chains, dtype=_lib.CHAIN)
        out = np.zeros((req.shape[0], NSLOT), dtype=BLOCK_RES)
        res = np.zeros((len(chains), _lib.CHAIN_MAX_STEPS), dtype=_lib.CHAIN_RES)
        check(lib().jmme_search_mbs_chains(self._ctx, int(mode), ptr(req), req.shape[0], ptr(out), ptr(chains),
                                           len(chains), ptr(res)))
        return out, res

    def search_chains_sp(self, mode: int, req: np.ndarray, chains: np.ndarray, sp: np.ndarray):
        """jmme_search_mbs_chains_sp: chains whose steps run SubPelME too; sp is
        one SUBPEL_REQ template per chain.  Returns (batch BLOCK_RES [n, 41],
        CHAIN_RES [n_chains, 4] integer answers, BLOCK_RES [n_chains, 4] refined)."""
        req = np.ascontiguousarray(req, dtype=MB_REQ)
        chains = np.ascontiguousarray(chains, dtype=_lib.CHAIN)
        sp = np.ascontiguousarray(sp, dtype=_lib.SUBPEL_REQ)
        if len(sp) != len(chains):
            raise ValueError("one sub-pel template per chain")
        out = np.zeros((req.shape[0], NSLOT), dtype=BLOCK_RES)
        res = np.zeros((len(chains), _lib.CHAIN_MAX_STEPS), dtype=_lib.CHAIN_RES)
        spo = np.zeros((len(chains), _lib.CHAIN_MAX_STEPS), dtype=BLOCK_RES)
        check(lib().jmme_search_mbs_chains_sp(self._ctx, int(mode), ptr(req), req.shape[0], ptr(out), ptr(chains),
                                              len(chains), ptr(sp), ptr(res), ptr(spo)))
        return out, res, spo

    def search_async(self, mode: int, d_req: int, n: int, d_out: int, stream: int = 0) -> None:
        """Device-resident variant: d_req/d_out are device addresses (e.g. torch data_ptr())."""
        check(lib().jmme_search_mbs_async(self._ctx, int(mode), ctypes.c_void_p(d_req), int(n),
                                          ctypes.c_void_p(d_out), ctypes.c_void_p(stream)))

    def search_planes_async(self, mode: int, d_cur: int, d_ref: int, pitch: int, width: int, height: int,
                            d_req: int, n: int, d_out: int, stream: int = 0) -> None:
        check(lib().jmme_search_mbs_planes_async(self._ctx, int(mode), ctypes.c_void_p(d_cur),
                                                 ctypes.c_void_p(d_ref), int(pitch), int(width), int(height),
                                                 ctypes.c_void_p(d_req), int(n), ctypes.c_void_p(d_out),
                                                 ctypes.c_void_p(stream)))

    def set_small_batch_limit(self, max_workgroups: int) -> None:
        """Largest batch (in 16x16-position workgroups) `search` serves by the low-latency path; 0: never."""
        check(lib().jmme_set_small_batch_limit(self._ctx, int(max_workgroups)))

    def prepare(self, max_units: int = 0) -> None:
        """Pay start-up costs now (jmme_prepare: every kernel launched once) and, with
        max_units, size the batch / staging / plane buffers (jmme_reserve)."""
        check(lib().jmme_prepare(self._ctx))
        if max_units:
            check(lib().jmme_reserve(self._ctx, int(max_units)))

    def search_status(self, stream: int = 0) -> None:
        """Raise if the last device-request search refused a request (synchronises)."""
        check(lib().jmme_search_status(self._ctx, ctypes.c_void_p(stream)))

    def last_kernel_ms(self) -> float:
        return float(lib().jmme_last_kernel_ms(self._ctx))

    def full_search_block(self, list_idx, ref_idx, pos_x, pos_y, blocktype, pred, center,
                          lambda_factor, search_range, check_for_00, min_mcost=_lib.DISTBLK_MAX):
        """full_search_motion_estimation's contract for one partition (JM global.h:459)."""
        p = JmmeMv(int(pred[0]), int(pred[1]))
        mv = JmmeMv(int(center[0]), int(center[1]))
        cost = lib().jmme_full_search_block(self._ctx, int(list_idx), int(ref_idx), int(pos_x), int(pos_y),
                                            int(blocktype), ctypes.byref(p), ctypes.byref(mv), int(min_mcost),
                                            int(lambda_factor), int(search_range), int(check_for_00))
        return (mv.mv_x, mv.mv_y), int(cost)

    # ---- transforms / quant / SATD -----------------------
    def transform(self, op: str, blocks: np.ndarray) -> np.ndarray:
        """JM transform `op` (forward4x4, inverse8x8, ...) of n row-major blocks."""
        code, ein, eout = _lib.TRANSFORM_OPS[op]
        blocks = np.ascontiguousarray(blocks, np.int32).reshape(-1, ein)
        out = np.empty((blocks.shape[0], eout), np.int32)
        check(lib().jmme_transform(self._ctx, code, ptr(blocks), ptr(out), blocks.shape[0]))
        return out

    def transform_async(self, op: str, d_in: int, d_out: int, n: int, stream: int = 0) -> None:
        check(lib().jmme_transform_async(self._ctx, _lib.TRANSFORM_OPS[op][0], d_in, d_out, int(n), stream))

    def satd(self, size: int, diff: np.ndarray) -> np.ndarray:
        """HadamardSAD4x4 / HadamardSAD8x8 of n int16 residual blocks."""
        diff = np.ascontiguousarray(diff, np.int16).reshape(-1, size * size)
        out = np.empty(diff.shape[0], np.int32)
        check(lib().jmme_satd(self._ctx, int(size), ptr(diff), ptr(out), diff.shape[0]))
        return out

    def satd_async(self, size: int, d_diff: int, d_out: int, n: int, stream: int = 0) -> None:
        check(lib().jmme_satd_async(self._ctx, int(size), d_diff, d_out, int(n), stream))

    def quant4x4(self, params: np.ndarray, coef: np.ndarray, coeff_cost: np.ndarray | None = None,
                 param_idx: np.ndarray | None = None):
        """quant_4x4_normal over n blocks -> (coef_out, levels[n,17], runs[n,16], coeff_cost, nonzero)."""
        params = np.ascontiguousarray(params, _lib.QUANT4x4_PARAMS).reshape(-1)
        coef = np.array(coef, np.int32).reshape(-1, 16)
        n = coef.shape[0]
        cost = np.zeros(n, np.int32) if coeff_cost is None else np.array(coeff_cost, np.int32).reshape(n)
        levels = np.empty((n, 17), np.int32)
        runs = np.empty((n, 16), np.int32)
        nz = np.empty(n, np.int32)
        idx = None if param_idx is None else np.ascontiguousarray(param_idx, np.int32).reshape(n)
        check(lib().jmme_quant4x4(self._ctx, ptr(params), params.shape[0], None if idx is None else ptr(idx),
                                  ptr(coef), ptr(levels), ptr(runs), ptr(cost), ptr(nz), n))
        return coef, levels, runs, cost, nz

    def residual4x4(self, params: np.ndarray, ores: np.ndarray, pred: np.ndarray, param_idx=None,
                    max_pel: int = 255) -> np.ndarray:
        """residual_transform_quant_luma_4x4 of n inter blocks (JM/lencod/src/block.c:660-724):
        ores / pred [n, 16] -> RESID4x4_RES records (what JM leaves: levels, runs, cost,
        nonzero, the dequantised block, mb_rres and the reconstruction)."""
        params = np.ascontiguousarray(params, _lib.QUANT4x4_PARAMS).reshape(-1)
        ores = np.asarray(ores, np.int32).reshape(-1, 16)
        n = ores.shape[0]
        req = np.zeros(n, _lib.RESID4x4_REQ)
        req["ores"] = ores
        req["pred"] = np.asarray(pred).reshape(n, 16)
        req["param"] = 0 if param_idx is None else np.asarray(param_idx, np.int32).reshape(n)
        req["max_pel"] = max_pel
        res = np.zeros(n, _lib.RESID4x4_RES)
        check(lib().jmme_residual4x4(self._ctx, ptr(params), params.shape[0], ptr(req), ptr(res), n))
        return res

    def quant4x4_async(self, d_params: int, d_param_idx: int, d_coef: int, d_levels: int, d_runs: int,
                       d_coeff_cost: int, d_nonzero: int, n: int, stream: int = 0) -> None:
        check(lib().jmme_quant4x4_async(self._ctx, d_params, d_param_idx or None, d_coef, d_levels, d_runs,
                                        d_coeff_cost, d_nonzero, int(n), stream))

    # ---- thesis fractal domain-range search ------------------
    def fractal_search(self, org: np.ndarray, ref: np.ndarray, search_range: int, req: np.ndarray) -> np.ndarray:
        """full_search (ZL/src/block_enc.c:1933) for each request -> FRACTAL_RES[n]."""
        org = np.ascontiguousarray(org, np.uint8)
        ref = np.ascontiguousarray(ref, np.uint8)
        h, w = org.shape
        req = np.ascontiguousarray(req, _lib.FRACTAL_REQ)
        out = np.zeros(len(req), _lib.FRACTAL_RES)
        check(lib().jmme_fractal_search(self._ctx, ptr(org), ptr(ref), w, w, h, int(search_range), ptr(req),
                                        len(req), ptr(out)))
        return out

    def fractal_words_async(self, d_ref: int, pitch: int, width: int, height: int, d_words: int,
                            stream: int = 0) -> None:
        check(lib().jmme_fractal_words_async(self._ctx, d_ref, pitch, width, height, d_words, stream))

    def fractal_search_async(self, d_org: int, pitch: int, d_words: int, width: int, height: int, search_range: int,
                             d_req: int, n: int, d_out: int, stream: int = 0) -> None:
        check(lib().jmme_fractal_search_async(self._ctx, d_org, pitch, d_words, width, height, int(search_range),
                                              d_req, int(n), d_out, stream))

    def fractal_set_pool_min_range(self, min_range: int) -> None:
        """radius from which fractal_search runs the pruned pool search (0: always, huge: never)."""
        check(lib().jmme_fractal_set_pool_min_range(self._ctx, int(min_range)))

    def fractal_set_pool_mfma(self, on: bool) -> None:
        """4x4 full-pool bound test on the matrix cores (default) or on the VALU."""
        check(lib().jmme_fractal_set_pool_mfma(self._ctx, int(bool(on))))

    def fractal_pool_survivors(self) -> int:
        """exactly evaluated pool-search candidates since the last call (synchronises)."""
        v = np.zeros(1, np.uint64)
        check(lib().jmme_fractal_pool_survivors(self._ctx, ptr(v)))
        return int(v[0])

    def fractal_box_sums(self, plane: np.ndarray, bsx: int, bsy: int):
        """compute_domain_Sum for one block size -> (sum, sum2) float64 [(H-bsy+1), (W-bsx+1)]."""
        plane = np.ascontiguousarray(plane, np.uint8)
        h, w = plane.shape
        s = np.zeros((h - bsy + 1, w - bsx + 1), np.float64)
        s2 = np.zeros_like(s)
        check(lib().jmme_fractal_box_sums(self._ctx, ptr(plane), w, w, h, int(bsx), int(bsy), ptr(s), ptr(s2)))
        return s, s2

    def epzs_search(self, req: np.ndarray, preds: np.ndarray, stale: np.ndarray | None = None) -> np.ndarray:
        """EPZS_motion_estimation / EPZS_subMB_motion_estimation (JM me_epzs.c:54, 417) for each
        request against the uploaded current frame and reference slots -> EPZS_RES[n]."""
        req = np.ascontiguousarray(req, _lib.EPZS_REQ)
        preds = np.ascontiguousarray(preds, np.int16).reshape(-1, 2)
        stale = np.zeros((0, 2), np.int16) if stale is None else np.ascontiguousarray(stale, np.int16).reshape(-1, 2)
        out = np.zeros(len(req), _lib.EPZS_RES)
        check(lib().jmme_epzs_search(self._ctx, ptr(req), len(req), ptr(preds), len(preds), ptr(stale), len(stale),
                                     ptr(out)))
        return out

    def epzs_speculate(self, req: np.ndarray, preds: np.ndarray, cond: np.ndarray | None = None,
                       stale: np.ndarray | None = None, max_visited: int = 64, sp_req: np.ndarray | None = None):
        """jmme_epzs_speculate: the searches with their predictor conditions, validity
        intervals and stamped cells, and (sp_req) a chained EPZS sub-pel refinement
        of each result -> (EPZS_RES[n], EPZS_BOUNDS[n], visited int16 [n, max_visited, 2],
        BLOCK_RES[n] or None)."""
        req = np.ascontiguousarray(req, _lib.EPZS_REQ)
        preds = np.ascontiguousarray(preds, np.int16).reshape(-1, 2)
        stale = np.zeros((0, 2), np.int16) if stale is None else np.ascontiguousarray(stale, np.int16).reshape(-1, 2)
        cnd = None if cond is None else np.ascontiguousarray(cond, np.uint8)
        n = len(req)
        out = np.zeros(n, _lib.EPZS_RES)
        bnd = np.zeros(n, _lib.EPZS_BOUNDS)
        vis = np.zeros((n, max_visited, 2), np.int16)
        spq = None if sp_req is None else np.ascontiguousarray(sp_req, _lib.SUBPEL_REQ)
        spo = None if sp_req is None else np.zeros(n, _lib.BLOCK_RES)
        check(lib().jmme_epzs_speculate(self._ctx, ptr(req), n, ptr(preds), None if cnd is None else ptr(cnd),
                                        len(preds), ptr(stale), len(stale), ptr(out), ptr(bnd), ptr(vis),
                                        int(max_visited), None if spq is None else ptr(spq),
                                        None if spo is None else ptr(spo)))
        return out, bnd, vis, spo

    def epzs_search_async(self, d_req: int, n: int, d_preds: int, d_stale: int, d_out: int, stream: int = 0) -> None:
        check(lib().jmme_epzs_search_async(self._ctx, d_req, int(n), d_preds, d_stale, d_out, stream))

    # ---- quarter-pel planes and sub-pel refinement ----
    def sub_images(self, list_idx: int, ref_idx: int) -> np.ndarray:
        """getSubImagesLuma (JM img_luma.c:611) of an uploaded reference, in JM's padded layout:
        uint16 [16, H+40, W+64], plane dy*4+dx, padded row 0 = picture row -20."""
        h, w = self._shape
        out = np.zeros((16, h + 2 * _lib.SUBPEL_PAD_Y, w + 2 * _lib.SUBPEL_PAD_X), np.uint16)
        RowP = ctypes.POINTER(ctypes.c_uint16)
        keep = []
        quad = (ctypes.POINTER(ctypes.POINTER(RowP)) * 4)()
        for dy in range(4):
            pair = (ctypes.POINTER(RowP) * 4)()
            for dx in range(4):
                plane = out[dy * 4 + dx]
                rows = (RowP * plane.shape[0])(*[ctypes.cast(plane[j].ctypes.data + 2 * _lib.SUBPEL_PAD_X, RowP)
                                                 for j in range(plane.shape[0])])
                # JM's row pointer array is offset so [0] is picture row 0
                base = ctypes.addressof(rows) + _lib.SUBPEL_PAD_Y * ctypes.sizeof(RowP)
                pair[dx] = ctypes.cast(base, ctypes.POINTER(RowP))
                keep.append(rows)
            quad[dy] = ctypes.cast(pair, ctypes.POINTER(ctypes.POINTER(RowP)))
            keep.append(pair)
        check(lib().jmme_get_sub_images(self._ctx, int(list_idx), int(ref_idx), quad))
        return out

    def subpel_refine(self, req: np.ndarray) -> np.ndarray:
        """sub_pel_motion_estimation / EPZS_sub_pel_motion_estimation (JM me_fullsearch.c:186,
        me_epzs_sub.c:30) for each request -> BLOCK_RES[n] (mv, cost)."""
        req = np.ascontiguousarray(req, _lib.SUBPEL_REQ)
        out = np.zeros(len(req), _lib.BLOCK_RES)
        check(lib().jmme_subpel_refine(self._ctx, ptr(req), len(req), ptr(out)))
        return out

    def subpel_refine_async(self, d_req: int, n: int, d_int: int, d_out: int, stream: int = 0) -> None:
        check(lib().jmme_subpel_refine_async(self._ctx, d_req, int(n), d_int, d_out, stream))

    def subpel_validate(self, req: np.ndarray) -> None:
        req = np.ascontiguousarray(req, _lib.SUBPEL_REQ)
        check(lib().jmme_subpel_validate(self._ctx, ptr(req), len(req)))

    def sub_images_async(self, d_src: int, src_pitch: int, width: int, height: int, d_dst: int, dst_pitch: int,
                         plane_stride: int, stream: int = 0) -> None:
        check(lib().jmme_sub_images_async(self._ctx, d_src, src_pitch, width, height, d_dst, dst_pitch,
                                          plane_stride, stream))

    def fractal_encode_mbs(self, org: np.ndarray, refs, search_range: int, tol_16: float = 8.0,
                           tol_8: float = 5.0) -> np.ndarray:
        """encode_one_macroblock (ZL/src/block_enc.c:508) for every macroblock of org against the
        reference views refs (view 0 first) -> FRACTAL_MB[(W/16)*(H/16)], raster order."""
        org = np.ascontiguousarray(org, np.uint8)
        refs = [np.ascontiguousarray(r, np.uint8) for r in refs]
        h, w = org.shape
        if any(r.shape != org.shape for r in refs):
            raise ValueError("reference views must match the range plane's shape")
        ptrs = (ctypes.c_void_p * len(refs))(*[ptr(r) for r in refs])
        out = np.zeros((w // 16) * (h // 16), _lib.FRACTAL_MB)
        check(lib().jmme_fractal_encode_mbs(self._ctx, ptr(org), ptrs, len(refs), w, w, h, int(search_range),
                                            float(tol_16), float(tol_8), ptr(out)))
        return out

    def fractal_decode_mbs(self, mbs: np.ndarray, views, component: int = 1) -> np.ndarray:
        """decode_one_macroblock (ZL/src/block_dec.c:20) for every macroblock: the
        reconstructed H x W plane of `component` (1 Y, 2 U, 3 V) from the trees `mbs`
        (FRACTAL_MB, as fractal_encode_mbs returns them) and the decoder's views."""
        views = [np.ascontiguousarray(v, np.uint8) for v in views]
        h, w = views[0].shape
        mbs = np.ascontiguousarray(mbs, _lib.FRACTAL_MB)
        ptrs = (ctypes.c_void_p * len(views))(*[v.ctypes.data for v in views])
        rec = np.zeros((h, w), np.uint8)
        check(lib().jmme_fractal_decode_mbs(self._ctx, ptr(mbs), ptrs, len(views), w, w, h, int(component),
                                            ptr(rec)))
        return rec

    def fractal_decode_mbs_async(self, d_mbs: int, d_views, pitch: int, width: int, height: int, component: int,
                                 d_rec: int, d_status: int = 0, stream: int = 0) -> None:
        ptrs = (ctypes.c_void_p * len(d_views))(*d_views)
        check(lib().jmme_fractal_decode_mbs_async(self._ctx, d_mbs, ptrs, len(d_views), pitch, width, height,
                                                  int(component), d_rec, d_status or None, stream))

    def fractal_encode_mbs_async(self, d_org: int, d_ref0: int, pitch: int, d_words, width: int, height: int,
                                 search_range: int, tol_16: float, tol_8: float, d_out: int, stream: int = 0) -> None:
        """device form: d_words = list of per-view words images (fractal_words_async)."""
        ptrs = (ctypes.c_void_p * len(d_words))(*d_words)
        check(lib().jmme_fractal_encode_mbs_async(self._ctx, d_org, d_ref0, pitch, ptrs, len(d_words), width, height,
                                                  int(search_range), float(tol_16), float(tol_8), d_out, stream))

    def fractal_encode_mb_rows_async(self, d_org: int, d_ref0: int, pitch: int, d_words, width: int, height: int,
                                     mb_row0: int, mb_row1: int, search_range: int, tol_16: float, tol_8: float,
                                     d_out: int, stream: int = 0) -> None:
        """fractal_encode_mbs_async for the macroblock rows [mb_row0, mb_row1) only (an MB-row band):
        d_out receives (width/16)*(mb_row1-mb_row0) FRACTAL_MB records."""
        ptrs = (ctypes.c_void_p * len(d_words))(*d_words)
        check(lib().jmme_fractal_encode_mb_rows_async(self._ctx, d_org, d_ref0, pitch, ptrs, len(d_words), width,
                                                      height, int(mb_row0), int(mb_row1), int(search_range),
                                                      float(tol_16), float(tol_8), d_out, stream))

    def fast_full_search_block(self, list_idx, ref_idx, pos_x, pos_y, blocktype, pred, search_center,
                               surface_range, block_range, rdopt, lambda_factor, min_mcost=_lib.DISTBLK_MAX):
        """fast_full_search_motion_estimation's contract for one partition (JM me_fullfast.c:618-689)."""
        p = JmmeMv(int(pred[0]), int(pred[1]))
        c = JmmeMv(int(search_center[0]), int(search_center[1]))
        mv = JmmeMv(0, 0)
        cost = lib().jmme_fast_full_search_block(self._ctx, int(list_idx), int(ref_idx), int(pos_x), int(pos_y),
                                                 int(blocktype), ctypes.byref(p), ctypes.byref(c),
                                                 int(surface_range), int(block_range), int(rdopt),
                                                 ctypes.byref(mv), int(min_mcost), int(lambda_factor))
        return (mv.mv_x, mv.mv_y), int(cost)
