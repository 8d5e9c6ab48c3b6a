"""The joint fractal + H.264 codec's per-frame GPU work (BASELINE configs[4],
the ZhangLing_Yu path), device-resident on one MI355X.

Per P-frame the thesis codec (ZL/src/code.c:215-305) runs
  start_oneframe + compute_domain_Sum  (ZL/src/image.c:145, compute.c:277)
  encode_Oneframe: encode_one_macroblock for every MB of Y, then U, V
                   (image.c:1108-1127, block_enc.c:508)
  decode_Oneframe: decode_one_macroblock (image.c:639, block_dec.c:20)
and the comparison codec's share of a frame is JM 18.5's integer-pel ME
(full search, mv_search.c:858 -> me_fullsearch.c:39).

`FractalPlane` owns one component's device buffers: the range plane, the
reference views (view 0 = the own reference, views 1..3 = H, M, N), their
"words" domain images, the trees and the reconstruction.  `HybridFrameCoder`
strings the three planes and an ME batch into one stream of launches with no
host round trip.  The oracle is not used here; tests and bench.py check the
results against it.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from ._lib import BLOCK_RES, FRACTAL_MB, FULL_SEARCH, MB_REQ, NSLOT
from .engine import MotionEstimator


class FractalPlane:
    """One component plane (1 Y, 2 U, 3 V) of the fractal P-frame coder."""

    def __init__(self, me: MotionEstimator, component: int, width: int, height: int, n_views: int,
                 device: torch.device, mb_rows: tuple[int, int] | None = None):
        if width % 16 or height % 16:
            raise ValueError(f"fractal plane {width}x{height}: need multiples of 16")
        self.me, self.component, self.W, self.H, self.device = me, component, width, height, device
        self.rows = mb_rows or (0, height // 16)
        self.n_mb = (width // 16) * (self.rows[1] - self.rows[0])
        self.org = torch.zeros((height, width), dtype=torch.uint8, device=device)
        self.views = [torch.zeros((height, width), dtype=torch.uint8, device=device) for _ in range(n_views)]
        self.words = [torch.empty(width * height, dtype=torch.int32, device=device) for _ in range(n_views)]
        self.trees = torch.zeros(self.n_mb * FRACTAL_MB.itemsize, dtype=torch.uint8, device=device)
        self.rec = torch.zeros((height, width), dtype=torch.uint8, device=device)

    def load(self, org: np.ndarray, views: Sequence[np.ndarray]) -> None:
        if len(views) != len(self.views):
            raise ValueError(f"{len(views)} views for a plane built with {len(self.views)}")
        self.org.copy_(torch.from_numpy(np.ascontiguousarray(org, np.uint8)))
        for d, v in zip(self.views, views):
            d.copy_(torch.from_numpy(np.ascontiguousarray(v, np.uint8)))

    def encode(self, search_range: int, tol_16: float, tol_8: float, stream: int = 0) -> None:
        """compute_domain_Sum's role (the views' words images) + the quadtree of the MB rows."""
        for v, w in zip(self.views, self.words):
            self.me.fractal_words_async(v.data_ptr(), self.W, self.W, self.H, w.data_ptr(), stream)
        self.me.fractal_encode_mb_rows_async(self.org.data_ptr(), self.views[0].data_ptr(), self.W,
                                             [w.data_ptr() for w in self.words], self.W, self.H, self.rows[0],
                                             self.rows[1], search_range, tol_16, tol_8, self.trees.data_ptr(), stream)

    def decode(self, stream: int = 0) -> None:
        """decode_one_macroblock of the whole plane (needs the whole plane's trees)."""
        if self.rows != (0, self.H // 16):
            raise ValueError("decode needs the whole plane's trees (gather the bands first)")
        self.me.fractal_decode_mbs_async(self.trees.data_ptr(), [v.data_ptr() for v in self.views], self.W, self.W,
                                         self.H, self.component, self.rec.data_ptr(), 0, stream)

    def trees_host(self) -> np.ndarray:
        return self.trees.cpu().numpy().view(FRACTAL_MB)


class HybridFrameCoder:
    """One P-frame of the joint codec: Y (W x H) and U, V (W/2 x H/2) fractal
    quadtrees over `n_views` reference views at the thesis's search range,
    their reconstruction, and JM's full-search ME of the frame's MB x ref units."""

    def __init__(self, width: int, height: int, n_views: int = 4, fractal_range: int = 7, tol_16: float = 8.0,
                 tol_8: float = 5.0, me_range: int = 32, device: int = 0):
        self.device = torch.device("cuda", device)
        self.me = MotionEstimator({"SearchRange": me_range, "SearchMode": -1, "RDOptimization": 0}, device=device)
        self.fractal_range, self.tol_16, self.tol_8 = fractal_range, tol_16, tol_8
        self.planes = [FractalPlane(self.me, 1, width, height, n_views, self.device),
                       FractalPlane(self.me, 2, width // 2, height // 2, n_views, self.device),
                       FractalPlane(self.me, 3, width // 2, height // 2, n_views, self.device)]
        self.n_units = 0
        self.d_req = self.d_out = None

    def close(self) -> None:
        self.me.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load_fractal(self, planes: Sequence[tuple[np.ndarray, Sequence[np.ndarray]]]) -> None:
        """[(org, views)] for Y, U, V."""
        for p, (org, views) in zip(self.planes, planes):
            p.load(org, views)

    def load_me(self, cur: np.ndarray, ref: np.ndarray, req: np.ndarray) -> None:
        """The frame's luma, its reconstructed reference and JM's MB x ref requests."""
        self.me.upload_cur(cur)
        self.me.upload_ref(0, 0, ref)
        req = np.ascontiguousarray(req, MB_REQ)
        self.n_units = len(req)
        self.d_req = torch.from_numpy(req.view(np.uint8).copy()).to(self.device)
        self.d_out = torch.zeros(self.n_units * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=self.device)

    def fractal_encode(self, stream: int = 0) -> None:
        for p in self.planes:
            p.encode(self.fractal_range, self.tol_16, self.tol_8, stream)

    def fractal_decode(self, stream: int = 0) -> None:
        for p in self.planes:
            p.decode(stream)

    def motion_search(self, stream: int = 0) -> None:
        if self.n_units:
            self.me.search_async(FULL_SEARCH, self.d_req.data_ptr(), self.n_units, self.d_out.data_ptr(), stream)

    def step(self, stream: int = 0) -> None:
        """The whole frame, enqueued on `stream`."""
        self.fractal_encode(stream)
        self.fractal_decode(stream)
        self.motion_search(stream)

    def me_results(self) -> np.ndarray:
        return self.d_out.cpu().numpy().view(BLOCK_RES).reshape(self.n_units, NSLOT)
