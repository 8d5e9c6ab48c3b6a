"""Sub-pel fixtures (tests/golden/subpel_*.npz, made by make_golden_subpel.py):
JM 18.5's quarter-pel sub-images and every sub-pel refinement of a captured
encode, grouped per (frame, list, ref) for the oracle and the HIP path."""
from __future__ import annotations

import os

import numpy as np

from golden_io import GOLDEN, Case, manifest

SPEC_FIELDS = ["pos_x", "pos_y", "bsx", "bsy", "blocktype", "ref", "pred_x", "pred_y", "lambda_h", "lambda_q",
               "rdopt", "slice_type", "start_hp", "start_qp", "metric_h", "metric_q", "test8x8", "search_pos2",
               "search_pos4", "subthres"]


def cases() -> list[str]:
    return sorted(k for k, v in manifest().items() if v.get("kind") == "subpel")


def subimg_cases() -> list[str]:
    return sorted(k for k, v in manifest().items() if v.get("kind") == "subpel" and v.get("n_subimg", 0))


class SubpelCase(Case):
    def __init__(self, name: str):
        super().__init__(name)
        z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
        self.sub_src = z["sub_src"] if "sub_src" in z.files else None
        self.sub_img = z["sub_img"] if "sub_img" in z.files else None

    def oracle_req(self, idx):
        """SPO_REQ rows (oracle_lib) for the refinements idx"""
        import oracle_lib as ol
        r = self.r
        q = np.zeros(len(idx), ol.SPO_REQ)
        for f in SPEC_FIELDS:
            q[f] = r[f][idx]
        q["mv_x"], q["mv_y"] = r["mv_in_x"][idx], r["mv_in_y"][idx]
        q["min_mcost"] = r["min_mcost_in"][idx]
        return q

    def expected(self, idx):
        r = self.r
        return np.stack([r["out_mv_x"][idx], r["out_mv_y"][idx]], 1), r["out_cost"][idx]
