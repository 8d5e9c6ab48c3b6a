"""JM EPZS capture records (oracle/capture/jm_epzs_capture.c) -> EPZS
search requests (jmme_epzs_req layout) grouped by picture, for the oracle
and the GPU parity tests.  Test infrastructure only."""
import numpy as np

import oracle_lib as ol


def requests_from_capture(recs, preds, stale):
    """-> (req EPZS_REQ[n], pred pool int16 [k,2], stale pool int16 [m,2]);
    req['plane'] is left 0 (the caller maps (frame, list, ref) to planes)"""
    n = len(recs)
    req = np.zeros(n, ol.EPZS_REQ)
    for f in ("pos_x", "pos_y", "bsx", "bsy", "blocktype", "pred_x", "pred_y", "center_x", "center_y", "lambda",
              "variant", "medthres"):
        req[f] = recs[f]
    req["ref_idx"] = recs["ref"]
    req["max_x"] = recs["sr_max_x"]
    req["max_y"] = recs["sr_max_y"]
    req["flags"] = (recs["structure"] == 0).astype(np.uint8) | ((recs["slice_type"] == 0).astype(np.uint8) << 1)
    req["pattern"] = recs["epzs_pattern"]
    req["dual"] = recs["epzs_dual"]
    req["prev_sad"] = recs["prev_sad_in"]
    req["stop_crit"] = recs["stop_crit"]
    req["n_pred"] = np.maximum(recs["n_pred"], 0)
    req["n_stale"] = recs["n_stale"]
    cnt = np.array([len(p) for p in preds], np.int64)
    req["pred_off"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if n else []
    scnt = np.array([len(s) for s in stale], np.int64)
    req["stale_off"] = np.concatenate([[0], np.cumsum(scnt)[:-1]]) if n else []
    pool = np.concatenate(preds).astype(np.int16) if cnt.sum() else np.zeros((0, 2), np.int16)
    spool = np.concatenate(stale).astype(np.int16) if scnt.sum() else np.zeros((0, 2), np.int16)
    return req, pool, spool


def cases():
    from golden_io import manifest
    return sorted(k for k, v in manifest().items() if v.get("kind") == "epzs")


class EpzsCase:
    """A committed EPZS fixture (tests/golden/make_golden_epzs.py)."""

    def __init__(self, name):
        import hashlib
        import os

        from golden_io import GOLDEN, manifest
        from jmme import synth
        self.name = name
        self.meta = m = manifest()[name]
        z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
        self.r = {k[2:]: z[k] for k in z.files if k.startswith("r_")}
        self.n = len(self.r["variant"])
        cur_fn, ref_key = z["cur_frame_no"], z["ref_key"]
        if "cur" in z.files:
            cur, ref = z["cur"], z["ref"]
        else:
            luma = synth.luma_sequence(m["w"], m["h"], m["frames"], seed=m["seed"], gmv=tuple(m["gmv"]))
            hc, wc = (m["h"] + 15) // 16 * 16, (m["w"] + 15) // 16 * 16
            orig = np.pad(luma, ((0, 0), (0, hc - m["h"]), (0, wc - m["w"])), mode="edge")
            cur = orig[cur_fn]
            ref = (orig[ref_key[:, 0] - 1 - ref_key[:, 2]].astype(np.int16)
                   + z["ref_residual"].astype(np.int16)).astype(np.uint8)
        for c, h in zip(cur, z["cur_md5"]):
            if hashlib.md5(c.tobytes()).hexdigest() != str(h):
                raise AssertionError(f"{name}: regenerated current frame does not match the fixture md5")
        self.cur = {int(f): cur[i] for i, f in enumerate(cur_fn)}
        self.ref = {(int(k[0]), int(k[1]), int(k[2])): ref[i] for i, k in enumerate(ref_key)}
        rec = np.zeros(self.n, [("n_pred", "<i4"), ("n_stale", "<i4")])
        rec["n_pred"] = np.maximum(self.r["n_pred"], 0)
        rec["n_stale"] = self.r["n_stale"]
        self.preds, self.stale = z["preds"], z["stale"]
        self.pred_off = np.concatenate([[0], np.cumsum(rec["n_pred"])[:-1]]).astype(np.int64)
        self.stale_off = np.concatenate([[0], np.cumsum(rec["n_stale"])[:-1]]).astype(np.int64)

    def requests(self, idx):
        r = self.r
        req = np.zeros(len(idx), ol.EPZS_REQ)
        for f in ("pos_x", "pos_y", "bsx", "bsy", "blocktype", "pred_x", "pred_y", "center_x", "center_y",
                  "lambda", "variant", "medthres"):
            req[f] = r[f][idx]
        req["ref_idx"] = r["ref"][idx]
        req["max_x"] = r["sr_max_x"][idx]
        req["max_y"] = r["sr_max_y"][idx]
        req["flags"] = ((r["structure"][idx] == 0).astype(np.uint8) |
                        ((r["slice_type"][idx] == 0).astype(np.uint8) << 1))
        req["pattern"] = r["epzs_pattern"][idx]
        req["dual"] = r["epzs_dual"][idx]
        req["prev_sad"] = r["prev_sad_in"][idx]
        req["stop_crit"] = r["stop_crit"][idx]
        req["n_pred"] = np.maximum(r["n_pred"][idx], 0)
        req["n_stale"] = r["n_stale"][idx]
        req["pred_off"] = self.pred_off[idx]
        req["stale_off"] = self.stale_off[idx]
        return req

    def frames(self):
        """yield (frame_no, cur plane, [ref planes], req with 'plane' set, expected EPZS_RES fields)"""
        r = self.r
        for f in sorted(set(int(v) for v in r["frame_no"])):
            idx = np.nonzero(r["frame_no"] == f)[0]
            keys = sorted(k for k in self.ref if k[0] == f)
            req = self.requests(idx)
            req["plane"] = [keys.index((f, int(l), int(rf))) for l, rf in zip(r["list"][idx], r["ref"][idx])]
            exp = np.zeros(len(idx), ol.EPZS_RES)
            exp["mv_x"], exp["mv_y"] = r["out_mv_x"][idx], r["out_mv_y"][idx]
            exp["cost"], exp["prev_sad"] = r["out_cost"][idx], r["prev_sad_out"][idx]
            yield f, self.cur[f], [self.ref[k] for k in keys], req, exp
