"""Reader for the binary log written by oracle/capture/jm_me_capture.c.

Test infrastructure only: used by tests/golden/make_golden.py to turn a real
JM 18.5 run into committed fixtures.  The record layout mirrors
`struct cap_search` in jm_me_capture.c (packed, little endian).
"""
from __future__ import annotations

import numpy as np

SEARCH_DTYPE = np.dtype([
    ("mode", "<i4"), ("frame_no", "<i4"), ("mb_addr", "<i4"),
    ("pix_x", "<i2"), ("pix_y", "<i2"),
    ("blocktype", "<i2"), ("block_x", "<i2"), ("block_y", "<i2"),
    ("pos_x", "<i2"), ("pos_y", "<i2"), ("bsx", "<i2"), ("bsy", "<i2"),
    ("list", "<i2"), ("ref", "<i2"),
    ("pred_x", "<i2"), ("pred_y", "<i2"), ("center_x", "<i2"), ("center_y", "<i2"),
    ("sr_min_x", "<i4"), ("sr_max_x", "<i4"), ("sr_min_y", "<i4"), ("sr_max_y", "<i4"),
    ("lambda", "<i4"), ("rdopt", "<i4"), ("slice_type", "<i4"),
    ("min_mcost_in", "<i8"),
    ("ffs_center_x", "<i2"), ("ffs_center_y", "<i2"),
    ("ffs_max_range", "<i4"), ("ffs_pos00", "<i4"), ("max_mvd", "<i4"),
    ("img_w", "<i4"), ("img_h", "<i4"),
    ("out_mv_x", "<i2"), ("out_mv_y", "<i2"), ("out_cost", "<i8"),
])
TAG_PLANE = 0x304E4C50
TAG_SEARCH = 0x30435253


def read_capture(path: str):
    """Return (planes, records).

    planes: dict {(frame_no, kind, list, ref): uint16 [H, W]} (kind 0 = current
    original, 1 = reference reconstruction as JM's imgY);
    records: structured array of SEARCH_DTYPE in call order.
    """
    buf = open(path, "rb").read()
    mv = memoryview(buf)
    off = 0
    planes = {}
    recs = []
    n = len(buf)
    rsz = SEARCH_DTYPE.itemsize
    while off < n:
        tag = int.from_bytes(mv[off:off + 4], "little")
        off += 4
        if tag == TAG_PLANE:
            hdr = np.frombuffer(mv[off:off + 24], dtype="<i4")
            off += 24
            frame_no, kind, lst, ref, w, h = (int(v) for v in hdr)
            a = np.frombuffer(mv[off:off + 2 * w * h], dtype="<u2").reshape(h, w).copy()
            off += 2 * w * h
            planes[(frame_no, kind, lst, ref)] = a
        elif tag == TAG_SEARCH:
            recs.append(np.frombuffer(mv[off:off + rsz], dtype=SEARCH_DTYPE)[0])
            off += rsz
        else:
            raise ValueError(f"bad tag {tag:#x} at {off - 4}")
    return planes, np.array(recs, dtype=SEARCH_DTYPE)


# ---- EPZS log (oracle/capture/jm_epzs_capture.c, struct cap_epzs) -------------
EPZS_DTYPE = np.dtype([
    ("variant", "<i4"), ("frame_no", "<i4"), ("mb_addr", "<i4"),
    ("mb_x", "<i2"), ("mb_y", "<i2"),
    ("blocktype", "<i2"), ("block_x", "<i2"), ("block_y", "<i2"),
    ("pos_x", "<i2"), ("pos_y", "<i2"), ("bsx", "<i2"), ("bsy", "<i2"),
    ("list", "<i2"), ("ref", "<i2"), ("list_offset", "<i2"),
    ("pred_x", "<i2"), ("pred_y", "<i2"), ("center_x", "<i2"), ("center_y", "<i2"),
    ("sr_min_x", "<i4"), ("sr_max_x", "<i4"), ("sr_min_y", "<i4"), ("sr_max_y", "<i4"),
    ("lambda", "<i4"), ("slice_type", "<i4"), ("structure", "<i4"),
    ("epzs_pattern", "<i4"), ("epzs_dual", "<i4"), ("blk_count", "<i4"),
    ("prev_sad_in", "<i8"), ("medthres", "<i8"), ("stop_crit", "<i8"),
    ("n_pred", "<i4"), ("n_stale", "<i4"), ("stale_overflow", "<i4"),
    ("img_w", "<i4"), ("img_h", "<i4"),
    ("min_mcost_in", "<i8"),
    ("out_mv_x", "<i2"), ("out_mv_y", "<i2"), ("out_cost", "<i8"), ("prev_sad_out", "<i8"),
])
TAG_EPZS = 0x305A5045


def read_epzs_capture(path: str):
    """Return (planes, records, preds, stale): records EPZS_DTYPE in call order;
    preds / stale int16 [total, 2] pools with per-record offsets in
    records' order (pred_off / stale_off arrays returned inside a dict)."""
    buf = open(path, "rb").read()
    mv = memoryview(buf)
    off, n = 0, len(buf)
    planes, recs, preds, stale = {}, [], [], []
    rsz = EPZS_DTYPE.itemsize
    while off < n:
        tag = int.from_bytes(mv[off:off + 4], "little")
        off += 4
        if tag == TAG_PLANE:
            hdr = np.frombuffer(mv[off:off + 24], dtype="<i4")
            off += 24
            frame_no, kind, lst, ref, w, h = (int(v) for v in hdr)
            planes[(frame_no, kind, lst, ref)] = np.frombuffer(mv[off:off + 2 * w * h], dtype="<u2").reshape(h, w).copy()
            off += 2 * w * h
        elif tag == TAG_EPZS:
            r = np.frombuffer(mv[off:off + rsz], dtype=EPZS_DTYPE)[0]
            off += rsz
            k = max(int(r["n_pred"]), 0)
            preds.append(np.frombuffer(mv[off:off + 4 * k], dtype="<i2").reshape(k, 2).copy())
            off += 4 * k
            s = int(r["n_stale"])
            stale.append(np.frombuffer(mv[off:off + 4 * s], dtype="<i2").reshape(s, 2).copy())
            off += 4 * s
            recs.append(r)
        else:
            raise ValueError(f"bad tag {tag:#x} at {off - 4}")
    return planes, np.array(recs, dtype=EPZS_DTYPE), preds, stale


# ---- sub-pel capture (oracle/capture/jm_subpel_capture.c) -------------------
SUBPEL_DTYPE = np.dtype([
    ("kind", "<i4"), ("frame_no", "<i4"), ("mb_addr", "<i4"),
    ("pix_x", "<i2"), ("pix_y", "<i2"),
    ("blocktype", "<i2"), ("block_x", "<i2"), ("block_y", "<i2"),
    ("pos_x", "<i2"), ("pos_y", "<i2"), ("bsx", "<i2"), ("bsy", "<i2"),
    ("list", "<i2"), ("ref", "<i2"),
    ("pred_x", "<i2"), ("pred_y", "<i2"), ("mv_in_x", "<i2"), ("mv_in_y", "<i2"),
    ("min_mcost_in", "<i8"),
    ("lambda_f", "<i4"), ("lambda_h", "<i4"), ("lambda_q", "<i4"),
    ("rdopt", "<i4"), ("slice_type", "<i4"), ("start_hp", "<i4"), ("start_qp", "<i4"),
    ("metric_h", "<i4"), ("metric_q", "<i4"), ("test8x8", "<i4"),
    ("search_pos2", "<i4"), ("search_pos4", "<i4"), ("chroma_me", "<i4"),
    ("subthres", "<i8"), ("img_w", "<i4"), ("img_h", "<i4"),
    ("out_mv_x", "<i2"), ("out_mv_y", "<i2"), ("out_cost", "<i8"),
])
TAG_SUBPEL = 0x304C5053
TAG_SUBIMG = 0x30425553


def read_subpel_capture(path: str):
    """Return (planes, subimgs, records): planes as read_capture (kind 2 = the
    source of an interpolation, keyed by its sequence number); subimgs {seq:
    uint16 [16, H+40, W+64]}; records SUBPEL_DTYPE in call order."""
    buf = open(path, "rb").read()
    mv = memoryview(buf)
    off, n = 0, len(buf)
    planes, subimgs, recs = {}, {}, []
    rsz = SUBPEL_DTYPE.itemsize
    while off < n:
        tag = int.from_bytes(mv[off:off + 4], "little")
        off += 4
        if tag == TAG_PLANE:
            frame_no, kind, lst, ref, w, h = (int(v) for v in np.frombuffer(mv[off:off + 24], dtype="<i4"))
            off += 24
            planes[(frame_no, kind, lst, ref)] = np.frombuffer(mv[off:off + 2 * w * h], "<u2").reshape(h, w).copy()
            off += 2 * w * h
        elif tag == TAG_SUBIMG:
            seq, w, h = (int(v) for v in np.frombuffer(mv[off:off + 12], dtype="<i4"))
            off += 12
            cnt = 16 * (h + 40) * (w + 64)
            subimgs[seq] = np.frombuffer(mv[off:off + 2 * cnt], "<u2").reshape(16, h + 40, w + 64).copy()
            off += 2 * cnt
        elif tag == TAG_SUBPEL:
            recs.append(np.frombuffer(mv[off:off + rsz], dtype=SUBPEL_DTYPE)[0])
            off += rsz
        else:
            raise ValueError(f"bad tag {tag:#x} at {off - 4}")
    return planes, subimgs, np.array(recs, dtype=SUBPEL_DTYPE)
