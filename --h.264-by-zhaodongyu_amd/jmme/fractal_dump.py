"""The thesis codec's per-frame dump of its fractal trees, trans_show_Y.txt and
trans_show_UV.txt (tran_show, ZL/src/image.c:996-1106, written by
encode_Oneframe, image.c:1134-1190), from jmme_fractal_mb records
(jmme_fractal_encode_mbs / FRACTAL_MB).

Per macroblock "\\nCurrentMb=%3d", then one "\\n<label>,mode=<m>\\n%d %2d %2d  %d
%3.2f  %3.3f" record per printed node (block_type, x, y, reference, offset/5,
scale*20): the 16x16 node, or the 8x8 level with its pairs / 4x4 blocks under
"mode=3.<partition>".  Chroma prints only the macroblock and 8x8 levels, labels
"2、chroma" (U) and "3、chroma" (V); the files are GBK text.

block_type: the encoder stores 0 in the macroblock node (block_enc.c:570);
the 8x8 nodes are malloc'd and their block_type never assigned, and the
thesis's own Debug/trans_show_Y.txt shows what that byte held in its MSVC debug
build -- the debug heap's 0xCD fill, printed as 205.  `sub_block_type`
(default 205) reproduces that file; pass 0 for a clean dump.
"""
from __future__ import annotations

import numpy as np

SUB_BLOCK_TYPE = 0xCD
ENCODING = "gbk"
Y_HEADER = "\n////////////////++++++++++++++current_frame = %2d+++++++++++++++/////////////////\n"    # image.c:1141
UV_HEADER = "\n//////////////+++++++++++++++current_frame = %2d+++++++++++++++/////////////////\n"    # image.c:1150


def _rec(label: str, mode: str, block_type: int, n) -> str:
    return "\n%s,mode=%s\n%d %2d %2d  %d  %3.2f  %3.3f" % (label, mode, block_type, int(n["x"]), int(n["y"]),
                                                          int(n["reference"]), float(n["offset"]) / 5,
                                                          float(n["scale"]) * 20)


def _luma_mb(t, sub_bt: int) -> str:
    """tran_show mode 1 (image.c:999-1043)"""
    mb = t["mb"]
    p = int(mb["partition"])
    if p == 0:
        return _rec("luma", "%d" % p, 0, mb)
    out = []
    if p in (1, 2):                    # 16x8 / 8x16 (never left by the encoder, printed as the thesis would)
        for i in range(2):
            out.append(_rec("luma", "%d" % int(t["b8"][i]["partition"]), sub_bt, t["b8"][i]))
        return "".join(out)
    for i in range(4):
        b = t["b8"][i]
        bp = int(b["partition"])
        if bp == 0:
            out.append(_rec("luma", "3.%d" % bp, sub_bt, b))
        elif bp in (1, 2):
            for j in range(2):
                out.append(_rec("luma", "3.%d" % bp, sub_bt, t["sub"][i][j]))
        else:
            for k in range(4):
                out.append(_rec("luma", "3.%d" % bp, sub_bt, t["sub"][i][k]))
    return "".join(out)


def _chroma_mb(t, label: str, sub_bt: int, v_plane: bool) -> str:
    """tran_show modes 2 and 3 (image.c:1044-1106): the 8x8 level only"""
    mb = t["mb"]
    p = int(mb["partition"])
    if p == 0:
        return _rec(label, "%d" % p, 0, mb)
    n = 2 if p in (1, 2) else 4
    # the V rect branch reads next[i].block_type, every other branch the macroblock's
    bt = sub_bt if (v_plane and p in (1, 2)) else 0
    return "".join(_rec(label, "%d" % p, bt, t["b8"][i]) for i in range(n))


def trans_show_y(mbs: np.ndarray, frame_no: int, sub_block_type: int = SUB_BLOCK_TYPE) -> str:
    """One frame's section of trans_show_Y.txt (image.c:1139-1146)."""
    parts = [Y_HEADER % frame_no]
    for m, t in enumerate(mbs):
        parts.append("\nCurrentMb=%3d" % m)
        parts.append(_luma_mb(t, sub_block_type))
    return "".join(parts)


def trans_show_uv(mbs_u: np.ndarray, mbs_v: np.ndarray, frame_no: int,
                  sub_block_type: int = SUB_BLOCK_TYPE) -> str:
    """One frame's section of trans_show_UV.txt (image.c:1148-1157)."""
    assert len(mbs_u) == len(mbs_v)
    parts = [UV_HEADER % frame_no]
    for m in range(len(mbs_u)):
        parts.append("\nCurrentMb=%3d" % m)
        parts.append(_chroma_mb(mbs_u[m], "2、chroma", sub_block_type, False))
        parts.append(_chroma_mb(mbs_v[m], "3、chroma", sub_block_type, True))
    return "".join(parts)


def write_trans_show(path_y: str, path_uv: str, frames, sub_block_type: int = SUB_BLOCK_TYPE) -> None:
    """frames: iterable of (frame_no, mbs_y, mbs_u, mbs_v); the thesis opens the
    files with "w" for the first fractal frame and appends the rest."""
    with open(path_y, "w", encoding=ENCODING, newline="") as fy, \
            open(path_uv, "w", encoding=ENCODING, newline="") as fuv:
        for frame_no, y, u, v in frames:
            fy.write(trans_show_y(y, frame_no, sub_block_type))
            fuv.write(trans_show_uv(u, v, frame_no, sub_block_type))
