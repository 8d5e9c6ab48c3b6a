"""trans_show dump format (jmme/fractal_dump.py, tran_show ZL/src/image.c:996-1106)
pinned by the thesis's own artefacts: tests/golden/trans_show/trans_show_{Y,UV}.txt
are the files in the reference's Debug/ directory (a 640x480 run; its input
YUV is not in the reference, so the trees cannot be recomputed).  Each file is
parsed into jmme_fractal_mb records and re-rendered: the bytes must be
identical.  Then a dump of encoder-made trees parses back to the same trees."""
import os
import re

import numpy as np

from fractal_scenes import gate_scene

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "trans_show")
REC = re.compile(r"\n(luma|2、chroma|3、chroma),mode=([0-9.]+)\n(-?\d+) +(-?\d+) +(-?\d+) +(-?\d+) +(-?[0-9.]+) +(-?[0-9.]+)")


def _node(m):
    return dict(bt=int(m.group(3)), x=int(m.group(4)), y=int(m.group(5)), reference=int(m.group(6)),
                offset=float(m.group(7)) * 5, scale=float(m.group(8)) / 20)


def _set(n, d, partition=0):
    n["x"], n["y"], n["reference"], n["offset"], n["scale"], n["partition"] = (d["x"], d["y"], d["reference"],
                                                                            d["offset"], d["scale"], partition)


def _parse_luma(body):
    """records of one macroblock -> FRACTAL_MB (mode 0, or the 3.k 8x8 level)"""
    from jmme import FRACTAL_MB
    t = np.zeros((), FRACTAL_MB)
    recs = [(m.group(2), _node(m)) for m in REC.finditer(body)]
    if recs[0][0] == "0":
        _set(t["mb"], recs[0][1])
        return t, {0}
    t["mb"]["partition"] = 3
    q = 0
    i = 0
    bts = set()
    while i < len(recs):
        k = int(recs[i][0].split(".")[1])
        n = {0: 1, 1: 2, 2: 2, 3: 4}[k]
        t["b8"][q]["partition"] = k
        bts.add(recs[i][1]["bt"])
        if k == 0:
            _set(t["b8"][q], recs[i][1])
        else:
            for j in range(n):
                _set(t["sub"][q][j], recs[i + j][1])
        i += n
        q += 1
    assert q == 4
    return t, bts


def _split_mbs(text):
    head, *mbs = re.split(r"\nCurrentMb=\s*(\d+)", text)
    return head, [(int(mbs[i]), mbs[i + 1]) for i in range(0, len(mbs), 2)]


def test_trans_show_y_round_trip():
    from jmme.fractal_dump import ENCODING, trans_show_y
    raw = open(os.path.join(HERE, "trans_show_Y.txt"), "rb").read()
    text = raw.decode(ENCODING)
    head, mbs = _split_mbs(text)
    frame = int(re.search(r"current_frame =\s*(\d+)", head).group(1))
    trees = []
    sub_bts = set()
    for k, (m, body) in enumerate(mbs):
        assert m == k
        t, bts = _parse_luma(body)
        if t["mb"]["partition"] == 3:
            sub_bts |= bts
        trees.append(t)
    assert sub_bts == {205}                      # the MSVC debug-heap fill, see fractal_dump
    trees = np.array(trees)
    assert (trees["mb"]["partition"] == 3).sum() == 2 and len(trees) == 1200
    assert trans_show_y(trees, frame).encode(ENCODING) == raw


def test_trans_show_uv_round_trip():
    from jmme import FRACTAL_MB
    from jmme.fractal_dump import ENCODING, trans_show_uv
    raw = open(os.path.join(HERE, "trans_show_UV.txt"), "rb").read()
    text = raw.decode(ENCODING)
    head, mbs = _split_mbs(text)
    frame = int(re.search(r"current_frame =\s*(\d+)", head).group(1))
    u = np.zeros(len(mbs), FRACTAL_MB)
    v = np.zeros(len(mbs), FRACTAL_MB)
    for k, (m, body) in enumerate(mbs):
        recs = list(REC.finditer(body))
        assert m == k and len(recs) == 2 and recs[0].group(2) == "0" and recs[1].group(2) == "0"
        _set(u[k]["mb"], _node(recs[0]))
        _set(v[k]["mb"], _node(recs[1]))
    assert trans_show_uv(u, v, frame).encode(ENCODING) == raw


def test_dump_of_encoder_trees_parses_back():
    import oracle_lib as ol
    from jmme import FRACTAL_MB
    from jmme.fractal_dump import trans_show_y
    org, refs = gate_scene(176, 144, 2, 4, scale=6)
    t = ol.fractal_encode_mbs(org, refs, 7, 4.0, 5.0).view(FRACTAL_MB)
    assert (t["mb"]["partition"] == 3).any()
    # the dump keeps 2 decimals of offset/5 and 3 of scale*20: exact for the thesis's quantised values
    text = trans_show_y(t, 3)
    _, mbs = _split_mbs(text)
    for k, (m, body) in enumerate(mbs):
        got, _ = _parse_luma(body)
        e = t[k]
        assert got["mb"]["partition"] == e["mb"]["partition"]
        if e["mb"]["partition"] == 0:
            nodes = [(got["mb"], e["mb"])]
        else:
            nodes = []
            for q in range(4):
                assert got["b8"][q]["partition"] == e["b8"][q]["partition"]
                p = int(e["b8"][q]["partition"])
                nodes += [(got["b8"][q], e["b8"][q])] if p == 0 else \
                    [(got["sub"][q][j], e["sub"][q][j]) for j in range({1: 2, 2: 2, 3: 4}[p])]
        for g, x in nodes:
            assert (g["x"], g["y"], g["reference"]) == (x["x"], x["y"], x["reference"])
            assert abs(g["offset"] - x["offset"]) < 1e-9 and abs(g["scale"] - x["scale"]) < 1e-9
